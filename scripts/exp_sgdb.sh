#!/bin/bash
# Wide step A/B, interleaved in one box session: batched vs per-fragment SGD epilogue
# (NNMPI_SGD_SERIAL) and paired vs separate backward launches (NNMPI_PAIR).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/sgdb
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
  -k "wide_pair or unsplit_wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for cfg in "0 0" "0 1" "1 0"; do
    set -- $cfg
    NNMPI_PAIR=$1 NNMPI_SGD_SERIAL=$2 timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
    echo "pair=$1 serial=$2 $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
