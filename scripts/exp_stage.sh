#!/bin/bash
# LDS-staged 256x256 forward epilogue (NNMPI_STAGE_EPI=1) vs fragment stores: bitwise test, then
# the wide step A/B interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/stage
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "staged_forward" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for v in 1 0; do
    NNMPI_STAGE_EPI=$v timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
    echo "wide stage=$v $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
