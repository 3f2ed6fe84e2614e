#!/bin/bash
# LDS-staged SGD epilogue (form 0) vs per-fragment (1) vs batched fragment rows (2): bitwise
# tests, wide step A/B interleaved, kernel stats of the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/sgdlds
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "sgd_epilogue_forms or wide_pair or unsplit_wgrad or fused_optimizer" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2 3; do
  for v in 0 1 2; do
    NNMPI_SGD_SERIAL=$v timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
    echo "wide form=$v $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
rm -rf $O/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config wide8192 --steps 20 --warmup 3 --no_extras > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
