#!/bin/bash
# Wide backward pairs (wgrad_i + SGD beside dgrad_{i-1} in one launch): bitwise tests, then the
# whole wide step A/B (NNMPI_PAIR=0 = separate launches), interleaved, then a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/pair
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "wide_pair or unsplit_wgrad or wide_chunked" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
for r in 1 2; do
  for p in 1 0; do
    NNMPI_PAIR=$p timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
    echo "pair=$p $(cut -c1-140 $O/b.json)" | tee -a $O/bench_ab.txt
  done
done
rm -rf $O/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config wide8192 --steps 20 --warmup 3 --no_extras > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
cut -d, -f1-4 $O/kernel_stats.csv | head -8
