#!/bin/bash
# Comm/compute CU contention, settled with a kernel trace (VERDICT r4 "Next round" 6): the wide
# model at one rank with --force_comm and the collective stand-in (csrc/experiments/standin.hip,
# experiments library) holding k CUs after each bucket for its bytes at 1.07 TB/s, k = 0, 1, 8, 32,
# each under rocprofv3 --kernel-trace; scripts/r5_standin_table.py then tabulates every GEMM
# kernel's duration by k (and whether a hold ran concurrently with it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1 NNMPI_BUILD_EXPERIMENTS=1
O=gpurun_out/r5/standin; mkdir -p $O
for k in 0 1 8 32; do
  ST="$k:1070"; [ $k = 0 ] && ST=""
  NNMPI_COMM_STANDIN=$ST timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/k$k -o t -- \
    python bench.py --config wide8192 --steps 12 --warmup 3 --force_comm --no_extras --comm_mode overlap \
    > $O/k$k.log 2>&1 || { tail -5 $O/k$k.log; exit 1; }
  echo "k=$k $(grep -o '"ms_per_step": [0-9.]*' $O/k$k.log)"
done
python scripts/r5_standin_table.py $O
