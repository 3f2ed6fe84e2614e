#!/bin/bash
# Round 6, first GPU call: split-kernel tests after the XCD-grouped band map, the map / local-store
# A/B at 1,024 / 2,048 / 4,096 rows, then the one-rank force-comm baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread -k "split or fused_update or small_wgrad or optimizer_pass or images" > gpurun_out/r6/split_tests.txt 2>&1 || { tail -30 gpurun_out/r6/split_tests.txt; exit 1; }
tail -3 gpurun_out/r6/split_tests.txt
timeout -k 10 600 python -u -m pytest tests/test_split_contention_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6/contention_tests.txt 2>&1 || { tail -30 gpurun_out/r6/contention_tests.txt; exit 1; }
tail -5 gpurun_out/r6/contention_tests.txt
for rows in 1024 2048 4096; do
  BARGS="--rows $rows" TOPK=3 bash scripts/r5_ab.sh r6map_$rows "NNMPI_EXPERIMENTS=1 NNMPI_RB_SPLIT_MAP=0" "NNMPI_EXPERIMENTS=1 NNMPI_RB_SPLIT_LOCAL=0" "-" || exit 1
done
bash scripts/r6_forcecomm.sh base 8192 1024 || exit 1
