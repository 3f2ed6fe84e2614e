#!/bin/bash
# Strip-form optimizer pass (optim.hip sgd_strips_kernel) vs the tiles: bitwise test, then
# interleaved one-rank force-comm A/B at 1,024 and 8,192 rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread -k "optimizer_pass" > gpurun_out/r6/strips_test.txt 2>&1 || { tail -30 gpurun_out/r6/strips_test.txt; exit 1; }
tail -2 gpurun_out/r6/strips_test.txt
BARGS="--rows 1024 --force_comm --comm_mode inline" TOPK=4 bash scripts/r5_ab.sh r6st_1024 "-" "NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=4" "NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=8" || exit 1
BARGS="--rows 8192 --force_comm --comm_mode inline" TOPK=4 bash scripts/r5_ab.sh r6st_8192 "-" "NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=4" "NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=8" || exit 1
