#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/rowband_tests.txt 2>&1 || { tail -30 gpurun_out/r6/rowband_tests.txt; exit 1; }
tail -2 gpurun_out/r6/rowband_tests.txt
BARGS="--rows 1024" TOPK=3 bash scripts/r5_ab.sh r6ks_1024 "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KSPLIT=1" "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KSPLIT=3" || exit 1
BARGS="--rows 2048" TOPK=3 bash scripts/r5_ab.sh r6ks_2048 "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KSPLIT=1" "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KSPLIT=4" || exit 1
BARGS="--rows 1024 --force_comm --comm_mode inline" TOPK=4 bash scripts/r5_ab.sh r6rt_1024 "NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=1" "-" || exit 1
