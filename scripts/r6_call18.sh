#!/bin/bash
# wgrad_small's image path (K-major operand fragments written by the split kernel): GPU tests,
# then interleaved step A/B against the LDS-DMA tiles (NNMPI_WGS_KIMG=0) at 1,024 / 2,048 rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest tests/test_rowband_gpu.py tests/test_split_contention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/kimg_tests.txt 2>&1 || { tail -40 gpurun_out/r6/kimg_tests.txt; exit 1; }
tail -2 gpurun_out/r6/kimg_tests.txt
for R in 1024 2048; do
BARGS="--rows $R" TOPK=3 bash scripts/r5_ab.sh r6ki_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
done
BARGS="--rows 1024 --force_comm --comm_mode inline" TOPK=4 bash scripts/r5_ab.sh r6ki_fc1024 "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" || exit 1
