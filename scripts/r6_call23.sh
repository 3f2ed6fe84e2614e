#!/bin/bash
# image path up to 4,096 rows: rowband tests, then step A/B (image vs slabs + combine) at 3,072 / 4,096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/k4096_tests.txt 2>&1 || { tail -40 $O/k4096_tests.txt; exit 1; }
tail -1 $O/k4096_tests.txt
for R in 4096 3072; do
BARGS="--rows $R" TOPK=3 bash scripts/r5_ab.sh r6k4_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
done
BARGS="--rows 4096 --force_comm --comm_mode inline" TOPK=4 bash scripts/r5_ab.sh r6k4_fc4096 "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" || exit 1
