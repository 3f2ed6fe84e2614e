#!/bin/bash
# wgrad_small tile order (NNMPI_WGS_GM 1 / 2 / 4): row tests under gm 2, then interleaved step A/B at
# 1,024 / 2,048 / 4,096 rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
NNMPI_WGS_GM=2 timeout -k 10 400 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/wgs_gm_tests.txt 2>&1 || { tail -30 gpurun_out/r6/wgs_gm_tests.txt; exit 1; }
tail -2 gpurun_out/r6/wgs_gm_tests.txt
for R in 1024 2048 4096; do
BARGS="--rows $R" TOPK=3 bash scripts/r5_ab.sh r6gm_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_GM=2" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_GM=4" || exit 1
done
BARGS="--rows 1024" TOPK=3 bash scripts/r5_ab.sh r6gm_1024b "NNMPI_EXPERIMENTS=1 NNMPI_WGS_GM=2" "-" || exit 1
