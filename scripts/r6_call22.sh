#!/bin/bash
# image path final form: full GPU suite, then step A/B (image vs LDS-DMA tiles) at 1,024 / 2,048 rows
# and the 1,024-row one-rank force-comm step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -2 $O/gpu_suite.txt
for R in 1024 2048; do
BARGS="--rows $R" TOPK=2 bash scripts/r5_ab.sh r6kf_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
done
BARGS="--rows 1024 --force_comm --comm_mode inline" TOPK=3 bash scripts/r5_ab.sh r6kf_fc1024 "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
