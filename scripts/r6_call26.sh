#!/bin/bash
# full-batch weight gradients from K-major images (wgrad_kimg): tests, then the driver-form step
# A/B against the row-major copy-outs + wgrad_multi (NNMPI_RB_WKIMG=0) and split counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread -k "image_path or oracle" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
TOPK=4 bash scripts/r5_ab.sh r6wk "-" "NNMPI_EXPERIMENTS=1 NNMPI_RB_WKIMG=0" "NNMPI_EXPERIMENTS=1 NNMPI_WGK_SPLITS=4" "NNMPI_EXPERIMENTS=1 NNMPI_WGK_SPLITS=8" "-" || exit 1
