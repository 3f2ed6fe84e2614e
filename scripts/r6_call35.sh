#!/bin/bash
# (experiment) full-batch image path with wgrad_multi's placement: numerics check, then step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 200 python -u scripts/r6_wkimg_check.py > $O/check.txt 2>&1 || { tail -20 $O/check.txt; exit 1; }
grep -v amdgpu.ids $O/check.txt
TOPK=4 bash scripts/r5_ab.sh r6wk2 "-" "NNMPI_EXPERIMENTS=1 NNMPI_RB_WKIMG=1" "-" "NNMPI_EXPERIMENTS=1 NNMPI_RB_WKIMG=1" || exit 1
