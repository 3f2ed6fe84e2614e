#!/bin/bash
# split kernel with the operand-image writes: placement A/B (after / before the arrival) vs no images
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
for rows in 1024 2048; do
  for v in "NNMPI_KFRAG_EARLY=0" "NNMPI_KFRAG_EARLY=1" "NNMPI_WGS_KIMG=0"; do
    env $v NNMPI_BUILD_EXPERIMENTS=1 NNMPI_EXPERIMENTS=1 timeout -k 10 300 python -u scripts/r5_split_stamps.py $rows 40 > $O/st_${rows}_$v.txt 2>&1 || { tail -20 $O/st_${rows}_$v.txt; exit 1; }
    echo "== rows $rows, $v"; grep -v amdgpu.ids $O/st_${rows}_$v.txt
  done
done
for R in 1024 2048; do
BARGS="--rows $R" TOPK=2 bash scripts/r5_ab.sh r6ke_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_KFRAG_EARLY=1" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "NNMPI_EXPERIMENTS=1 NNMPI_KFRAG_EARLY=1" "-" || exit 1
done
