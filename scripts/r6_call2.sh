#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r6_contend.sh || exit 1
for rows in 1024 2048 4096; do
  BARGS="--rows $rows" TOPK=3 bash scripts/r5_ab.sh r6map_$rows "NNMPI_EXPERIMENTS=1 NNMPI_RB_SPLIT_MAP=0" "NNMPI_EXPERIMENTS=1 NNMPI_RB_SPLIT_LOCAL=0" "-" || exit 1
done
bash scripts/r6_forcecomm.sh base 8192 1024 || exit 1
