#!/bin/bash
# split-kernel phase stamps (experiments library: the stamped twin), XCD-grouped map vs the round-5 map
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_BUILD_EXPERIMENTS=1 NNMPI_EXPERIMENTS=1
O=gpurun_out/r6s; mkdir -p $O
for rows in 1024 2048; do
  for map in 1 0; do
    NNMPI_RB_SPLIT_MAP=$map timeout -k 10 300 python -u scripts/r5_split_stamps.py $rows 40 > $O/stamps_${rows}_map$map.txt 2>&1 || { tail -20 $O/stamps_${rows}_map$map.txt; exit 1; }
    echo "== rows $rows, NNMPI_RB_SPLIT_MAP=$map"; grep -v amdgpu.ids $O/stamps_${rows}_map$map.txt
  done
done
