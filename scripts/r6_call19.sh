#!/bin/bash
# wgrad_small image path: per-block stamps (experiments library) image vs LDS-DMA tiles at 1,024 /
# 2,048 rows, then the PMC groups at 1,024 rows (production library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
for rows in 1024 2048; do
  for k in 1 0; do
    NNMPI_BUILD_EXPERIMENTS=1 NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=$k timeout -k 10 300 python -u scripts/r5_wgs_stamps.py $rows 40 > $O/wgs_${rows}_k$k.txt 2>&1 || { tail -20 $O/wgs_${rows}_k$k.txt; exit 1; }
    echo "== rows $rows, NNMPI_WGS_KIMG=$k"; grep -v amdgpu.ids $O/wgs_${rows}_k$k.txt
  done
done
ROWS=1024 bash scripts/r6_pmc.sh && cat gpurun_out/r6pmc/summary_rows1024.txt
