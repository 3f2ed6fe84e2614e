#!/bin/bash
# wgrad_small image path: tile patch order (NNMPI_WGS_GM 2 default / 1 row / 4) -- stamps, tests, step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gm_tests.txt 2>&1 || { tail -40 $O/gm_tests.txt; exit 1; }
tail -1 $O/gm_tests.txt
for rows in 1024 2048; do
  for gm in 2 1 4; do
    NNMPI_BUILD_EXPERIMENTS=1 NNMPI_EXPERIMENTS=1 NNMPI_WGS_GM=$gm timeout -k 10 300 python -u scripts/r5_wgs_stamps.py $rows 40 > $O/wgsgm_${rows}_$gm.txt 2>&1 || { tail -20 $O/wgsgm_${rows}_$gm.txt; exit 1; }
    echo "== rows $rows, NNMPI_WGS_GM=$gm"; grep -v amdgpu.ids $O/wgsgm_${rows}_$gm.txt
  done
done
for R in 1024 2048; do
BARGS="--rows $R" TOPK=2 bash scripts/r5_ab.sh r6gm2_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_GM=1" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
done
