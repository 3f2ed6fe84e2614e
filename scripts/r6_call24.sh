#!/bin/bash
# own fragments written inside the gather (stores younger than the loads): tests, step A/B at
# 1,024 / 2,048 / 4,096 rows against no images (NNMPI_WGS_KIMG=0), split-kernel stamps at 4,096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_rowband_gpu.py tests/test_split_contention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kg_tests.txt 2>&1 || { tail -40 $O/kg_tests.txt; exit 1; }
tail -1 $O/kg_tests.txt
for R in 1024 2048 4096; do
BARGS="--rows $R" TOPK=3 bash scripts/r5_ab.sh r6kg_$R "-" "NNMPI_EXPERIMENTS=1 NNMPI_WGS_KIMG=0" "-" || exit 1
done
for v in "NNMPI_WGS_KIMG=1" "NNMPI_WGS_KIMG=0"; do
  env $v NNMPI_BUILD_EXPERIMENTS=1 NNMPI_EXPERIMENTS=1 timeout -k 10 300 python -u scripts/r5_split_stamps.py 4096 40 > $O/stg_4096_$v.txt 2>&1 || { tail -20 $O/stg_4096_$v.txt; exit 1; }
  echo "== rows 4096, $v"; grep -v amdgpu.ids $O/stg_4096_$v.txt
done
