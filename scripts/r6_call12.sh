#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py tests/test_split_contention_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6/rowband_tests2.txt 2>&1 || { tail -30 gpurun_out/r6/rowband_tests2.txt; exit 1; }
tail -2 gpurun_out/r6/rowband_tests2.txt
for rows in 1024 2048 4096; do
  BARGS="--rows $rows" TOPK=3 bash scripts/r5_ab.sh r6head_$rows "-" "-" || exit 1
done
