#!/bin/bash
# optimizer pass with momentum loads not gated by the device hyper-parameters: tests, then the
# one-rank force-comm A/B (no comm / inline / overlap_rowband) at 8,192 and 1,024 rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sgd or optimizer or fused_update or momentum or weight_images" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
bash scripts/r6_forcecomm.sh r6p 8192 1024
