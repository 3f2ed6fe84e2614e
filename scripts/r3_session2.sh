#!/bin/bash
# head timings + 1-rank RCCL wide trace, then the driver's torchrun form rehearsed at N = 2, 4, 8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ONLY_TAIL=1 bash scripts/r3_gemm_ab.sh || exit $?
timeout -k 10 600 python -u -m pytest tests/test_bench.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_bench_gpu.log 2>&1
rc=$?; echo "[s2] bench gpu tests rc=$rc" | tee -a gpurun_out/s2.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/r3_rehearsal.sh
