#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r3h
timeout -k 10 200 python scripts/head_debug.py > gpurun_out/r3h/debug.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "head" > gpurun_out/r3h/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r3h/summary.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/head_bench.py > gpurun_out/r3h/head.jsonl 2> gpurun_out/r3h/head.err
echo "head rc=$?" >> gpurun_out/r3h/summary.txt
