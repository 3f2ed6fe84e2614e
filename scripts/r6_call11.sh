#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests/test_bench.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r6/bench_tests.txt 2>&1; echo "bench tests rc=$?"
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r6/bench_tests.txt | tail -15
BARGS="--config mnist" TOPK=6 bash scripts/r5_ab.sh r6mnist "-" || exit 1
