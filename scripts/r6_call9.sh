#!/bin/bash
# the whole GPU suite, then the 2-rank shared-GPU rehearsal of the multi-rank bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r6/gpu_suite.txt 2>&1
rc=$?
tail -5 gpurun_out/r6/gpu_suite.txt
grep -E "FAILED|ERROR" gpurun_out/r6/gpu_suite.txt | head -20
[ $rc -ne 0 ] && exit 1
bash scripts/r6_final.sh reh
