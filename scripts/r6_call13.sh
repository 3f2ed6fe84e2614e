#!/bin/bash
# near-final: the whole GPU suite, smoke(), then every bench config / shard size, kernel stats and
# the 2-rank rehearsal (scripts/r6_final.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6/gpu_suite.txt 2>&1
rc=$?
tail -3 gpurun_out/r6/gpu_suite.txt; grep -E "FAILED|ERROR" gpurun_out/r6/gpu_suite.txt | head
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.txt 2>&1 || { tail -5 gpurun_out/r6/smoke.txt; exit 1; }
tail -1 gpurun_out/r6/smoke.txt
bash scripts/r6_final.sh bench
