#!/bin/bash
# End-of-round check on one GPU: smoke(), the whole GPU suite, the driver-form bench x3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4end; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo "smoke ok"; tail -2 $O/smoke.log
bash scripts/r4_check.sh r4end "tests -m gpu"
