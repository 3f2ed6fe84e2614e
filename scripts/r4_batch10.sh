#!/bin/bash
# force_comm A/B (overlap_rowband / inline vs no comm), then the whole GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_forcecomm.sh || exit $?
bash scripts/r4_check.sh r4full "tests -m gpu"
