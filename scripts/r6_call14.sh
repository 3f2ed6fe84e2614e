#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r6_final.sh prof || exit 1
bash scripts/r6_final.sh reh || exit 1
