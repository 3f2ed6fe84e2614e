#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
REPS=3 bash scripts/r6_fc2.sh final 8192 1024 || exit 1
ROWS="1024 2048 8192" bash scripts/r6_pmc.sh || exit 1
