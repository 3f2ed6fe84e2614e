#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
export NNMPI_EXPERIMENTS=1
for v in "-" "NNMPI_RB_SPLIT_MAP=0" "NNMPI_RB_WGSMALL=0" "NNMPI_RB_SPLIT=0"; do
  E=""; [ "$v" != "-" ] && E="$v"
  echo "== $v"
  env $E NNMPI_ROWBAND_MIN_ROWS=6144 timeout -k 5 200 python scripts/r6_determinism.py 1024 20 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== 8192 band kernel"
NNMPI_ROWBAND_MIN_ROWS=1 timeout -k 5 200 python -c "
import sys; sys.argv=['x','8192','20']; exec(open('scripts/r6_determinism.py').read())" 2>&1 | grep -v amdgpu.ids
