#!/bin/bash
# row-band step: weight-gradient split-K count A/B (NNMPI_RB_SPLITS, experiments), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r4splits; mkdir -p $O
for i in 1 2 3; do
  for sp in 5 4 6 8; do
    NNMPI_RB_SPLITS=$sp timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_extras > $O/b_${sp}_$i.json 2> $O/b_${sp}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/b_${sp}_$i.json').read().strip().splitlines()[-1]); print('splits=$sp', d['ms_per_step'])"
  done
done
