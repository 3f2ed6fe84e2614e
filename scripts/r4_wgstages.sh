#!/bin/bash
# Round 4: grouped weight-gradient DMA ring depth on the headline proxy step -- 4 stages
# (default) vs 2 (NNMPI_WG_STAGES=2, experiments), interleaved, then kernel stats of the default.
# Usage: scripts/r4_wgstages.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-r4wg}; mkdir -p $O
for i in 1 2 3; do
  for ns in 4 2; do
    NNMPI_EXPERIMENTS=1 NNMPI_WG_STAGES=$ns timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      > $O/bench_ns${ns}_$i.json 2> $O/bench_ns${ns}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_ns${ns}_$i.json').read().strip().splitlines()[-1]); print('stages=$ns', d['ms_per_step'], d['value'], d['config']['schedule'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o proxy -- \
  python bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -8
