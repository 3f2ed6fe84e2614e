#!/bin/bash
# Round 4: row-band epilogue store order (odd rows store the tile-pair partner first) (NNMPI_RB_EPISWAP, experiments) --
# proxy bench 0 / 1 interleaved (the replica hash must match: results are bitwise independent of
# the store order), then per-kernel stats of each.  Usage: scripts/r4_episwap.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-r4es}; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2 3; do
  for m in 0 1; do
    NNMPI_EXPERIMENTS=1 NNMPI_RB_EPISWAP=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      > $O/bench_m${m}_$i.json 2> $O/bench_m${m}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_m${m}_$i.json').read().strip().splitlines()[-1]); print('swap=$m', d['ms_per_step'], d['replica_hash'], d['knobs']['env'])"
  done
done
for m in 0 1; do
  NNMPI_EXPERIMENTS=1 NNMPI_RB_EPISWAP=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $O/prof_m$m -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof_m$m.log 2>&1 || exit $?
  f=$(find $O/prof_m$m -name "*kernel_stats.csv" | head -1)
  echo "swap=$m"; cut -d, -f1-4 "$f" | head -6
done
