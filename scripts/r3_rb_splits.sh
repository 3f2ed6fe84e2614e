#!/bin/bash
# Row-band step: weight-gradient split-K factor A/B (per-kernel times + proxy bench).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbs
mkdir -p $O
for sp in 4 5 8 10 16; do
  rm -rf $O/p_$sp
  NNMPI_ROWBAND=1 NNMPI_RB_SPLITS=$sp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$sp -o run -- python3 bench.py --steps 30 --warmup 5 > $O/log_$sp.txt 2>&1 || exit $?
  f=$(find $O/p_$sp -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$sp" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'rowband' in r['Name'] or 'multi' in r['Name']:
        print("splits", sys.argv[2], r['Name'][:40], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
for r in 1 2; do
  for sp in 5 8 10; do
    NNMPI_ROWBAND=1 NNMPI_RB_SPLITS=$sp timeout -k 10 300 python bench.py > $O/b.json 2>> $O/bench.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('bench splits $sp', d['ms_per_step'])"
  done
done
