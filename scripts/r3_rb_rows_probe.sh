#!/bin/bash
# Row-band kernel: per-kernel time vs rows (blocks = rows / 32): does a pass get faster per
# block when fewer CUs stream the weights at once (L2-aggregate bound) or not (per-CU bound)?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbr
mkdir -p $O
for rows in 8192 4096 2048 1024; do
  rm -rf $O/p_$rows
  NNMPI_ROWBAND=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$rows -o run -- python3 bench.py --rows $rows --steps 30 --warmup 5 > $O/log_$rows.txt 2>&1 || exit $?
  f=$(find $O/p_$rows -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$rows" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'rowband' in r['Name'] or 'multi' in r['Name']:
        print("rows", sys.argv[2], r['Name'][:40], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
