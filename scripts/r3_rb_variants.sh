#!/bin/bash
# Row-band kernel variants (rotation of column groups, forward-only diagnostic): per-kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbv
mkdir -p $O
for v in "1 0" "0 0" "1 1" "0 1"; do
  set -- $v
  rm -rf $O/p_$1_$2
  NNMPI_RB_ROT=$1 NNMPI_RB_DIAG=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 bench.py --steps 30 --warmup 5 > $O/log_$1_$2.txt 2>&1 || exit $?
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$1" "$2" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'rowband' in r['Name'] or 'multi' in r['Name']:
        print("rot", sys.argv[2], "diag", sys.argv[3], r['Name'][:40], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
