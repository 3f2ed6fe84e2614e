#!/bin/bash
# Row-band A/B: two activation images + one stage per wave (default) vs one image updated in place
# + two stage buffers per wave (NNMPI_RB_DB=1).  Numerics of both, kernel times, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbdb
mkdir -p $O
for db in 1 0; do
  NNMPI_RB_DB=$db timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_$db.log 2>&1 || { tail -40 $O/pytest_$db.log; exit 1; }
  echo "db $db: $(tail -1 $O/pytest_$db.log)"
done
for db in 0 1; do
  rm -rf $O/p_$db
  NNMPI_RB_DB=$db timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$db -o run -- python3 bench.py --steps 30 --warmup 5 > $O/log_$db.txt 2>&1 || exit $?
  f=$(find $O/p_$db -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$db" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rowband' in r['Name']:
        print("db", sys.argv[2], r['Name'][:44], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
for r in 1 2; do
  for db in 0 1; do
    NNMPI_RB_DB=$db timeout -k 10 300 python bench.py > $O/b.json 2>> $O/bench.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('bench db $db', d['ms_per_step'])"
  done
done
