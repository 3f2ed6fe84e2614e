#!/bin/bash
# Row-band forward A/B: staged (0) vs direct permuted-k loads (1); numerics, kernel times, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbf
mkdir -p $O
NNMPI_RB_FWD=1 timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread -k "oracle or graph" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "0 1" "1 1" "0 0" "1 0"; do
  set -- $v
  rm -rf $O/p_$1_$2
  NNMPI_RB_FWD=$1 NNMPI_RB_DIAG=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 bench.py --steps 30 --warmup 5 > $O/log_$1_$2.txt 2>&1 || exit $?
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$1" "$2" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rowband' in r['Name']:
        print("fwd", sys.argv[2], "diag", sys.argv[3], r['Name'][:40], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
for r in 1 2; do
  for fw in 0 1; do
    NNMPI_RB_FWD=$fw timeout -k 10 300 python bench.py > $O/b.json 2>> $O/bench.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('bench fwd $fw', d['ms_per_step'])"
  done
done
