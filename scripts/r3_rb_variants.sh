#!/bin/bash
# Row-band kernel: GPU tests, then per-kernel times of the full step and of the forward-only
# diagnostic (NNMPI_RB_DIAG=1), and the proxy bench with / without the row-band step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbv
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "1 0" "1 1"; do
  set -- $v
  rm -rf $O/p_$1_$2
  NNMPI_ROWBAND=1 NNMPI_RB_ROT=$1 NNMPI_RB_DIAG=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$1_$2 -o run -- python3 bench.py --steps 30 --warmup 5 > $O/log_$1_$2.txt 2>&1 || exit $?
  f=$(find $O/p_$1_$2 -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$1" "$2" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'rowband' in r['Name'] or 'multi' in r['Name']:
        print("rot", sys.argv[2], "diag", sys.argv[3], r['Name'][:40], round(float(r['AverageNs'])/1000, 2), round(float(r['MinNs'])/1000, 2))
PY
done
for r in 1 2; do
  NNMPI_ROWBAND=1 timeout -k 10 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  NNMPI_ROWBAND=0 timeout -k 10 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
python3 -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print('bench', d['ms_per_step'], d['value'])"
