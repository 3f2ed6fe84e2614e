#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rowband.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest_rowband.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python -c "import json,sys; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['config']['schedule'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 60 --warmup 5 --no_extras > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
echo "prof rc=$?"
python3 - $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if "nnmpi" in r["Name"]: print(r["Name"][:60], r["Calls"], "%.2f us" % (float(r["AverageNs"])/1000))
PY
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_multirank_gpu.py -x -v -k "uneven_scatterv" --timeout 600 --timeout-method thread > $O/pytest_uneven.log 2>&1
echo "uneven tests rc=$?"; tail -4 $O/pytest_uneven.log
