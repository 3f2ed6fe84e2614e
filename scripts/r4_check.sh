#!/bin/bash
# Round 4 GPU check: selected test files (heartbeat for the silence detector; each pytest has
# its own limits), then the driver-form bench three times.
# Usage: scripts/r4_check.sh OUTDIR "pytest selection args..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-r4chk}; mkdir -p $O
SEL=${2:-tests -m gpu}
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest $SEL -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
kill $HB
echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -30 | cut -c1-200
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python -c "import json,sys; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['config']['schedule'], d['knobs'])"
done
exit $rc
