#!/bin/bash
# Round 5: row-band GPU tests + phase stamps + driver-form proxy bench.  Usage: r5_check.sh TAG [pytest-files...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-x}; shift
O=gpurun_out/r5/$TAG; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/pytest.txt 2>&1
  rc=$?; tail -5 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u scripts/r5_rb_stamps.py 8192 40 > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || exit 1
  python -c "import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['value'], d['config']['schedule'])"
done
