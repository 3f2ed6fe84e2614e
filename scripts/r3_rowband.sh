#!/bin/bash
# Row-band step on one MI355X: its GPU tests, the proxy bench with and without it, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rb
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for r in 1 2; do
  NNMPI_ROWBAND=1 timeout -k 10 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  NNMPI_ROWBAND=0 timeout -k 10 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
python -c "
import json
for l in open('$O/bench.jsonl'):
    d=json.loads(l); print(d['ms_per_step'], d['value'])"
rm -rf $O/prof
NNMPI_ROWBAND=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
