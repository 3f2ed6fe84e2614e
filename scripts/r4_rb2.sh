#!/bin/bash
# Round 4: row-band v2 (fragment-major weight images) -- tests, A/B bench vs v1, kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
O=gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests/test_rowband_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_rowband.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/pytest_rowband.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for i in 1 2; do
  for v in 2 1; do
    NNMPI_RB_V2=$([ $v = 2 ] && echo 1 || echo 0) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_v${v}_$i.json 2> $O/bench_v${v}_$i.err || exit $?
    python -c "import json,sys; d=json.loads(open('$O/bench_v${v}_$i.json').read().strip().splitlines()[-1]); print('v$v', d['ms_per_step'], d['value'], d['config']['schedule'], d['replicas_bitwise_equal'], d['final_loss'])"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_v2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 60 --warmup 5 --no_extras > $GRAFT_REPO_ROOT/$O/prof_v2.log 2>&1
rc=$?; echo "prof rc=$rc"
find $GRAFT_REPO_ROOT/$O/prof_v2 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -6 {} | cut -c1-160'
