#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 300 python scripts/r4_rb2_diag.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log | tail -30; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_v2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 60 --warmup 5 --no_extras > $GRAFT_REPO_ROOT/$O/prof_v2.log 2>&1
rc=$?; echo "prof rc=$rc"
find $GRAFT_REPO_ROOT/$O/prof_v2 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -8 {} | cut -c1-150'
