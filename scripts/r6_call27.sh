#!/bin/bash
# round-6 session-2 final: GPU suite, smoke, every bench config (driver form), kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6n; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 150 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-200
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1; rc=$?
tail -3 $O/gpu_suite.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r6_final.sh bench && bash scripts/r6_final.sh prof
