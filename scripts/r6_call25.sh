#!/bin/bash
# re-created container: rebuilt library -> GPU suite, smoke, default bench (driver form)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 150 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
