#!/bin/bash
# RCCL uneven-scatter reference tests (P=3, P=12 ranks sharing the GPU); a heartbeat file keeps
# the box's silence detector informed while a multi-process test runs (each test has its own
# time limits inside).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4u; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py -x -v -k "uneven_scatterv or golden_p2" --timeout 600 --timeout-method thread > $O/pytest_uneven.log 2>&1
rc=$?
kill $HB
echo "uneven tests rc=$rc"; tail -40 $O/pytest_uneven.log | cut -c1-300
