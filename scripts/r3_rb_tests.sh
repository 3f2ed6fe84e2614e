#!/bin/bash
# Row-band GPU tests + the multi-rank row-band test (RCCL ranks sharing the GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbt
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py "tests/test_multirank_gpu.py::test_rowband_rccl_two_ranks_inline_and_zero1_match_one_rank" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -20 $O/pytest.log
exit $rc
