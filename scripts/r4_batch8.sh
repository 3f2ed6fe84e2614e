#!/bin/bash
# head block-cap A/B, then the multi-rank selection (ordered fp32 reduce at P=3, the bf16 tuner
# rehearsal after the chunk-workspace fix)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_head_cap.sh || exit $?
bash scripts/r4_check.sh r4chk6 "tests/test_bench.py::test_bench_tunes_the_bf16_reduction_algorithm tests/test_multirank_gpu.py"
