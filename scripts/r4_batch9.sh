#!/bin/bash
# multi-rank selection (bf16 tuner rehearsal, ordered fp32 reduce at P=3 incl. overlap_rowband vs
# inline bitwise), then the collective stand-in sweep on the wide model
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_check.sh r4chk7 "tests/test_bench.py::test_bench_tunes_the_bf16_reduction_algorithm tests/test_multirank_gpu.py" || exit $?
bash scripts/r4_standin.sh
