#!/bin/bash
# Round 4 GPU batch: bf16-split fused head (r4_head.sh), then the multi-rank / row-band / bench
# test selection (ordered fp32 reduce, transposed-image staging).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_head.sh r4head2 || exit $?
bash scripts/r4_check.sh r4chk5 "tests/test_multirank_gpu.py::test_rowband_overlap_matches_inline_bitwise tests/test_rowband_gpu.py tests/test_bench.py::test_bench_two_rank_rehearsal_on_one_gpu tests/test_bench.py::test_bench_three_rank_rowband_uneven_rehearsal tests/test_bench.py::test_bench_tunes_the_bf16_reduction_algorithm tests/test_multirank_gpu.py"
