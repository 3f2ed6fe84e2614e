#!/bin/bash
# Round 4 GPU batch: fused head (r4_head.sh), hipBLASLt kernel names of the wide GEMMs, then the
# multi-rank / row-band / tuner test selection (r4_check.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_head.sh r4head || exit $?
bash scripts/r4_wgstages.sh r4wg || exit $?
mkdir -p gpurun_out/r4blt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4blt/prof -o blt -- \
  python scripts/r4_hipblaslt_names.py > gpurun_out/r4blt/log 2>&1 || exit $?
f=$(find gpurun_out/r4blt/prof -name "*kernel_stats.csv" | head -1)
cut -c1-300 "$f" | head -8
bash scripts/r4_check.sh r4chk4 "tests/test_multirank_gpu.py::test_rccl_reference_golden_p2_scatterv tests/test_multirank_gpu.py::test_rccl_reference_uneven_scatterv_matches_cpu tests/test_multirank_gpu.py::test_rowband_overlap_matches_inline_bitwise tests/test_rowband_gpu.py tests/test_bench.py::test_bench_three_rank_rowband_uneven_rehearsal tests/test_bench.py::test_bench_tunes_the_bf16_reduction_algorithm"
