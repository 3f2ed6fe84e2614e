#!/bin/bash
# 8192-wide GEMMs: 256x256 ping-pong default (late LDS-read retire + grouped tile order GM 4)
# vs variants 16 (neither), 17 (late retire only), 18 (GM 8), and hipBLASLt (impl 0); own variants checked bitwise against the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_bench.py --rows 4096 --inf 8192 --outf 8192 --rounds 3 --iters 5 --impls 0,2 --tiles 256 --variants 0,16,17,18 > gpurun_out/wide_variants.json 2> gpurun_out/wide_variants.err
