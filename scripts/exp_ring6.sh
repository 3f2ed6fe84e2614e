#!/bin/bash
# 6-slot ring forms (less L2 pressure) vs the default 256x256 kernel; bitwise checks first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/ring6
mkdir -p $O
timeout -k 10 200 python scripts/gemm_bench.py --rows 1000 --inf 1032 --outf 776 --rounds 1 --iters 1 \
  --impls 2 --tiles 256 --variants 0,23,24 > $O/ragged.json 2> $O/ragged.err || exit $?
timeout -k 10 300 python scripts/gemm_bench.py --rows 4096 --inf 8192 --outf 8192 --rounds 5 --iters 5 \
  --impls 0,2 --tiles 0 --variants 0,20,23,24 > $O/wide.json 2> $O/wide.err || exit $?
cat $O/ragged.json $O/wide.json
