#!/bin/bash
# Deep-ring (10-slot, 160 KiB) 256x256 GEMM vs the 8-slot ping-pong kernel and hipBLASLt:
# correctness on ragged shapes (bitwise vs the default kernel), standalone 8192-wide timings,
# and the whole wide step interleaved A/B.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ring
mkdir -p $O
set -o pipefail
# ragged shapes through the forced 256x256 tile: every own variant must be bitwise equal
timeout -k 10 200 python scripts/gemm_bench.py --rows 1000 --inf 1032 --outf 776 --rounds 1 --iters 1 \
  --impls 2 --tiles 256 --variants 0,19,20,21,22 > $O/ragged.json 2> $O/ragged.err || exit $?
timeout -k 10 200 python scripts/gemm_bench.py --rows 4096 --inf 2048 --outf 8192 --rounds 1 --iters 1 \
  --impls 2 --tiles 256 --variants 0,19,20,21,22 >> $O/ragged.json 2>> $O/ragged.err || exit $?
cat $O/ragged.json
timeout -k 10 300 python scripts/gemm_bench.py --rows 4096 --inf 8192 --outf 8192 --rounds 5 --iters 5 \
  --impls 0,2 --tiles 0 --variants 0,19,20,21,22 > $O/wide.json 2> $O/wide.err || exit $?
cat $O/wide.json
for r in 1 2; do
  for v in 0 20 21 22; do
    timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras --gemm_variant $v >> $O/bench_wide.jsonl 2>> $O/bench_wide.err || exit $?
  done
done
cut -c1-200 $O/bench_wide.jsonl
