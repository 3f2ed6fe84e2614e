#!/bin/bash
# fused head block cap A/B (NNMPI_HEAD_BLOCKS 256 / 128 / 64): stamps + MNIST bench, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r4cap; mkdir -p $O
for cap in 256 128 64; do
  NNMPI_HEAD_BLOCKS=$cap timeout -k 10 120 python scripts/r4_head_stamps.py > $O/stamps_$cap.txt 2>&1 || exit $?
  head -2 $O/stamps_$cap.txt
done
for i in 1 2; do
  for cap in 256 128 64; do
    NNMPI_HEAD_BLOCKS=$cap timeout -k 10 300 python bench.py --config mnist --steps 20 --warmup 5 \
      > $O/bench_${cap}_$i.json 2> $O/bench_${cap}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_${cap}_$i.json').read().strip().splitlines()[-1]); print('cap=$cap', d['ms_per_step'])"
  done
done
