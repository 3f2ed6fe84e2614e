#!/bin/bash
# MNIST step: weight-gradient split caps (the layer-0 combine reads 8 slabs by default) and
# forward variants, interleaved in one process (scripts/step_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 500 python -u scripts/step_ab.py --config mnist --rounds 5 --steps 64 \
  --configs '[{}, {"wsplit": 4}, {"wsplit": 2}, {"gasync": 2}, {"slab": 2}, {}]' > $O/mnist_ab.txt 2> $O/mnist_ab.err || { tail -20 $O/mnist_ab.err; exit 1; }
cat $O/mnist_ab.txt
