#!/bin/bash
# headline step knob A/B, interleaved in one process (scripts/step_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 500 python -u scripts/step_ab.py --config proxy512 --rounds 5 --steps 128 --chunk 64 \
  --configs '[{}, {"wsplit": 4}, {"slab": 1}, {"slab": 2}, {"gasync": 2}, {"gasync": 3}, {}]' > $O/proxy_ab.txt 2> $O/proxy_ab.err || { tail -20 $O/proxy_ab.err; exit 1; }
cat $O/proxy_ab.txt
