#!/bin/bash
# Full GPU suite, then proxy / MNIST / wide A/B of the optimizer-operand prefetch in the split-K
# combines and the batched SGD epilogue (NNMPI_SGD_SERIAL=1 = the previous per-fragment forms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/sgdpre
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for c in proxy512 mnist; do
    for v in 0 1; do
      NNMPI_SGD_SERIAL=$v timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 20 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
      echo "$c serial=$v $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
    done
  done
done
