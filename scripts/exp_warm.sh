#!/bin/bash
# Driver-shaped runs (--steps 20 --warmup 5): timed graphs captured before the warm-up steps
# (default) vs after them (NNMPI_BENCH_LATE_CAPTURE=1), interleaved.
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/exp_warm.jsonl; : > $o
run() { tag=$1; shift
  env NNMPI_BENCH_LATE_CAPTURE=$tag timeout -k 10 120 python bench.py --no_extras "$@" > gpurun_out/u.json 2>> gpurun_out/exp_warm.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/u.json')); print(json.dumps({'late': '$tag', 'args': '$*', 'ms': d['ms_per_step']}))" >> $o
}
for r in 1 2 3 4; do
  run 0 --gpus 1 --steps 20 --warmup 5
  run 1 --gpus 1 --steps 20 --warmup 5
done
run 0 --config mnist --gpus 1 --steps 20 --warmup 5
run 1 --config mnist --gpus 1 --steps 20 --warmup 5
run 0 --steps 200 --warmup 20
cat $o
