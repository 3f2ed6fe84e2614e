#!/bin/bash
# Driver-shaped bench runs (--steps 20 --warmup 5), graph upload on vs off, interleaved,
# plus 200-step runs for reference.  One JSON line per run in gpurun_out/exp_upload.jsonl.
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/exp_upload.jsonl; : > $o
run() { tag=$1; shift
  env NNMPI_GRAPH_UPLOAD=$tag timeout -k 10 120 python bench.py --no_extras "$@" > gpurun_out/u.json 2>> gpurun_out/exp_upload.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open('gpurun_out/u.json')); print(json.dumps({'upload': '$tag', 'args': '$*', 'ms': d['ms_per_step']}))" >> $o
}
for r in 1 2 3; do
  run 1 --gpus 1 --steps 20 --warmup 5
  run 0 --gpus 1 --steps 20 --warmup 5
done
run 1 --steps 200 --warmup 20
run 0 --steps 200 --warmup 20
cat $o
