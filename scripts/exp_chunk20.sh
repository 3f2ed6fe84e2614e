#!/bin/bash
# Driver-shaped runs (--steps 20 --warmup 5): one 20-step graph (auto) vs 16 + 4 (--graph_chunk 16),
# interleaved.  One JSON line per run in gpurun_out/exp_chunk20.jsonl.
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/exp_chunk20.jsonl; : > $o
run() { timeout -k 10 120 python bench.py --no_extras "$@" > gpurun_out/u.json 2>> gpurun_out/exp_chunk20.err
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/u.json')); print(json.dumps({'args': '$*', 'ms': d['ms_per_step'], 'chunk': d['config']['graph_chunk']}))" >> $o
}
for r in 1 2 3; do
  run --gpus 1 --steps 20 --warmup 5
  run --gpus 1 --steps 20 --warmup 5 --graph_chunk 16
done
run --config mnist --gpus 1 --steps 20 --warmup 5
run --config mnist --gpus 1 --steps 20 --warmup 5 --graph_chunk 16
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.json 2>> gpurun_out/exp_chunk20.err || exit $?
cat $o gpurun_out/bench_full.json
