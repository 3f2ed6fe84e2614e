#!/bin/bash
# Per-rank step time vs rows per rank (the strong-scaling shards: 8192/N rows), 1 GPU, plus a
# kernel trace of the 1024-row step.
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/rows.jsonl; : > $o
for r in 8192 4096 2048 1024; do
  timeout -k 10 120 python bench.py --no_extras --steps 200 --warmup 20 --rows $r > gpurun_out/r.json 2>> gpurun_out/rows.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r.json')); print(json.dumps({'rows': $r, 'ms': d['ms_per_step']}))" >> $o
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1024 -o run -- python3 bench.py --no_extras --steps 50 --warmup 5 --rows 1024 > gpurun_out/prof_r1024.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r1024 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kstats_r1024.csv
f=$(find gpurun_out/prof_r1024 -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/ktrace_r1024.csv
rm -rf gpurun_out/prof_r1024
cat $o
