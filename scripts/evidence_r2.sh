# Round-2 evidence run (1 GPU): headline bench, every config, kernel traces, 2-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_proxy512.json 2> gpurun_out/bench.err || exit $?
for c in mnist wide8192 ref mlp512x3; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 >> gpurun_out/bench_all.jsonl 2>> gpurun_out/bench.err || exit $?
done
timeout -k 10 400 python bench.py --gpus 2 --shared_gpu_rehearsal --steps 20 --warmup 3 --tune_steps 8 > gpurun_out/rehearsal_2rank.json 2> gpurun_out/rehearsal.err || exit $?
bash scripts/prof_r2.sh || exit $?
