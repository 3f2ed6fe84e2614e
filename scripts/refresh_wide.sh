#!/bin/bash
# bench (RCCL path through a 1-rank communicator) + trainer metrics smoke + wide-config kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --force_comm --steps 100 --warmup 10 > gpurun_out/bench_fc.json 2> gpurun_out/bench_fc.err || exit $?
timeout -k 10 240 python dataParallelTraining_NN_MPI.py --device cuda --preset proxy512 --nepochs 20 --lr 1e-5 --profile_steps --metrics_json gpurun_out/metrics.jsonl --ref_samples_per_s 8e7 --print_rank none > gpurun_out/train_metrics.log 2>&1 || exit $?
rm -rf gpurun_out/prof_wide8192
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wide8192 -o run -- python3 bench.py --config wide8192 --steps 20 --warmup 3 > gpurun_out/prof_wide8192.log 2>&1
