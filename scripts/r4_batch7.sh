#!/bin/bash
# fused head stamps + MNIST A/B, then the bf16 tuner rehearsal alone with its output kept
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
bash scripts/r4_head.sh r4head5 || exit $?
mkdir -p gpurun_out/r4tune
timeout -k 10 600 python bench.py --config wide2048 --gpus 3 --shared_gpu_rehearsal --rows 1024 \
  --chunk_tiles 16 --steps 4 --warmup 2 --tune_steps 3 --no_extras > gpurun_out/r4tune/out.json 2> gpurun_out/r4tune/err.txt
echo "tune rc=$?"; tail -c 1500 gpurun_out/r4tune/out.json; grep -E "supervisor|Error|error" gpurun_out/r4tune/err.txt | head -20
