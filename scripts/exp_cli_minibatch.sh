#!/bin/bash
# The compat CLI with mini-batches (--batch_size 1024: 8 steps per epoch of the 8192-row proxy
# shard) on one GPU: mean epoch time from --metrics_json.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for bs in 1024 4096; do
  timeout -k 10 200 python dataParallelTraining_NN_MPI.py --preset proxy512 --batch_size $bs --nepochs 300 --print_rank none --metrics_json gpurun_out/m.jsonl > /dev/null 2>> gpurun_out/cli.err || exit $?
  python3 -c "
import json; r=[json.loads(l) for l in open('gpurun_out/m.jsonl')][50:]
print(json.dumps({'batch_size': $bs, 'epochs': len(r), 'steps_per_epoch': r[0]['steps'], 'mean_epoch_ms': round(1e3*sum(x['epoch_s'] for x in r)/len(r), 4)}))" >> gpurun_out/cli_mb.jsonl
  rm -f gpurun_out/m.jsonl
done
cat gpurun_out/cli_mb.jsonl
