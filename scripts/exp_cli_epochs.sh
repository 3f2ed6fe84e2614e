#!/bin/bash
# The compat CLI on one GPU (512-wide proxy, full-batch epochs): fast epoch replay vs one
# replay + loss readback per epoch; mean epoch time over 2000 epochs from --metrics_json.
cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out
for f in "" "--no_fast_epochs"; do
  timeout -k 10 200 python dataParallelTraining_NN_MPI.py --preset proxy512 --nepochs 2000 --print_rank none --metrics_json gpurun_out/m.jsonl $f > /dev/null 2>> gpurun_out/cli.err || exit $?
  python3 -c "
import json; r=[json.loads(l) for l in open('gpurun_out/m.jsonl')][100:]
print(json.dumps({'flags': '$f', 'epochs': len(r), 'mean_epoch_ms': round(1e3*sum(x['epoch_s'] for x in r)/len(r), 4)}))" >> gpurun_out/cli_epochs.jsonl
  rm -f gpurun_out/m.jsonl
done
cat gpurun_out/cli_epochs.jsonl
