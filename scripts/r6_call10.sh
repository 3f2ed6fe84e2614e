#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python bench.py --gpus 2 --shared_gpu_rehearsal --steps 8 --warmup 2 --tune_steps 4 > gpurun_out/r6/reh_test.json 2> gpurun_out/r6/reh_test.err
echo "rc=$?"
python -c "
import json; d=json.loads(open('gpurun_out/r6/reh_test.json').read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ('fallback','attempts','measured_mode','extras_error')})[:3000])
print(d['config'].get('comm_mode'), d['config'].get('comm_tune_ms_per_step'))
"
tail -40 gpurun_out/r6/reh_test.err
