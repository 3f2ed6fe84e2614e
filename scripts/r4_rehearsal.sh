#!/bin/bash
# The driver's N-GPU bench form (torch.distributed.run ... bench.py --gpus N) rehearsed with N RCCL
# ranks sharing the one GPU (--shared_gpu_rehearsal), N = 2 and 4: every schedule + algorithm
# candidate tuned, one JSON line, replicas bitwise equal (loopback numbers, not xGMI)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4reh; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
for n in 2 4; do
  port=$((29500 + n * 7))
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 10 --warmup 3 --shared_gpu_rehearsal \
    > $O/n$n.json 2> $O/n$n.err || exit $?
  python -c "import json; d=json.loads(open('$O/n$n.json').read().strip().splitlines()[-1]); c=d['config']; print('N=$n', d['ms_per_step'], c['comm_mode'], c['schedule'], c['f32_reduce'], d['replicas_bitwise_equal'], d['fallback'], json.dumps(c['comm_tune_ms_per_step']))"
done
