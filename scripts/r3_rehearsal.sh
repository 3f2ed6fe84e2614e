#!/bin/bash
# The driver's multi-GPU bench command form, rehearsed with the ranks sharing the one GPU
# (--shared_gpu_rehearsal: NCCL_HOSTID per rank, RCCL over loopback): NOT a measurement, a check
# that the supervised torchrun path prints one line with replicas_bitwise_equal at N = 2, 4, 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
for n in ${NS:-2 4 8}; do
  port=$((29000 + n))
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 20 --warmup 5 --shared_gpu_rehearsal > $O/torchrun_$n.json 2> $O/torchrun_$n.err
  rc=$?
  echo "[r3r] torchrun n=$n rc=$rc" | tee -a $O/summary.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
