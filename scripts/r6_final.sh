#!/bin/bash
# Round 6 end-of-round numbers: every bench config (driver form), the strong-scaling shard sizes,
# kernel stats of proxy / 1,024-row shard / MNIST / wide, and the 2-rank shared-GPU rehearsal
# (its strong_scaling block runs the column-split row-band step).  Usage: r5_final.sh [part]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=${R6OUT:-gpurun_out/r6final}; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
PART=${1:-all}
show() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); c=d['config']; print('$2', d['ms_per_step'], d['value'], d['vs_baseline'], c.get('schedule'), c.get('global_batch'))"; }
if [ "$PART" = all ] || [ "$PART" = bench ]; then
  for cfg in proxy512 mnist wide8192 ref; do
    timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
    show $O/bench_$cfg.json $cfg
  done
  for rows in 1024 2048 4096 5000; do
    timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 > $O/bench_rows$rows.json 2> $O/bench_rows$rows.err || exit $?
    show $O/bench_rows$rows.json rows$rows
  done
fi
if [ "$PART" = all ] || [ "$PART" = prof ]; then
  for cfg in proxy512 mnist wide8192; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o k -- \
      python bench.py --config $cfg --steps 20 --warmup 5 > $O/prof_$cfg.log 2>&1 || exit $?
  done
  for rows in 1024 2048; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rows$rows -o k -- \
      python bench.py --rows $rows --steps 20 --warmup 5 > $O/prof_rows$rows.log 2>&1 || exit $?
  done
fi
if [ "$PART" = all ] || [ "$PART" = reh ]; then
  n=2; port=29517
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 10 --warmup 3 --shared_gpu_rehearsal \
    > $O/reh_n$n.json 2> $O/reh_n$n.err || exit $?
  python -c "import json; d=json.loads(open('$O/reh_n$n.json').read().strip().splitlines()[-1]); c=d['config']; print('N=$n', d['ms_per_step'], c['comm_mode'], c['schedule'], d['replicas_bitwise_equal'], json.dumps(d.get('strong_scaling')), json.dumps(c.get('comm_tune_ms_per_step')))"
fi
echo done
