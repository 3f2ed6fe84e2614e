#!/bin/bash
# final tree: GPU suite, smoke, default bench (driver form), 4-rank shared-GPU RCCL rehearsal
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6q; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { tail -30 $O/bench_20.err; exit 1; }
tail -1 $O/bench_20.json | cut -c1-220
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1; rc=$?
tail -3 $O/gpu_suite.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 4 --steps 10 --warmup 3 --shared_gpu_rehearsal > $O/reh_n4.json 2> $O/reh_n4.err || { tail -20 $O/reh_n4.err; exit 1; }
python -c "import json; d=json.loads(open('$O/reh_n4.json').read().strip().splitlines()[-1]); c=d['config']; print('N=4', d['ms_per_step'], c['comm_mode'], c['schedule'], d['replicas_bitwise_equal'], json.dumps(d.get('strong_scaling')), json.dumps(c.get('comm_tune_ms_per_step')))"
