#!/bin/bash
# Comm/compute CU contention on the overlapped wide schedule (VERDICT r3 Next 3): one rank with
# --force_comm (the RCCL comm path, which issues no kernels at one rank) plus the collective
# stand-in holding k CUs after each bucket for its bytes at 1.07 TB/s (all 7 xGMI links) and at
# 0.3 TB/s; k = 0, 8, 16, 32; the inline (no-overlap) schedule for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r4standin; mkdir -p $O
run() {  # name standin mode
  NNMPI_COMM_STANDIN=$2 timeout -k 10 300 python bench.py --config wide8192 --steps 12 --warmup 3 \
      --force_comm --no_extras --comm_mode $3 > $O/$1.json 2> $O/$1.err || return $?
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['config']['comm_mode'], d['config']['n_buckets'])" | tee -a $O/summary.txt
}
for rep in 1 2; do
  run inline_$rep "" inline || exit $?
  for k in 0 8 16 32; do
    run ov_k${k}_1070_$rep $k:1070 overlap || exit $?
  done
  for k in 16 32; do
    run ov_k${k}_300_$rep $k:300 overlap || exit $?
  done
done
