#!/bin/bash
# One rank, RCCL path forced: no comm vs inline, interleaved, N reps at the given rows
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=$1; shift; REPS=${REPS:-4}
O=gpurun_out/r6fc/$TAG; mkdir -p $O
for rows in "$@"; do
  for i in $(seq 1 $REPS); do
    for m in none inline; do
      if [ $m = none ]; then args=""; else args="--force_comm --comm_mode inline"; fi
      timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 --no_extras $args > $O/${m}_${rows}_$i.json 2> $O/${m}_${rows}_$i.err || { tail -5 $O/${m}_${rows}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${m}_${rows}_$i.json').read().strip().splitlines()[-1]); print('rows $rows', '$m', d['ms_per_step'], d['config']['schedule'], d['config'].get('comm_mode'))" | tee -a $O/summary.txt
    done
  done
done
