#!/bin/bash
# one rank: the row-band step without comm vs with the RCCL path forced (inline and
# overlap_rowband), interleaved; VERDICT r3 Next 4 (<= 3 % over no-comm)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4fc; mkdir -p $O
for i in 1 2 3; do
  for m in none inline overlap_rowband; do
    if [ $m = none ]; then args=""; else args="--force_comm --comm_mode $m"; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_extras $args > $O/${m}_$i.json 2> $O/${m}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/${m}_$i.json').read().strip().splitlines()[-1]); print('$m', d['ms_per_step'], d['config']['schedule'], d['config']['comm_mode'], d['config'].get('f32_reduce'))" | tee -a $O/summary.txt
  done
done
