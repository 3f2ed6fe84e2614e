#!/bin/bash
# Short timed regions: is the 20/50-step gap to 200 steps a warm-up (clock) effect?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/warm
mkdir -p $O
for r in 1 2; do
  for sw in "20 5" "20 200" "50 5" "50 200" "200 20"; do
    set -- $sw
    timeout -k 10 300 python bench.py --steps $1 --warmup $2 > $O/b.json 2>> $O/bench.err || exit $?
    echo "steps=$1 warmup=$2 $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
