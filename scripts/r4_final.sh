#!/bin/bash
# Round 4 end-of-round numbers: every bench config (driver form) + kernel stats of proxy / MNIST / wide
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r4final; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
for cfg in proxy512 mnist wide8192 ref; do
  timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
  python -c "import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'], d['vs_baseline'], d['config']['schedule'])"
done
for cfg in proxy512 mnist wide8192; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o k -- \
    python bench.py --config $cfg --steps 20 --warmup 5 > $O/prof_$cfg.log 2>&1 || exit $?
done
echo done
