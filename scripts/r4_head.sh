#!/bin/bash
# Round 4: fused multi-output head (head_mo.hip) on the GPU -- head oracle tests, MNIST-config
# bench fused vs two launches (NNMPI_HEAD_FUSED=0, experiments), kernel stats of the fused step.
# Usage: scripts/r4_head.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-r4head}; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "head" -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20 | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/r4_head_stamps.py > $O/stamps.txt 2>&1 || exit $?
cat $O/stamps.txt
for i in 1 2 3; do
  for f in 1 0; do
    NNMPI_EXPERIMENTS=1 NNMPI_HEAD_FUSED=$f timeout -k 10 300 python bench.py --config mnist \
      --steps 20 --warmup 5 > $O/bench_f${f}_$i.json 2> $O/bench_f${f}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_f${f}_$i.json').read().strip().splitlines()[-1]); print('fused=$f', d['ms_per_step'], d['value'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mnist -- \
  python bench.py --config mnist --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -12
