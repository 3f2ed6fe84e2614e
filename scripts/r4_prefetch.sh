#!/bin/bash
# Round 4: operand prefetch in the 8192-wide weight gradient's SGD epilogue (pp256_tile PF) --
# kernel A/B with bitwise check (scripts/r4_wgrad_prefetch_ab.py), then the wide step with
# NNMPI_PP_PREFETCH 0 / 1 / 2 interleaved (experiments).  Usage: scripts/r4_prefetch.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pf}; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
NNMPI_EXPERIMENTS=1 timeout -k 10 240 python -u scripts/r4_wgrad_prefetch_ab.py > $O/ab.txt 2>&1
rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for pf in 0 1 2; do
    NNMPI_EXPERIMENTS=1 NNMPI_PP_PREFETCH=$pf timeout -k 10 300 python bench.py --config wide8192 \
      --steps 20 --warmup 5 > $O/bench_pf${pf}_$i.json 2> $O/bench_pf${pf}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_pf${pf}_$i.json').read().strip().splitlines()[-1]); print('pf=$pf', d['ms_per_step'], d['knobs'])"
  done
done
