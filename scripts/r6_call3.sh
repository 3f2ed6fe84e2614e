#!/bin/bash
# Round 6: the band kernel below 6,144 rows (4,097-6,143-row shards ran the
# 8-launch grouped schedule) -- driver-form bench at 4,500 / 5,000 / 6,000 rows with the band
# threshold at 4,097 vs 6,144; then the PMC passes (scripts/r6_pmc.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6thr; mkdir -p $O
for rows in 4500 5000 6000; do
  for i in 1 2; do
    for thr in 6144 4097; do
      NNMPI_EXPERIMENTS=1 NNMPI_ROWBAND_MIN_ROWS=$thr timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 --no_extras > $O/b_${rows}_${thr}_$i.json 2> $O/b_${rows}_${thr}_$i.err || { tail -5 $O/b_${rows}_${thr}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/b_${rows}_${thr}_$i.json').read().strip().splitlines()[-1]); print('rows $rows threshold $thr', d['ms_per_step'], d['config']['schedule'])" | tee -a $O/summary.txt
    done
  done
done
bash scripts/r6_pmc.sh || exit 1
