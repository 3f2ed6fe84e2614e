#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest tests/test_split_contention_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r6/contention_tests.txt 2>&1; echo "contention pytest rc=$?"; tail -6 gpurun_out/r6/contention_tests.txt
bash scripts/r6_contend.sh || exit 1
REPS=3 bash scripts/r6_fc2.sh nozero 8192 1024 || exit 1
O=gpurun_out/r6thr; mkdir -p $O
for rows in 4500 5000 6000; do
  for thr in 6144 4097; do
    NNMPI_EXPERIMENTS=1 NNMPI_ROWBAND_MIN_ROWS=$thr timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 --no_extras > $O/b_${rows}_${thr}.json 2> $O/b_${rows}_${thr}.err || { tail -5 $O/b_${rows}_${thr}.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/b_${rows}_${thr}.json').read().strip().splitlines()[-1]); print('rows $rows threshold $thr', d['ms_per_step'], d['config']['schedule'])" | tee -a $O/summary.txt
  done
done
