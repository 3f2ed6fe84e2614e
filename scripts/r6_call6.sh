#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/rowband_tests.txt 2>&1 || { tail -30 gpurun_out/r6/rowband_tests.txt; exit 1; }
tail -2 gpurun_out/r6/rowband_tests.txt
O=gpurun_out/r6fc/rt; mkdir -p $O
for rows in 8192 1024; do
  for i in 1 2; do
    for v in none rt1 rt2; do
      E=""; args="--force_comm --comm_mode inline"
      [ $v = none ] && args=""
      [ $v = rt1 ] && E="NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=1"
      env $E timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 --no_extras $args > $O/${v}_${rows}_$i.json 2> $O/${v}_${rows}_$i.err || { tail -5 $O/${v}_${rows}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${v}_${rows}_$i.json').read().strip().splitlines()[-1]); print('rows $rows', '$v', d['ms_per_step'])" | tee -a $O/summary.txt
    done
  done
done
for v in rt1 rt2; do
  E=""; [ $v = rt1 ] && E="NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILE_RT=1"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o k -- python bench.py --rows 1024 --steps 20 --warmup 5 --no_extras --force_comm --comm_mode inline > $O/p_$v.log 2>&1 || { tail -5 $O/p_$v.log; exit 1; }
  echo "== $v"; grep -h sgd_tiles $(find $O/p_$v -name "*kernel_stats.csv") | cut -d, -f1-5
done
ROWS="1024 8192" bash scripts/r6_pmc.sh || exit 1
