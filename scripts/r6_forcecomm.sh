#!/bin/bash
# One rank, the RCCL path forced (--force_comm): no comm vs inline vs overlap_rowband at the given
# row counts, interleaved, plus a kernel trace of each comm mode (VERDICT r5 "Next" 1).
# Usage: r6_forcecomm.sh TAG [ROWS...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
ROWS=${@:-8192 1024}
O=gpurun_out/r6fc/$TAG; mkdir -p $O
for rows in $ROWS; do
  for i in 1 2; do
    for m in none inline inline_elementwise overlap_rowband; do
      E=""
      if [ $m = none ]; then args=""; elif [ $m = inline_elementwise ]; then args="--force_comm --comm_mode inline"; E="NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILES=0"; else args="--force_comm --comm_mode $m"; fi
      env $E timeout -k 10 300 python bench.py --rows $rows --steps 20 --warmup 5 --no_extras $args > $O/${m}_${rows}_$i.json 2> $O/${m}_${rows}_$i.err || { tail -5 $O/${m}_${rows}_$i.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${m}_${rows}_$i.json').read().strip().splitlines()[-1]); print('rows $rows', '$m', d['ms_per_step'], d['config']['schedule'], d['config'].get('comm_mode'), d['config'].get('f32_reduce'))" | tee -a $O/summary.txt
    done
  done
  for m in none inline inline_elementwise overlap_rowband; do
    E=""
    if [ $m = none ]; then args=""; elif [ $m = inline_elementwise ]; then args="--force_comm --comm_mode inline"; E="NNMPI_EXPERIMENTS=1 NNMPI_SGD_TILES=0"; else args="--force_comm --comm_mode $m"; fi
    env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${m}_$rows -o k -- \
      python bench.py --rows $rows --steps 20 --warmup 5 --no_extras $args > $O/p_${m}_$rows.log 2>&1 || { tail -5 $O/p_${m}_$rows.log; exit 1; }
    st=$(find $O/p_${m}_$rows -name "*kernel_stats.csv" | head -1)
    echo "== rows $rows $m kernels" | tee -a $O/summary.txt
    python - "$st" <<'PY' | tee -a $O/summary.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    n = r["Name"].replace("void ", "").replace("nnmpi::", "")[:70]
    print(f"   {float(r['AverageNs'])/1e3:8.2f} us  x{r['Calls']:>5}  {n}")
PY
  done
done
echo done
