#!/bin/bash
# Round 5 A/B: driver-form proxy bench + per-kernel durations (rocprofv3 kernel trace) for a list of
# environment variants.  Usage: [BARGS="--rows 1024"] [TOPK=8] r5_ab.sh TAG "ENV1" "ENV2" ...
# (ENV: space-separated K=V, or "-")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/r5/$TAG; mkdir -p $O
i=0
for V in "$@"; do
  i=$((i+1))
  E=""; [ "$V" != "-" ] && E="$V"
  # plain run first (timing), then a profiled run (kernel durations)
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no_extras $BARGS > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  ms=$(python -c "import json; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'])")
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$i -o k -- \
    python bench.py --steps 20 --warmup 5 --no_extras $BARGS > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
  st=$(find $O/p$i -name "*kernel_stats.csv" | head -1)
  echo "== [$i] $V : bench ${ms} ms"
  python - "$st" "${TOPK:-4}" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:int(sys.argv[2])]:
    n = r["Name"].replace("void ", "").replace("nnmpi::", "")[:60]
    print(f"   {float(r['AverageNs'])/1e3:8.2f} us  x{r['Calls']:>5}  {n}")
PY
done
