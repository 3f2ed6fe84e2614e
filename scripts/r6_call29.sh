#!/bin/bash
# weight-gradient tile probe: 128 x 128 DMA tile vs 256 x 256 ping-pong tile, split caps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 200 python -u scripts/r6_wgrad_tile_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python scripts/r6_wgrad_tile_probe.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python - $(find $O/prof -name "*kernel_stats.csv" | head -1) <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f"   {float(r['AverageNs'])/1e3:8.2f} us  x{r['Calls']:>5}  {r['Name'].replace('void ', '').replace('nnmpi::', '')[:90]}")
PY
