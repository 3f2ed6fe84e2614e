#!/bin/bash
# Round 5: row-band phase stamps + the driver-form proxy bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r5s; mkdir -p $O
timeout -k 10 300 python -u scripts/r5_rb_stamps.py 8192 40 > $O/stamps.txt 2>&1 || { cat $O/stamps.txt; exit 1; }
cat $O/stamps.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['config']['schedule'])"
