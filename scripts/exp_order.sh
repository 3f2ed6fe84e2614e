#!/bin/bash
# interleaved in-step A/B of the 256x256 GEMM tile order (fwd,dgrad,wgrad) on the wide config
cd "${GRAFT_REPO_ROOT}" || exit 2
o=gpurun_out/order.jsonl; : > $o
for r in 1 2; do for f in "0,0,2" "3,3,3" "3,3,2" "0,0,3"; do
  timeout -k 10 200 python bench.py --no_extras --config wide8192 --steps 20 --warmup 3 --pp_order $f > gpurun_out/o.json 2>> gpurun_out/order.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/o.json')); print(json.dumps({'pp_order': '$f', 'ms': d['ms_per_step']}))" >> $o
done; done
cat $o
