#!/bin/bash
# Round 3 GEMM session: 256x256 DMA-issue placement A/B (one half per phase vs 1/0/2/1), the wide
# step with both, the 1-rank RCCL wide step's kernel timeline, general-head timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
step() { echo "[r3g] $1 rc=$2" | tee -a $O/summary.txt; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
if [ -z "$ONLY_TAIL" ]; then
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "pp256_one_half or wide_pair or wide_sgd or test_reference_config_on_gpu" > $O/pytest.log 2>&1
step pytest $?
timeout -k 10 300 python scripts/gemm_bench.py --rows 4096 --inf 8192 --outf 8192 --rounds 5 --iters 5 --impls 0,2 --tiles 0 --variants 15,16,17,18 > $O/gemm_wide.jsonl 2> $O/gemm_wide.err
step gemm_wide $?
for r in 1 2; do
  for o in 0,0,1 2,2,3; do
    timeout -k 10 300 python bench.py --config wide8192 --steps 50 --warmup 5 --no_extras --pp_order $o >> $O/wide_step.jsonl 2>> $O/wide_step.err
    step "wide $o" $?
  done
done
timeout -k 10 400 python scripts/step_ab.py --config proxy512 --rounds 7 --steps 128 --configs '[{}, {"slab": 2}, {"slab": 1}, {}]' > $O/proxy_slab_ab.jsonl 2> $O/proxy_slab_ab.err
step proxy_slab_ab $?
timeout -k 10 400 python scripts/step_ab.py --config wide8192 --rounds 3 --steps 20 --chunk 10 --configs '[{}, {"pp": "2,2,3"}, {"pp": "0,0,3"}, {"pp": "2,2,1"}]' > $O/wide_pp_ab.jsonl 2> $O/wide_pp_ab.err
step wide_pp_ab $?
fi
timeout -k 10 300 python scripts/head_bench.py > $O/head.jsonl 2> $O/head.err
step head $?
rm -rf $O/trace_fc
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_fc -o run -- python3 bench.py --config wide8192 --force_comm --comm_mode overlap --steps 10 --warmup 3 --no_extras > $O/trace_fc.log 2>&1
step trace_fc $?
f=$(find $O/trace_fc -name "*kernel_trace.csv" | head -1)
python scripts/trace_step.py "$f" 60 > $O/trace_fc_timeline.txt
cp "$f" $O/trace_fc_kernel_trace.csv
echo done >> $O/summary.txt
