#!/bin/bash
# Round 4 PMC counters (each group its own rocprofv3 pass, kernel-trace only): the proxy step
# (row-band v2, grouped weight gradients, combines), the MNIST step (fused head) and the wide step
# (256x256 GEMMs).  Summaries: python3 scripts/pmc_summary.py gpurun_out/r4pmc/<cfg>_g*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4pmc; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
for cfg in proxy512 mnist wide8192; do
  steps=8; [ $cfg = wide8192 ] && steps=3
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/${cfg}_g$i -o run -- \
      python3 $R/bench.py --config $cfg --steps $steps --warmup 2 --graph_chunk 1 --no_extras > $O/${cfg}_g$i.log 2>&1
    echo "$cfg pmc group $i rc=$?"
  done
done
exit 0
