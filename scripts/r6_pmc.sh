#!/bin/bash
# Round 6 PMC counters (VERDICT r5 "Next" 4 and 7): the strong-scaling shard step (column-split
# row-band kernel + wgrad_small) at 1,024 / 2,048 rows and the headline proxy step (rowband2,
# wgrad_multi, slab_multi) at 8,192 rows; each counter group its own rocprofv3 pass (kernel-trace
# only).  Summaries: python3 scripts/pmc_summary.py gpurun_out/r6pmc/<tag>_g*
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r6pmc; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
for rows in ${ROWS:-1024 2048 8192}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/rows${rows}_g$i -o run -- \
      python3 $R/bench.py --rows $rows --steps 8 --warmup 2 --graph_chunk 1 --no_extras > $O/rows${rows}_g$i.log 2>&1
    rc=$?
    echo "rows $rows pmc group $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/rows${rows}_g$i.log; exit 1; }
  done
  python3 $R/scripts/pmc_summary.py $O/rows${rows}_g* > $O/summary_rows$rows.txt
done
exit 0
