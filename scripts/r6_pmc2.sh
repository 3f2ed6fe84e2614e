#!/bin/bash
# Round 6 PMC, second set: the multi-rank step's kernels (one rank with the RCCL path forced:
# the tiled image-refreshing optimizer pass sgd_tiles, the no-update wgrad_small / slab_multi) at
# 1,024 and 8,192 rows, and the MNIST step after the round-6 head LDS padding.  Each counter group
# its own rocprofv3 pass (kernel-trace only).  Summaries: scripts/pmc_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$(pwd); O=$R/gpurun_out/r6pmc2; mkdir -p $O
( while true; do date > $O/heartbeat; sleep 50; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
for tag in fc1024 fc8192 mnist; do
  case $tag in
    fc1024) BA="--rows 1024 --force_comm --comm_mode inline" ;;
    fc8192) BA="--rows 8192 --force_comm --comm_mode inline" ;;
    mnist) BA="--config mnist" ;;
  esac
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/${tag}_g$i -o run -- \
      python3 $R/bench.py $BA --steps 8 --warmup 2 --graph_chunk 1 --no_extras > $O/${tag}_g$i.log 2>&1
    rc=$?
    echo "$tag pmc group $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/${tag}_g$i.log; exit 1; }
  done
  python3 $R/scripts/pmc_summary.py $O/${tag}_g* > $O/summary_$tag.txt
done
exit 0
