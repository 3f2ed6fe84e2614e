#!/bin/bash
# PMC counters for the MLP GEMM kernels (counters in their own runs, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}; mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1
ARGS="scripts/gemm_bench.py --rounds 2 --iters 5 --impls ${IMPLS:-2} --tiles ${TILES:-0} --only ${ONLY:-fwd,dgrad,wgrad} ${EXTRA:-}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $ARGS > $OUT/g$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $OUT/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
