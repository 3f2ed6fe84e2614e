#!/bin/bash
# PMC counters per kernel of the training step (bench.py) and of the standalone proxy GEMMs
# (gemm_bench.py), one counter group per rocprofv3 run, --kernel-trace only beside --pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
BENCH="bench.py --steps 8 --warmup 2 --graph_chunk 1 ${BENCH_ARGS:-}"
GEMM="scripts/gemm_bench.py --rounds 2 --iters 5 --impls 2 --tiles 0"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" ; do
  i=$((i+1))
  for prog in ${PROGS:-bench gemm}; do
    if [ $prog = bench ]; then ARGS=$BENCH; else ARGS=$GEMM; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/${prog}_g$i -o run -- python3 $ARGS > $OUT/${prog}_g$i.log 2>&1
    rc=$?
    echo "$prog group $i rc=$rc" >> $OUT/summary.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
exit 0
