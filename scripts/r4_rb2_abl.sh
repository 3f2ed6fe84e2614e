#!/bin/bash
# Ablations of the v2 row-band kernel: 0 full, 1 no MFMA, 2 no weight refills, 3 no copy-outs;
# plus 1,024 rows (32 blocks) and PMC counters of the full kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r4abl; mkdir -p $O
cd /tmp
for a in 0 1 2 3 0; do
  NNMPI_RB2_ABL=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/abl$a -o run -- python3 $R/bench.py --steps 40 --warmup 3 --no_extras > $O/abl$a.log 2>&1 || exit $?
  echo "abl $a: $(grep rowband2 $O/abl$a/run_kernel_stats.csv | cut -d, -f3-5)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r1024 -o run -- python3 $R/bench.py --steps 40 --warmup 3 --no_extras --rows 1024 > $O/r1024.log 2>&1 || exit $?
echo "rows 1024: $(grep rowband $O/r1024/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-120)"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc_g$i -o run -- python3 $R/bench.py --steps 8 --warmup 2 --graph_chunk 1 --no_extras > $O/pmc_g$i.log 2>&1
  echo "pmc group $i rc=$?"
done
python3 $R/scripts/pmc_summary.py $O/pmc_g* --match rowband2 2>&1 | head -20
exit 0
