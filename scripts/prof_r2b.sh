#!/bin/bash
# Late round-2 evidence: PMC counters of the 8192-wide training step's kernels (one counter
# group per rocprofv3 run) and kernel traces of the wide step with the bf16-payload overlapped
# schedule (1-rank RCCL) and of the headline proxy step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc_wide PROGS=bench BENCH_ARGS="--config wide8192 --no_extras" bash scripts/pmc_step.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_wide/bench_g* > gpurun_out/pmc_wide8192_step_kernels.txt || exit $?
rm -rf gpurun_out/pmc_wide
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$n -o run -- python3 bench.py --no_extras "$@" > gpurun_out/prof_$n.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_$n -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kstats_$n.csv
  f=$(find gpurun_out/prof_$n -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/ktrace_$n.csv
  rm -rf gpurun_out/prof_$n
}
run wideov16 --config wide8192 --steps 10 --warmup 3 --force_comm --comm_mode overlap
run proxy --steps 50 --warmup 5
