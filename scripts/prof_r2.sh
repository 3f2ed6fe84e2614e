# rocprofv3 kernel traces of the headline bench (1 GPU), the overlapped schedule through the
# RCCL path (1-rank communicator) and the other configs; summaries land in gpurun_out/prof_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/prof_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$n -o run -- python3 bench.py --no_extras "$@" > gpurun_out/prof_$n.log 2>&1 || exit $?
}
run proxy --steps 50 --warmup 5
run proxyov --steps 50 --warmup 5 --force_comm --comm_mode overlap
run wide --config wide8192 --steps 10 --warmup 3
run mnist --config mnist --steps 50 --warmup 5
for n in proxy proxyov wide mnist; do
  f=$(find gpurun_out/prof_$n -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/kstats_$n.csv
  f=$(find gpurun_out/prof_$n -name "*kernel_trace.csv" | head -1); cp "$f" gpurun_out/ktrace_$n.csv
done
rm -rf gpurun_out/prof_proxy gpurun_out/prof_proxyov gpurun_out/prof_wide gpurun_out/prof_mnist
