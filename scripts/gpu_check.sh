#!/bin/bash
# One GPU-box session: smoke -> GPU tests -> 1-GPU bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout (rc not in {0,1}) ends the script.
# Usage: scripts/gpu_check.sh [steps...]   (default: smoke tests bench prof)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${*:-smoke tests bench prof}"

ok_or_stop() {  # $1 = rc, $2 = name
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "[gpu_check] $2 ended with rc=$1 -> stopping" | tee -a gpurun_out/summary.txt
    exit "$1"
  fi
  echo "[gpu_check] $2 rc=$1" | tee -a gpurun_out/summary.txt
}

for s in $STEPS; do
  case "$s" in
    smoke)
      timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      ok_or_stop $? smoke ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      ok_or_stop $? tests ;;
    multirank)
      # P >= 2 on the one GPU: gloo-shared and RCCL (per-rank NCCL_HOSTID) rank processes
      timeout -k 10 1000 python -u -m pytest tests/test_multirank_gpu.py tests/test_bench.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/pytest_multirank.log 2>&1
      ok_or_stop $? multirank ;;
    testsall)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      ok_or_stop $? testsall ;;
    gemm)
      timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.json 2> gpurun_out/gemm_bench.err
      ok_or_stop $? gemm
      timeout -k 10 300 python scripts/gemm_bench.py --inf 8192 --outf 8192 --rows 4096 --rounds 3 --iters 5 --tiles 0 >> gpurun_out/gemm_bench.json 2>> gpurun_out/gemm_bench.err
      ok_or_stop $? gemm8k
      cat gpurun_out/gemm_bench.json ;;
    bench)
      timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
      ok_or_stop $? bench
      cat gpurun_out/bench.json ;;
    abgroup)
      for r in 1 2; do
        timeout -k 10 300 python bench.py >> gpurun_out/ab_group.json 2>> gpurun_out/ab_group.err
        ok_or_stop $? "bench grouped"
        timeout -k 10 300 python bench.py --no_group >> gpurun_out/ab_group.json 2>> gpurun_out/ab_group.err
        ok_or_stop $? "bench ungrouped"
      done
      cat gpurun_out/ab_group.json ;;
    gemmwide)
      timeout -k 10 300 python scripts/gemm_bench.py --rows 4096 --inf 8192 --outf 8192 --rounds 3 --iters 5 --impls 0,2 --tiles 0,128,256 --variants 0,9 > gpurun_out/gemm_wide.json 2> gpurun_out/gemm_wide.err
      ok_or_stop $? gemmwide
      timeout -k 10 300 python scripts/gemm_bench.py --rows 8192 --inf 1024 --outf 1024 --rounds 5 --iters 10 --impls 0,2 --tiles 0,128,256 >> gpurun_out/gemm_wide.json 2>> gpurun_out/gemm_wide.err
      ok_or_stop $? gemmmnist
      cat gpurun_out/gemm_wide.json ;;
    variants)
      timeout -k 10 300 python scripts/gemm_bench.py --impls 2 --tiles 128 --variants 0,1,2,3,8 > gpurun_out/variants.json 2> gpurun_out/variants.err
      ok_or_stop $? variants512
      timeout -k 10 300 python scripts/gemm_bench.py --inf 1024 --outf 1024 --impls 2 --tiles 128 --variants 0,1,2,3,8 >> gpurun_out/variants.json 2>> gpurun_out/variants.err
      ok_or_stop $? variants1024
      cat gpurun_out/variants.json ;;
    sweep512)
      # proxy-shape GEMMs: every 128/64-tile DMA variant vs hipBLASLt (impl 0), one process
      timeout -k 10 300 python scripts/gemm_bench.py --rows 8192 --inf 512 --outf 512 --rounds 8 --iters 20 --impls 0,2 --tiles 0,128 --variants 0,1,2,3,5,6,7,8 > gpurun_out/sweep512.json 2> gpurun_out/sweep512.err
      ok_or_stop $? sweep512
      cat gpurun_out/sweep512.json ;;
    stepab)
      # whole-step knob A/B (forward variant, grouped-backward LDS read mode, wgrad splits)
      timeout -k 10 400 python scripts/step_ab.py > gpurun_out/step_ab.json 2> gpurun_out/step_ab.err
      ok_or_stop $? stepab
      cat gpurun_out/step_ab.json ;;
    benchall)
      for c in proxy512 mnist wide8192 ref; do
        timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 >> gpurun_out/bench_all.json 2>> gpurun_out/bench_all.err
        ok_or_stop $? "bench $c"
      done
      cat gpurun_out/bench_all.json ;;
    profcfg)
      # per-kernel stats of the other bench configs (mnist / ref / wide8192)
      for c in mnist ref wide8192; do
        rm -rf gpurun_out/prof_$c
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 3 > gpurun_out/prof_$c.log 2>&1
        ok_or_stop $? "prof $c"
      done ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 5 > gpurun_out/prof.log 2>&1
      ok_or_stop $? prof
      find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \; ;;
  esac
done
echo "[gpu_check] done" | tee -a gpurun_out/summary.txt
