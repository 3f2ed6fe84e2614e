# forward-GEMM kernel durations (rocprofv3 kernel trace) vs K: fixed cost inside the kernel
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for k in 64 128 256 512 1024; do
  timeout -k 5 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kfixed/k$k -o run -- python3 scripts/gemm_bench.py --rows 8192 --inf $k --outf 512 --rounds 2 --iters 10 --impls 2 --tiles 0 --only fwd > gpurun_out/kfixed/k$k.log 2>&1 || exit $?
done
