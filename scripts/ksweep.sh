cd $GRAFT_REPO_ROOT
for shp in "8192 512 512" "8192 1024 512" "8192 2048 512" "8192 256 512" "4096 512 512" "16384 512 512" "8192 512 1024"; do
  set -- $shp
  timeout -k 5 120 python scripts/gemm_bench.py --rows $1 --inf $2 --outf $3 --rounds 5 --iters 20 --impls 2 --tiles 0 --only fwd,wgrad >> gpurun_out/ksweep.json 2>>gpurun_out/ksweep.err || exit $?
done
