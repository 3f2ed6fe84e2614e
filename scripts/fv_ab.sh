set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k forward_variants --timeout 120 --timeout-method thread > gpurun_out/fv_tests.log 2>&1
for v in 0 10 11 12 13 0 10 11 12 13; do
  timeout -k 10 120 python bench.py --config mnist --steps 100 --warmup 10 --fwd_variant $v | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('mnist v$v', d['ms_per_step'])" >> gpurun_out/fv.txt
done
