cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config wide8192 --steps 20 --warmup 3 > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
