#!/bin/bash
# End-of-session check on one MI355X: smoke, full GPU suite, the driver's bench forms, a 4-rank
# shared-GPU rehearsal of the multi-rank bench path.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.json 2>> $O/bench.err || exit $?
timeout -k 10 600 python bench.py --gpus 4 --shared_gpu_rehearsal --steps 20 --warmup 5 > $O/rehearsal_4rank.json 2> $O/rehearsal.err || exit $?
for f in bench_20_5 bench_default rehearsal_4rank; do
  echo "$f $(python -c "import json;d=json.load(open('$O/$f.json'));print(d['n_gpus'], d['ms_per_step'], d['value'], d['warmup_steps_run'], d['config']['comm_mode'])")"
done
