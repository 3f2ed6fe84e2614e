#!/bin/bash
# Warm-up top-up: the driver's short forms, a 2-rank shared-GPU rehearsal (every rank must run
# the same top-up), bench GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/warm2
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
  echo "20/5 $(python -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d['warmup_steps_run'])")" | tee -a $O/ab.txt
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/b.json 2>> $O/bench.err || exit $?
echo "200/20 $(python -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d['warmup_steps_run'])")" | tee -a $O/ab.txt
timeout -k 10 300 python bench.py --config wide8192 --steps 20 --warmup 5 > $O/b.json 2>> $O/bench.err || exit $?
echo "wide 20/5 $(python -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d['warmup_steps_run'])")" | tee -a $O/ab.txt
timeout -k 10 400 python bench.py --gpus 2 --shared_gpu_rehearsal --steps 20 --warmup 5 > $O/r2.json 2>> $O/r2.err || exit $?
echo "rehearsal dp2 $(python -c "import json;d=json.load(open('$O/r2.json'));print(d['ms_per_step'], d['warmup_steps_run'], d['rccl_ranks'], d['config']['comm_mode'])")" | tee -a $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_bench.py -m gpu > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
