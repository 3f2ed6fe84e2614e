#!/bin/bash
# grouped weight-gradient launch: register-staged operands (NNMPI_WG_REG=1) vs the LDS-DMA ring,
# proxy512 bench interleaved (final loss must match: bitwise-equal gradients), row-band tests with
# the register variant, kernel stats of it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp NNMPI_EXPERIMENTS=1
O=gpurun_out/r4wgreg; mkdir -p $O
for i in 1 2 3; do
  for r in 1 0; do
    NNMPI_WG_REG=$r timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_r${r}_$i.json 2> $O/bench_r${r}_$i.err || exit $?
    python -c "import json; d=json.loads(open('$O/bench_r${r}_$i.json').read().strip().splitlines()[-1]); print('reg=$r', d['ms_per_step'], d['final_loss'])"
  done
done
NNMPI_WG_REG=1 timeout -k 10 300 python -m pytest tests/test_rowband_gpu.py -x -q --timeout 200 > $O/pytest.log 2>&1; echo "rowband tests (reg) rc=$?"; tail -2 $O/pytest.log
NNMPI_WG_REG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o k -- python bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -5
