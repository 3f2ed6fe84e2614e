#!/bin/bash
# Row-band step: copy-out store policy A/B (0 plain, 1 nt, 2 sc1) on the proxy bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/rbst
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rowband_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for pol in 0 1 2; do
    NNMPI_ROWBAND=1 NNMPI_RB_STORE=$pol timeout -k 10 300 python bench.py > $O/b.json 2>> $O/bench.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('bench store $pol', d['ms_per_step'])"
  done
  NNMPI_ROWBAND=0 timeout -k 10 300 python bench.py > $O/b.json 2>> $O/bench.err || exit $?
  python3 -c "import json; d=json.load(open('$O/b.json')); print('bench grouped', d['ms_per_step'])"
done
