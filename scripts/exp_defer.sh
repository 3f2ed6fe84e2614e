#!/bin/bash
# Deferred updates fused into chunk weight-gradient epilogues (several ranks, bf16 payload):
# bitwise tests (1-rank RCCL overlap vs inline; 2 RCCL ranks), then the wide overlapped step
# A/B (NNMPI_DEFER=0: separate per-bucket SGD passes), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/defer
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_engine_gpu.py tests/test_multirank_gpu.py \
  -k "wide_chunked or chunked_buckets or bf16_payload" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest.log | tail -8
for r in 1 2 3; do
  for d in 1 0; do
    NNMPI_DEFER=$d timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras --force_comm --comm_mode overlap > $O/b.json 2>> $O/bench.err || exit $?
    echo "wide overlap defer=$d $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 python bench.py --config wide8192 --steps 30 --warmup 5 --no_extras > $O/b.json 2>> $O/bench.err || exit $?
echo "wide nocomm $(python -c "import json;print(json.load(open('$O/b.json'))['ms_per_step'])")" | tee -a $O/ab.txt
