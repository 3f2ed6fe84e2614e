#!/bin/bash
# The wide model through the RCCL path at one rank (--force_comm, overlapped chunk buckets):
# 4 vs 2 chunk buckets per layer, per-chunk vs per-layer deferred-update waits; no-comm step for
# reference.  Interleaved rounds, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
B="python bench.py --config wide8192 --steps 50 --warmup 5 --no_extras"
for r in 1 2; do
  for v in "nocomm" "c4 chunk" "c4 layer" "c2 layer"; do
    set -- $v
    case $1 in
      nocomm) cmd="$B" ;;
      c4) cmd="$B --force_comm --comm_mode overlap" ;;
      c2) cmd="$B --force_comm --comm_mode overlap --chunk_tiles 512" ;;
    esac
    NNMPI_DEFER_WAIT=${2:-layer} timeout -k 10 300 $cmd > $O/tmp.json 2>> $O/err.txt
    rc=$?
    echo "{\"variant\": \"$v\", \"round\": $r, \"rc\": $rc, \"line\": $(cat $O/tmp.json || echo null)}" >> $O/ab.jsonl
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "hash or wide_chunked or comm_overlap or defer" > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/ab.jsonl
