cd "${GRAFT_REPO_ROOT}" || exit 2
o=gpurun_out/chunk.jsonl
for r in 1 2 3; do for c in 16 50 200; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --graph_chunk $c >> $o 2>> gpurun_out/chunk.err || exit $?
done; done
