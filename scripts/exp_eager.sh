cd "${GRAFT_REPO_ROOT}" || exit 2
o=gpurun_out/eager.jsonl
for args in "--no_graph" "--no_graph --force_comm --comm_mode inline" "--no_graph --force_comm --comm_mode overlap" "--force_comm --comm_mode overlap --graph_chunk 1" "--force_comm --comm_mode overlap --bucket_mb 8"; do
  timeout -k 10 200 python bench.py --no_extras --steps 200 --warmup 20 $args >> $o 2>> gpurun_out/eager.err || exit $?
done
