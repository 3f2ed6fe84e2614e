cd "${GRAFT_REPO_ROOT}" || exit 2
o=gpurun_out/store.jsonl
for r in 1 2 3; do for pol in 0 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --store_policy $pol >> $o 2>> gpurun_out/store.err || exit $?
done; done
for pol in 0 1 2; do
  timeout -k 10 120 python bench.py --config mnist --steps 100 --warmup 10 --store_policy $pol >> $o 2>> gpurun_out/store.err || exit $?
done
