# interleaved A/B of one bench flag: exp_ab.sh "<flags A>" "<flags B>"
cd "${GRAFT_REPO_ROOT}" || exit 2
o=gpurun_out/ab.jsonl
for r in 1 2 3; do for f in "$1" "$2"; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 $f >> $o 2>> gpurun_out/ab.err || exit $?
  timeout -k 10 120 python bench.py --config mnist --steps 100 --warmup 10 $f >> $o 2>> gpurun_out/ab.err || exit $?
done; done
for f in "$1" "$2"; do
  timeout -k 10 200 python bench.py --config wide8192 --steps 20 --warmup 3 $f >> $o 2>> gpurun_out/ab.err || exit $?
done
