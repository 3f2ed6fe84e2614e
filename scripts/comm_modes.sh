# 1-GPU timing of every gradient-sync schedule through the RCCL path (--force_comm: a 1-rank
# communicator, so the collectives are no-ops and the numbers show the schedule's own cost)
cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
o=gpurun_out/comm_modes.jsonl; e=gpurun_out/comm_modes.err
: > $o; : > $e
run() { timeout -k 10 240 python bench.py --no_extras "$@" >> $o 2>> $e; rc=$?; echo "rc=$rc $*" >> gpurun_out/comm_modes.rc; [ $rc -eq 0 ] || exit $rc; }
run --steps 200 --warmup 20
run --steps 200 --warmup 20 --force_comm --comm_mode inline
run --steps 200 --warmup 20 --force_comm --comm_mode zero1
run --steps 200 --warmup 20 --force_comm --comm_mode overlap
run --config mnist --steps 100 --warmup 10
run --config mnist --steps 100 --warmup 10 --force_comm --comm_mode overlap
run --config wide8192 --steps 20 --warmup 3
run --config wide8192 --steps 20 --warmup 3 --force_comm --comm_mode overlap
run --config wide8192 --steps 20 --warmup 3 --force_comm --comm_mode overlap --grad_dtype fp32
