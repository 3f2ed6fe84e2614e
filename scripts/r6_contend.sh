#!/bin/bash
# Two processes running split steps on one GPU: default / write-through only / consecutive map
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r6c
for v in "-" "NNMPI_RB_SPLIT_LOCAL=0" "NNMPI_RB_SPLIT_MAP=0"; do
  E=""; [ "$v" != "-" ] && E="$v"
  for rep in 1 2; do
    d=$(mktemp -d)
    ( env $E NNMPI_ROWBAND_MIN_ROWS=6144 NNMPI_EXPERIMENTS=1 timeout -k 5 200 python tests/_split_contend_entry.py $d 0 1024 > gpurun_out/r6c/a.txt 2>&1 ) &
    ( env $E NNMPI_ROWBAND_MIN_ROWS=6144 NNMPI_EXPERIMENTS=1 timeout -k 5 200 python tests/_split_contend_entry.py $d 1 4096 > gpurun_out/r6c/b.txt 2>&1 ) &
    wait
    echo "[$v rep $rep] 1024: $(tail -1 gpurun_out/r6c/a.txt)  4096: $(tail -1 gpurun_out/r6c/b.txt)"
    rm -rf $d
  done
done
