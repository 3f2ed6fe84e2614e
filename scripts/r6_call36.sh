#!/bin/bash
# MNIST strong-scaling shard (1,024 rows per GPU): step and per-kernel times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
BARGS="--config mnist --rows 1024" TOPK=10 bash scripts/r5_ab.sh r6mn1024 "-" || exit 1
BARGS="--config mnist --rows 2048" TOPK=10 bash scripts/r5_ab.sh r6mn2048 "-" || exit 1
