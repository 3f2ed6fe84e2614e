#!/bin/bash
# headline step: XCD-contiguous band order + 8 XCD-aligned weight-gradient splits (split s of every
# layer on XCD s reads the rows XCD s wrote) against the defaults; interleaved, driver form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TOPK=3 bash scripts/r5_ab.sh r6bm "-" "NNMPI_EXPERIMENTS=1 NNMPI_RB_BANDMAP=1 NNMPI_RB_SPLITS=8" \
  "NNMPI_EXPERIMENTS=1 NNMPI_RB_BANDMAP=1" "NNMPI_EXPERIMENTS=1 NNMPI_RB_SPLITS=8" \
  "NNMPI_EXPERIMENTS=1 NNMPI_RB_BANDMAP=1 NNMPI_RB_SPLITS=4" "-" || exit 1
