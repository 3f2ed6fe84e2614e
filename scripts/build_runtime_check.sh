#!/bin/bash
# Build the native runtime check with HOST AddressSanitizer + UBSan (device code uninstrumented:
# every -fsanitize= sits behind -Xarch_host).  Output: native_tests/runtime_check_asan (in-tree,
# git-ignored, travels to the GPU box with the tree).  Run it there with
#   ASAN_OPTIONS=detect_leaks=0 ./neural-networks-parallel-training-with-mpi_amd/native_tests/runtime_check_asan
set -euo pipefail
cd "$(dirname "$0")/../neural-networks-parallel-training-with-mpi_amd"
ROCM=${ROCM_PATH:-/opt/rocm}
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer"
"$ROCM/bin/hipcc" --offload-arch=gfx950 -O1 -g -std=c++17 $SAN \
  -I csrc -I "$ROCM/include" -Wno-unused-command-line-argument \
  -x hip native_tests/runtime_check.cpp -x hip csrc/comm/rccl_comm.cpp \
  csrc/kernels/optim.hip csrc/kernels/data.hip \
  -L "$ROCM/lib" -lrccl -Wl,-rpath,"$ROCM/lib" -o native_tests/runtime_check_asan
echo "built native_tests/runtime_check_asan"
