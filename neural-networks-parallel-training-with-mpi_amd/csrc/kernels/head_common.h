// Shared pieces of the skinny output-layer kernels (head.hip, head_mo.hip): the argument
// block, 8-wide activation loads/stores and the multi-output MFMA head's LDS weight-image
// layout and per-lane row-group loads.
#pragma once
#include "common.h"
#include "kernels.h"

namespace nnmpi {

constexpr int HEAD_OMAX = 16;

template <typename TA>
__device__ __forceinline__ void load8(const TA* p, float (&v)[8]);

struct HeadArgs {
  const void* a;
  int rows, in;
  const float* W;
  const float* b;
  int out;
  const float* y;
  const int64_t* labels;
  float inv_count;
  int act_prev;
  void* dz_prev;
  float* dlogits;
  float* loss_part;
  int xcd_rows;   // 1: rows of an XCD-remapped logical block (set_head_xcd_rows; experiment)
};

template <typename TA>
__device__ __forceinline__ void load8(const TA* p, float (&v)[8]) {
  if constexpr (sizeof(TA) == 2) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
  } else {
    const float4 x0 = *reinterpret_cast<const float4*>(p);
    const float4 x1 = *reinterpret_cast<const float4*>(p + 4);
    v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
    v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
  }
}

template <typename TA>
__device__ __forceinline__ void store8(TA* p, const float (&v)[8]) {
  if constexpr (sizeof(TA) == 2) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
    *reinterpret_cast<bf16x8*>(p) = x;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

constexpr int MH_WAVES = 4;

__device__ __forceinline__ int mh_off(int n, int k, int in) { return n * in + (((k >> 2) ^ (n & 15)) << 2) + (k & 3); }

// Global inputs of one 16-row group for one lane (row r = lane & 15, column group g = lane >> 4)
template <int Q>
struct MhLoads {
  bf16x8 xs[Q / 32];   // this wave's quarter, 8 features per 32-chunk (logits operand, and the
                       // saved activation the dZ of the same features needs)
  float yv[4];         // MSE targets of outputs 4g .. 4g+3
  int lab;             // cross-entropy label
};

template <int Q, int LOSS>
__device__ __forceinline__ void mh_load(MhLoads<Q>& L, const HeadArgs& p, const bf16* A, int rowc,
                                        int w, int g) {
  constexpr int in = 4 * Q;
  const bf16* ar = A + (long long)rowc * in + w * Q;
#pragma unroll
  for (int c = 0; c < Q / 32; ++c) L.xs[c] = *reinterpret_cast<const bf16x8*>(ar + c * 32 + g * 8);
  if constexpr (LOSS == LOSS_XENT) {
    L.lab = (int)p.labels[rowc];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) L.yv[j] = p.y[(long long)rowc * p.out + min(4 * g + j, p.out - 1)];
  }
}

}  // namespace nnmpi
