// Shared device helpers for the CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace nnmpi {

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };

constexpr int WAVE = 64;

__device__ __forceinline__ float act_fwd(float x, int act) {
  if (act == ACT_RELU) return x > 0.f ? x : 0.f;
  if (act == ACT_TANH) return tanhf(x);
  return x;
}

// Derivative of the activation expressed through its OUTPUT a = act(z):
// relu'(z) = [a > 0] (threshold_backward on the result), tanh'(z) = 1 - a^2.
__device__ __forceinline__ float act_bwd_from_out(float a, int act) {
  if (act == ACT_RELU) return a > 0.f ? 1.f : 0.f;
  if (act == ACT_TANH) return 1.f - a * a;
  return 1.f;
}

template <int ACT>
__device__ __forceinline__ float act_fwd_t(float x) {
  if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == ACT_TANH) return tanhf(x);
  else return x;
}

template <int ACT>
__device__ __forceinline__ float act_bwd_t(float a) {
  if constexpr (ACT == ACT_RELU) return a > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == ACT_TANH) return 1.f - a * a;
  else return 1.f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Grouped tile order: consecutive block ids walk a GM-row band column by column, so the
// blocks one XCD runs at the same time (consecutive ids after xcd_remap) cover a GM x (n/GM)
// patch of output tiles and share GM A panels + n/GM B panels in that XCD's L2, instead of one
// A panel + n distinct B panels (row-major order).  Bijective for any gx, gy (the last band may
// be shorter).
__device__ __forceinline__ void grouped_tile(int bid, int gx, int gy, int gm, int& tx, int& ty) {
  if (gm <= 1) {
    tx = bid % gx;
    ty = bid / gx;
    return;
  }
  const int per = gm * gx, first = (bid / per) * gm;
  const int gsz = min(gy - first, gm), r = bid % per;
  ty = first + r % gsz;
  tx = r / gsz;
}

// torch.optim.SGD update of one element (sgd.py semantics; dampening/nesterov/weight decay).
// Contraction is pinned (explicit fmaf, no compiler contraction) so every kernel that applies
// the update -- the standalone optimizer pass or a fused reducer epilogue -- rounds identically.
__device__ __forceinline__ float sgd_elem(float p, float g, float& buf, float lr, float mom,
                                          float damp, float wd, float gs, bool nesterov,
                                          bool first) {
#pragma clang fp contract(off)
  float d = g * gs;
  if (wd != 0.f) d = fmaf(wd, p, d);
  if (mom != 0.f) {
    buf = first ? d : fmaf(mom, buf, (1.f - damp) * d);
    d = nesterov ? fmaf(mom, buf, d) : buf;
  }
  return fmaf(-lr, d, p);
}

__device__ __forceinline__ void sgd_fused_store(const SgdFuse& f, const float* gaddr, float g) {
  const long long off = gaddr - f.g_base;
  float buf = f.m_base[off];
  const float pn = sgd_elem(f.p_base[off], g, buf, f.hp[0], f.hp[1], f.hp[2], f.hp[3], f.hp[4],
                            f.nesterov != 0, f.first != 0);
  f.p_base[off] = pn;
  if (f.hp[1] != 0.f) f.m_base[off] = buf;
  if (f.s_base) f.s_base[off] = (bf16)pn;
}

// sgd_fused_store4 in two halves, so a caller can issue the master / momentum / hyper-parameter
// loads BEFORE the loads that produce the gradient (a split-K combine: the slab sums), keeping
// them off the dependent chain.  Same arithmetic: bitwise identical.
struct SgdPre4 {
  f32x4 p, b;
  long long off;
  float lr, mom, damp, wd, gs;
};
__device__ __forceinline__ SgdPre4 sgd_pre4(const SgdFuse& f, const float* gaddr) {
  SgdPre4 q;
  q.off = gaddr - f.g_base;
  q.p = *reinterpret_cast<const f32x4*>(f.p_base + q.off);
  q.b = *reinterpret_cast<const f32x4*>(f.m_base + q.off);
  q.lr = f.hp[0]; q.mom = f.hp[1]; q.damp = f.hp[2]; q.wd = f.hp[3]; q.gs = f.hp[4];
  return q;
}
__device__ __forceinline__ f32x4 sgd_apply4(const SgdFuse& f, SgdPre4 q, f32x4 g) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float bb = q.b[r];
    q.p[r] = sgd_elem(q.p[r], g[r], bb, q.lr, q.mom, q.damp, q.wd, q.gs, f.nesterov != 0, f.first != 0);
    q.b[r] = bb;
  }
  *reinterpret_cast<f32x4*>(f.p_base + q.off) = q.p;
  if (q.mom != 0.f) *reinterpret_cast<f32x4*>(f.m_base + q.off) = q.b;
  if (f.s_base) {
    bf16x4 sv;
#pragma unroll
    for (int r = 0; r < 4; ++r) sv[r] = (bf16)q.p[r];
    *reinterpret_cast<bf16x4*>(f.s_base + q.off) = sv;
  }
  return q.p;
}

__device__ __forceinline__ f32x4 sgd_fused_store4(const SgdFuse& f, const float* gaddr, f32x4 g) {
  const long long off = gaddr - f.g_base;
  f32x4 p = *reinterpret_cast<const f32x4*>(f.p_base + off);
  f32x4 b = *reinterpret_cast<const f32x4*>(f.m_base + off);
  const float lr = f.hp[0], mom = f.hp[1], damp = f.hp[2], wd = f.hp[3], gs = f.hp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float bb = b[r];
    p[r] = sgd_elem(p[r], g[r], bb, lr, mom, damp, wd, gs, f.nesterov != 0, f.first != 0);
    b[r] = bb;
  }
  *reinterpret_cast<f32x4*>(f.p_base + off) = p;
  if (mom != 0.f) *reinterpret_cast<f32x4*>(f.m_base + off) = b;
  if (f.s_base) {
    bf16x4 sv;
#pragma unroll
    for (int r = 0; r < 4; ++r) sv[r] = (bf16)p[r];
    *reinterpret_cast<bf16x4*>(f.s_base + off) = sv;
  }
  return p;
}

// Element offset of (row n, column k) of a [N][K] bf16 matrix (K % 32 == 0) in its FRAGMENT-MAJOR
// image (rowband.hip v2): fragment (n >> 4, k >> 5) is 1 KiB, the v_mfma_f32_16x16x32_bf16
// operand map -- lane (n & 15) + 16 * ((k >> 3) & 3) holds its 8 consecutive k at (k & 7).
__host__ __device__ __forceinline__ long long rb_pk_off(int n, int k, int K) {
  return (((long long)(n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((n & 15) + 16 * ((k >> 3) & 3))) * 8 + (k & 7);
}

// The updated values p of M[m][n .. n+3] ([M][N] row-major, n % 4 == 0) into the fragment-major
// images of M (pkf, may be null) and of M^T (pkd, may be null).
__device__ __forceinline__ void rb_pack_store4(bf16* pkf, bf16* pkd, int m, int n, int M, int N, f32x4 p) {
  if (pkf) {
    bf16x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (bf16)p[r];
    *reinterpret_cast<bf16x4*>(pkf + rb_pk_off(m, n, N)) = v;
  }
  if (pkd) {
#pragma unroll
    for (int r = 0; r < 4; ++r) pkd[rb_pk_off(n + r, m, M)] = (bf16)p[r];
  }
}

}  // namespace nnmpi
