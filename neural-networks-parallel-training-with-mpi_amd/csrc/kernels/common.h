// Shared device helpers for the CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nnmpi {

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
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

}  // namespace nnmpi
