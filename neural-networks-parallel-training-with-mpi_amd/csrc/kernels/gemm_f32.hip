// Exact-fp32 MFMA GEMM (v_mfma_f32_16x16x4_f32) for the fp32 training mode.
//
// gfx950 has no xf32/TF32 path; its f32-input MFMA is bit-for-bit a k-ordered fmaf chain at the
// f32 vector rate and leaves the VALU free for the epilogue (cdna_hip_programming.md §3
// "FP32-input MFMA").  This kernel serves the reference-precision (float32, ref.py:159) configs
// above the tiny-MLP limit.  Same orientation/epilogue contract as gemm_bf16.hip: swapped MFMA
// operands so a lane owns 4 consecutive output columns; operands staged as [k][x] fp32 LDS
// images padded by 16 floats (ds_read_b32 halves land on disjoint bank sets); split-K slabs +
// the shared deterministic reducer for the wgrad orientation.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace nnmpi {

namespace f32g {
enum Layout : int { KMAJ = 0, XMAJ = 1 };
constexpr int BX = 64, BK = 32, LDX = BX + 16, THREADS = 256;

struct Params {
  const float* A;
  const float* B;
  int lda, ldb, M, N, K, k_per_split;
  float* C;
  int ldc;
  long long c_split_stride;
  const float* bias;
  const float* aux;
  int ldaux;
  float* bias_grad;
  long long bg_split_stride;
};

template <int LAYOUT>
__device__ __forceinline__ void load_tile(float (*lds)[LDX], const float* __restrict__ base, int ld,
                                          int x0, int X, int k0, int kend, int tid) {
#pragma unroll
  for (int it = 0; it < BX * BK / THREADS; ++it) {
    const int e = tid + it * THREADS;
    int x, k;
    if constexpr (LAYOUT == KMAJ) { k = e % BK; x = e / BK; }
    else { x = e % BX; k = e / BX; }
    const int gx = x0 + x, gk = k0 + k;
    float v = 0.f;
    if (gx < X && gk < kend) v = (LAYOUT == KMAJ) ? base[(long long)gx * ld + gk] : base[(long long)gk * ld + gx];
    lds[k][x] = v;
  }
}

template <int LA, int LB, int EPI, int ACT, bool BG>
__global__ void __launch_bounds__(THREADS) gemm_f32_kernel(Params p) {
  __shared__ float As[BK][LDX];
  __shared__ float Bs[BK][LDX];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int gx = gridDim.x, gy = gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
  const int tx = bid % gx, ty = bid / gx;
  const int m0 = ty * BX, n0 = tx * BX;
  const int split = blockIdx.z;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  f32x4 acc[2][2];
  f32x4 accb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool do_bg = BG && tx == 0 && wn == 0;
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    load_tile<LA>(As, p.A, p.lda, m0, p.M, k0, kend, tid);
    load_tile<LB>(Bs, p.B, p.ldb, n0, p.N, k0, kend, tid);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      const int k = ks + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[k][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[k][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[j], a[i], acc[i][j], 0, 0, 0);
      if constexpr (BG) {
        if (do_bg) {
#pragma unroll
          for (int i = 0; i < 2; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(1.f, a[i], accb[i], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 32 + i * 16 + (lane & 15);
    if (m >= p.M) continue;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane >> 4) * 4;
      f32x4 v = acc[i][j];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (n + r >= p.N) continue;
        float x = v[r];
        if constexpr (EPI == EPI_BIAS_ACT) {
          if (p.bias) x += p.bias[n + r];
          x = act_fwd_t<ACT>(x);
          p.C[(long long)m * p.ldc + n + r] = x;
        } else if constexpr (EPI == EPI_DACT) {
          x *= act_bwd_t<ACT>(p.aux[(long long)m * p.ldaux + n + r]);
          p.C[(long long)m * p.ldc + n + r] = x;
        } else {
          p.C[split * p.c_split_stride + (long long)m * p.ldc + n + r] = x;
        }
      }
    }
  }
  if constexpr (BG) {
    if (do_bg && (lane >> 4) == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = m0 + wm * 32 + i * 16 + lane;
        if (m < p.M) p.bias_grad[split * p.bg_split_stride + m] = accb[i][0];
      }
    }
  }
}

template <int LA, int LB, int EPI, bool BG>
static hipError_t launch(const Params& p, int act, int splits, hipStream_t s) {
  dim3 grid((p.N + BX - 1) / BX, (p.M + BX - 1) / BX, splits);
  switch (act) {
    case ACT_RELU: hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, EPI, ACT_RELU, BG>), grid, dim3(THREADS), 0, s, p); break;
    case ACT_TANH: hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, EPI, ACT_TANH, BG>), grid, dim3(THREADS), 0, s, p); break;
    default: hipLaunchKernelGGL((gemm_f32_kernel<LA, LB, EPI, ACT_NONE, BG>), grid, dim3(THREADS), 0, s, p);
  }
  return hipGetLastError();
}

static int splits_for(int M, int N, int K) {
  const int tiles = ((M + BX - 1) / BX) * ((N + BX - 1) / BX);
  const int ksteps = (K + BK - 1) / BK;
  int s = 1;
  while (tiles * s < 256 && s * 2 <= ksteps && s < 64) s *= 2;
  return s;
}
}  // namespace f32g

hipError_t linear_fwd_f32(const float* X, int ldx, const float* W, int ldw, const float* bias,
                          float* Y, int ldy, int M, int N, int K, int act, hipStream_t s) {
  f32g::Params p{};
  p.A = X; p.lda = ldx; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K; p.k_per_split = K;
  p.C = Y; p.ldc = ldy; p.bias = bias;
  return f32g::launch<f32g::KMAJ, f32g::KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s);
}

hipError_t linear_dgrad_f32(const float* dZ, int lddz, const float* W, int ldw,
                            const float* Aprev, int lda_prev, float* dX, int lddx, int M, int N,
                            int K, int act, hipStream_t s) {
  f32g::Params p{};
  p.A = dZ; p.lda = lddz; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K; p.k_per_split = K;
  p.C = dX; p.ldc = lddx; p.aux = Aprev; p.ldaux = lda_prev;
  return f32g::launch<f32g::KMAJ, f32g::XMAJ, EPI_DACT, false>(p, act, 1, s);
}

size_t wgrad_f32_workspace_bytes(int M, int N, int K) {
  const int s = f32g::splits_for(M, N, K);
  return s == 1 ? 0 : (size_t)s * ((size_t)M * N + M) * sizeof(float);
}

hipError_t linear_wgrad_f32(const float* dZ, int lddz, const float* X, int ldx, float* dW,
                            float* db, int M, int N, int K, float* ws, hipStream_t s) {
  const int splits = f32g::splits_for(M, N, K);
  const int ksteps = (K + f32g::BK - 1) / f32g::BK;
  f32g::Params p{};
  p.A = dZ; p.lda = lddz; p.B = X; p.ldb = ldx; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((ksteps + splits - 1) / splits) * f32g::BK;
  if (splits == 1) {
    p.C = dW; p.ldc = N; p.bias_grad = db;
    return db ? f32g::launch<f32g::XMAJ, f32g::XMAJ, EPI_F32, true>(p, 0, 1, s)
              : f32g::launch<f32g::XMAJ, f32g::XMAJ, EPI_F32, false>(p, 0, 1, s);
  }
  if (!ws) return hipErrorInvalidValue;
  p.C = ws; p.ldc = N; p.c_split_stride = (long long)M * N;
  float* bws = ws + (size_t)splits * M * N;
  p.bias_grad = bws; p.bg_split_stride = M;
  hipError_t e = db ? f32g::launch<f32g::XMAJ, f32g::XMAJ, EPI_F32, true>(p, 0, splits, s)
                    : f32g::launch<f32g::XMAJ, f32g::XMAJ, EPI_F32, false>(p, 0, splits, s);
  if (e != hipSuccess) return e;
  if (N % 4 != 0) return hipErrorInvalidValue;
  return splitk_reduce(ws, splits, (long long)M * N, M, N, dW, N, db ? bws : nullptr, M, db,
                       nullptr, 0, 0.f, nullptr, s);
}

}  // namespace nnmpi
