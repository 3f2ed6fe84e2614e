// Output layer + loss, forward AND backward, for skinny heads (out <= 16).
//
// Replaces reference ops K3-K8 (ref.py:44,94,173,176): the last Linear (N = out is 1 for the
// regressor, 10 for MNIST-shape classification — far below one MFMA tile), MSELoss / softmax
// cross-entropy and their gradients, and the first dgrad of the backward pass.  One wave per row:
// the row's activations are read once with 16-byte loads, the logits are wave-reduced, the loss
// and dlogits are computed in registers, and dZ_prev = (dlogits . W) * act'(a) is written in the
// same pass.  The head's weight gradient (a GEMV over the batch) runs as a separate skinny
// kernel writing deterministic per-split partials that one reduce combines (fixed order).
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace nnmpi {

constexpr int HEAD_OMAX = 16;

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

template <typename TA, int CMAX, int LOSS, int ACT>
__global__ void __launch_bounds__(256) head_fwd_kernel(HeadArgs p) {
  extern __shared__ __attribute__((aligned(16))) float wl[];  // [out][in]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nW = p.out * p.in;
  for (int i = tid * 4; i < nW; i += 256 * 4)
    *reinterpret_cast<float4*>(wl + i) = *reinterpret_cast<const float4*>(p.W + i);
  __shared__ float red[4];
  __syncthreads();

  const int nch = p.in >> 3;
  const TA* A = reinterpret_cast<const TA*>(p.a);
  TA* DZ = reinterpret_cast<TA*>(p.dz_prev);
  float wave_loss = 0.f;
  for (int r = blockIdx.x * 4 + w; r < p.rows; r += gridDim.x * 4) {
    float av[CMAX][8];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      const int ch = c * 64 + lane;
      if (ch < nch) load8<TA>(A + (long long)r * p.in + ch * 8, av[c]);
      else {
#pragma unroll
        for (int e = 0; e < 8; ++e) av[c][e] = 0.f;
      }
    }
    float lg[HEAD_OMAX];
#pragma unroll
    for (int o = 0; o < HEAD_OMAX; ++o) {
      float s = 0.f;
      if (o < p.out) {
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
          const int ch = c * 64 + lane;
          if (ch < nch) {
            const float* wr = wl + o * p.in + ch * 8;
#pragma unroll
            for (int e = 0; e < 8; ++e) s += av[c][e] * wr[e];
          }
        }
        s = wave_sum(s) + p.b[o];
      }
      lg[o] = s;
    }
    float dl[HEAD_OMAX];
    float row_loss = 0.f;
    if constexpr (LOSS == LOSS_MSE) {
#pragma unroll
      for (int o = 0; o < HEAD_OMAX; ++o) {
        float d = 0.f;
        if (o < p.out) d = lg[o] - p.y[(long long)r * p.out + o];
        row_loss += d * d;
        dl[o] = 2.f * d * p.inv_count;
      }
    } else {
      float mx = -INFINITY;
#pragma unroll
      for (int o = 0; o < HEAD_OMAX; ++o) if (o < p.out) mx = fmaxf(mx, lg[o]);
      float se = 0.f;
#pragma unroll
      for (int o = 0; o < HEAD_OMAX; ++o) if (o < p.out) se += __expf(lg[o] - mx);
      const float lse = mx + __logf(se);
      const int lab = (int)p.labels[r];
      float lgl = 0.f;
#pragma unroll
      for (int o = 0; o < HEAD_OMAX; ++o) {
        if (o == lab) lgl = lg[o];
        dl[o] = (o < p.out) ? (__expf(lg[o] - lse) - (o == lab ? 1.f : 0.f)) * p.inv_count : 0.f;
      }
      row_loss = lse - lgl;
    }
    wave_loss += row_loss;
    float myd = 0.f;
#pragma unroll
    for (int o = 0; o < HEAD_OMAX; ++o) if (lane == o) myd = dl[o];
    if (lane < p.out) p.dlogits[(long long)r * p.out + lane] = myd;
    if (DZ != nullptr) {
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        const int ch = c * 64 + lane;
        if (ch < nch) {
          float g[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
          for (int o = 0; o < HEAD_OMAX; ++o) {
            if (o < p.out) {
              const float* wr = wl + o * p.in + ch * 8;
#pragma unroll
              for (int e = 0; e < 8; ++e) g[e] += dl[o] * wr[e];
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] *= act_bwd_t<ACT>(av[c][e]);
          store8<TA>(DZ + (long long)r * p.in + ch * 8, g);
        }
      }
    }
  }
  if (lane == 0) red[w] = wave_loss;
  __syncthreads();
  if (tid == 0) p.loss_part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int head_fwd_parts(int rows) { return std::max(1, std::min((rows + 3) / 4, 1024)); }

template <typename TA, int CMAX, int LOSS>
static hipError_t head_launch_act(const HeadArgs& a, int act, int blocks, size_t smem, hipStream_t s) {
  switch (act) {
    case ACT_RELU:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_RELU>), dim3(blocks), dim3(256), smem, s, a);
      break;
    case ACT_TANH:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_TANH>), dim3(blocks), dim3(256), smem, s, a);
      break;
    default:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_NONE>), dim3(blocks), dim3(256), smem, s, a);
  }
  return hipGetLastError();
}

template <typename TA, int LOSS>
static hipError_t head_launch_c(const HeadArgs& a, int act, int blocks, size_t smem, hipStream_t s) {
  const int nch = a.in / 8;
  if (nch <= 64) return head_launch_act<TA, 1, LOSS>(a, act, blocks, smem, s);
  if (nch <= 128) return head_launch_act<TA, 2, LOSS>(a, act, blocks, smem, s);
  if (nch <= 256) return head_launch_act<TA, 4, LOSS>(a, act, blocks, smem, s);
  if (nch <= 1024) return head_launch_act<TA, 16, LOSS>(a, act, blocks, smem, s);
  return hipErrorInvalidValue;
}

hipError_t head_fwd(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                    int out, const float* y, const int64_t* labels, int loss, float inv_count,
                    int act_prev, void* dz_prev, float* dlogits, float* loss_part, hipStream_t s) {
  if (out < 1 || out > HEAD_OMAX || in % 8 != 0 || in > 8192) return hipErrorInvalidValue;
  const size_t smem = (size_t)out * in * sizeof(float);
  if (smem > 65536) return hipErrorInvalidValue;
  HeadArgs h{a, rows, in, W, b, out, y, labels, inv_count, act_prev, dz_prev, dlogits, loss_part};
  const int blocks = head_fwd_parts(rows);
  if (a_bf16) {
    return loss == LOSS_XENT ? head_launch_c<bf16, LOSS_XENT>(h, act_prev, blocks, smem, s)
                             : head_launch_c<bf16, LOSS_MSE>(h, act_prev, blocks, smem, s);
  }
  return loss == LOSS_XENT ? head_launch_c<float, LOSS_XENT>(h, act_prev, blocks, smem, s)
                           : head_launch_c<float, LOSS_MSE>(h, act_prev, blocks, smem, s);
}

// ---- head weight gradient: gW[o][i] = sum_r dl[r][o] a[r][i], gb[o] = sum_r dl[r][o] ----
template <typename TA, int OMAX>
__global__ void __launch_bounds__(64) head_wgrad_kernel(const TA* __restrict__ a, int rows, int in,
                                                        const float* __restrict__ dl, int out,
                                                        int rows_per_split, float* __restrict__ ws,
                                                        float* __restrict__ wsb) {
  const int lane = threadIdx.x;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int split = blockIdx.y;
  const int r0 = split * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float acc[OMAX][8];
  float accb[OMAX];
#pragma unroll
  for (int o = 0; o < OMAX; ++o) {
    accb[o] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
  }
  const bool active = c0 < in;
  for (int r = r0; r < r1; ++r) {
    float av[8];
    if (active) load8<TA>(a + (long long)r * in + c0, av);
#pragma unroll
    for (int o = 0; o < OMAX; ++o) {
      if (o < out) {
        const float d = dl[(long long)r * out + o];
        accb[o] += d;
        if (active) {
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[o][e] += d * av[e];
        }
      }
    }
  }
  if (active) {
#pragma unroll
    for (int o = 0; o < OMAX; ++o) {
      if (o < out) {
        float* dst = ws + ((long long)split * out + o) * in + c0;
        *reinterpret_cast<float4*>(dst) = make_float4(acc[o][0], acc[o][1], acc[o][2], acc[o][3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[o][4], acc[o][5], acc[o][6], acc[o][7]);
      }
    }
  }
  if (blockIdx.x == 0 && lane == 0) {
#pragma unroll
    for (int o = 0; o < OMAX; ++o) if (o < out) wsb[(long long)split * out + o] = accb[o];
  }
}

static int head_splits(int rows, int in) {
  const int gx = (in + 511) / 512;
  int s = std::max(1, 512 / gx);
  s = std::min(s, std::max(1, rows / 16));
  return s;
}

size_t head_wgrad_workspace_bytes(int rows, int in, int out) {
  const int s = head_splits(rows, in);
  return (size_t)s * ((size_t)out * in + out) * sizeof(float);
}

hipError_t head_wgrad(const void* a, int a_bf16, int rows, int in, const float* dlogits, int out,
                      float* gW, float* gb, float* ws, const float* loss_part, int n_loss_part,
                      float loss_scale, float* loss_out, hipStream_t s) {
  if (out < 1 || out > HEAD_OMAX || in % 8 != 0) return hipErrorInvalidValue;
  const int S = head_splits(rows, in);
  const int rps = (rows + S - 1) / S;
  float* wsb = ws + (size_t)S * out * in;
  dim3 grid((in + 511) / 512, S);
  if (a_bf16) {
    const bf16* A = reinterpret_cast<const bf16*>(a);
    if (out == 1) hipLaunchKernelGGL((head_wgrad_kernel<bf16, 1>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
    else if (out <= 4) hipLaunchKernelGGL((head_wgrad_kernel<bf16, 4>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
    else hipLaunchKernelGGL((head_wgrad_kernel<bf16, 16>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
  } else {
    const float* A = reinterpret_cast<const float*>(a);
    if (out == 1) hipLaunchKernelGGL((head_wgrad_kernel<float, 1>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
    else if (out <= 4) hipLaunchKernelGGL((head_wgrad_kernel<float, 4>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
    else hipLaunchKernelGGL((head_wgrad_kernel<float, 16>), grid, dim3(64), 0, s, A, rows, in, dlogits, out, rps, ws, wsb);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return splitk_reduce(ws, S, (long long)out * in, out, in, gW, in, wsb, out, gb, loss_part,
                       n_loss_part, loss_scale, loss_out, s);
}

}  // namespace nnmpi
