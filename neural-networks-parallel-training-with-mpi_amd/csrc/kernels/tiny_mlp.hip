// Whole training step of a tiny MLP in ONE launch (fp32, widths <= 16, <= 4 Linear layers).
//
// The reference config (2 -> 3 -> 1 ReLU regressor on 16 rows, ref.py:41-45,72) is pure launch
// overhead: every GEMM is far below one MFMA tile ("the tiny configs need a
// single-launch fused whole-MLP kernel").  One lane owns one row: forward through all layers,
// MSE / cross-entropy loss and gradient, and backward through all layers stay in registers.
// Parameter gradients are wave-reduced with shuffles and accumulated per wave in LDS in a fixed
// order, then the 4 wave slots are summed in order -> bitwise deterministic.  With one block the
// gradients are written straight into the arena; with more blocks each block writes an
// arena-shaped slab and the split-K reducer combines them in block order.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace nnmpi {

constexpr int TW = 16;
constexpr int TL = 4;

// Layer widths: FIX = 1 compiles the reference model (2 -> 3 -> 1, ref.py:41-45) in, so every
// `o < wout` / `i < win` test of the unrolled 16 x 16 loops folds away.  With runtime widths the
// kernel executes ~1,000 uniform compare-and-branch pairs per step whatever the model's size
// (16.9 us per step for the 2-3-1 model, profiles/r2s2_final_kstats_ref.csv).
template <int FIX>
__device__ __forceinline__ int tiny_w(const TinyMLPDesc& d, int l) {
  if constexpr (FIX == 1) {
    constexpr int w[TL + 1] = {2, 3, 1, 0, 0};
    return w[l];
  } else {
    return d.widths[l];
  }
}

template <int ACT, int LOSS, int FIX>
__global__ void __launch_bounds__(256) tiny_mlp_kernel(TinyMLPDesc d, const float* P,
                                                       const float* __restrict__ X,
                                                       const float* __restrict__ Y,
                                                       const int64_t* __restrict__ labels, int rows,
                                                       float inv_count, float* __restrict__ gout,
                                                       long long slab, int numel,
                                                       float* __restrict__ loss_part,
                                                       float loss_scale, float* __restrict__ loss_out,
                                                       SgdFuse sg) {
  extern __shared__ __attribute__((aligned(16))) float wsum[];  // [4][numel] + params [numel]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // the model's parameters are staged in LDS by one coalesced pass: every later weight read is
  // an LDS read instead of a dependent global round trip inside the unrolled layer loops
  const int pbase = d.w_off[d.n_layers - 1];
  float* PL = wsum + 4 * numel - pbase;      // PL[arena offset] for offsets in [pbase, +numel)
  for (int i = tid; i < 4 * numel; i += 256) wsum[i] = 0.f;
  for (int i = tid; i < numel; i += 256) PL[pbase + i] = P[pbase + i];
  __shared__ float red[4];
  __syncthreads();
  const int L = FIX == 1 ? 2 : d.n_layers;
  const int out_w = FIX == 1 ? 1 : d.widths[L];
  float wave_loss = 0.f;
  for (int base = blockIdx.x * 256; base < rows; base += gridDim.x * 256) {
    const int r = base + w * 64 + lane;
    const bool valid = r < rows;
    float a[TL + 1][TW];
#pragma unroll
    for (int k = 0; k < TW; ++k) a[0][k] = (valid && k < tiny_w<FIX>(d, 0)) ? X[(long long)r * tiny_w<FIX>(d, 0) + k] : 0.f;
    float outv[TW];
#pragma unroll
    for (int l = 0; l < TL; ++l) {
      if (l < L) {
        const int win = tiny_w<FIX>(d, l), wout = tiny_w<FIX>(d, l + 1);
        const float* W = PL + d.w_off[l];
        const float* B = PL + d.b_off[l];
#pragma unroll
        for (int o = 0; o < TW; ++o) {
          float z = 0.f;
          if (o < wout) {
            z = B[o];
#pragma unroll
            for (int i = 0; i < TW; ++i) if (i < win) z += W[o * win + i] * a[l][i];
          }
          a[l + 1][o] = (l < L - 1) ? act_fwd_t<ACT>(z) : z;
          if (l == L - 1) outv[o] = z;
        }
      } else {
#pragma unroll
        for (int o = 0; o < TW; ++o) a[l + 1][o] = 0.f;
      }
    }
    float delta[TW];
    float row_loss = 0.f;
    if constexpr (LOSS == LOSS_MSE) {
#pragma unroll
      for (int o = 0; o < TW; ++o) {
        float df = 0.f;
        if (o < out_w && valid) df = outv[o] - Y[(long long)r * out_w + o];
        row_loss += df * df;
        delta[o] = 2.f * df * inv_count;
      }
    } else {
      float mx = -INFINITY;
#pragma unroll
      for (int o = 0; o < TW; ++o) if (o < out_w) mx = fmaxf(mx, outv[o]);
      float se = 0.f;
#pragma unroll
      for (int o = 0; o < TW; ++o) if (o < out_w) se += __expf(outv[o] - mx);
      const float lse = mx + __logf(se);
      const int lab = valid ? (int)labels[r] : -1;
      float ll = 0.f;
#pragma unroll
      for (int o = 0; o < TW; ++o) {
        if (o == lab) ll = outv[o];
        delta[o] = (valid && o < out_w) ? (__expf(outv[o] - lse) - (o == lab ? 1.f : 0.f)) * inv_count : 0.f;
      }
      row_loss = valid ? lse - ll : 0.f;
    }
    wave_loss += row_loss;
    // backward, last layer first
#pragma unroll
    for (int l = TL - 1; l >= 0; --l) {
      if (l < L) {
        const int win = tiny_w<FIX>(d, l), wout = tiny_w<FIX>(d, l + 1);
        const float* W = PL + d.w_off[l];
        float* gw = wsum + w * numel + d.w_off[l] - d.w_off[L - 1];
        float* gb = wsum + w * numel + d.b_off[l] - d.w_off[L - 1];
#pragma unroll
        for (int o = 0; o < TW; ++o) {
          if (o < wout) {
#pragma unroll
            for (int i = 0; i < TW; ++i) {
              if (i < win) {
                const float c = wave_sum(delta[o] * a[l][i]);
                if (lane == 0) gw[o * win + i] += c;
              }
            }
            const float cb = wave_sum(delta[o]);
            if (lane == 0) gb[o] += cb;
          }
        }
        if (l > 0) {
          float dp[TW];
#pragma unroll
          for (int i = 0; i < TW; ++i) {
            float s = 0.f;
            if (i < win) {
#pragma unroll
              for (int o = 0; o < TW; ++o) if (o < wout) s += delta[o] * W[o * win + i];
              s *= act_bwd_t<ACT>(a[l][i]);
            }
            dp[i] = s;
          }
#pragma unroll
          for (int i = 0; i < TW; ++i) delta[i] = dp[i];
        }
      }
    }
  }
  __syncthreads();
  // arena region covered by this model starts at the last layer's W (reverse layout)
  float* dst = gout + (long long)blockIdx.x * slab;
  for (int i = tid; i < numel; i += 256) {
    const float g = ((wsum[i] + wsum[numel + i]) + wsum[2 * numel + i]) + wsum[3 * numel + i];
    // single block + single rank: the gradient is final -> optimizer update right here (every
    // read of the parameters happened before the barrier above); else store it
    if (sg.g_base) sgd_fused_store(sg, dst + i, g);
    else dst[i] = g;
  }
  wave_loss = wave_sum(wave_loss);  // lanes own different rows here
  if (lane == 0) red[w] = wave_loss;
  __syncthreads();
  if (tid == 0) {
    const float t = red[0] + red[1] + red[2] + red[3];
    loss_part[blockIdx.x] = t;
    if (loss_out) *loss_out = t * loss_scale;   // one block: no separate loss reduce
  }
}

static int tiny_blocks(int rows) { return std::max(1, std::min((rows + 255) / 256, 256)); }

size_t tiny_mlp_workspace_bytes(int rows, int arena_numel) {
  const int nb = tiny_blocks(rows);
  return (size_t)(nb > 1 ? nb * (size_t)arena_numel : 0) * sizeof(float) +
         (size_t)(((nb + 3) & ~3) + 4) * sizeof(float);
}

hipError_t tiny_mlp_step(const TinyMLPDesc& d, const float* params, const float* X,
                         const float* y, const int64_t* labels, int rows, float inv_count,
                         float* grad, int arena_numel, float* ws, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd, float loss_scale_in) {
  if (d.n_layers < 1 || d.n_layers > TL) return hipErrorInvalidValue;
  for (int l = 0; l <= d.n_layers; ++l)
    if (d.widths[l] < 1 || d.widths[l] > TW) return hipErrorInvalidValue;
  const int nb = tiny_blocks(rows);
  // the model occupies arena[w_off[L-1] .. arena_numel) (reverse layer order, W_{L-1} first)
  const int base = d.w_off[d.n_layers - 1];
  const int numel = arena_numel - base;
  const size_t smem = (size_t)5 * numel * sizeof(float);
  if (smem > 150 * 1024) return hipErrorInvalidValue;
  float* loss_part = ws;
  float* slabs = ws + ((nb + 3) & ~3) + 4;  // keep 16-byte alignment for the vector reducer
  float* gout = nb > 1 ? slabs : grad + base;
  const long long slab = nb > 1 ? numel : 0;
  const float loss_scale = loss_scale_in >= 0.f ? loss_scale_in
                           : d.loss == LOSS_XENT ? 1.f / rows : 1.f / ((float)rows * d.widths[d.n_layers]);
  // one block: loss written and (single rank) optimizer applied in-kernel -> ONE launch per step
  SgdFuse sg{};
  if (nb == 1 && sgd) sg = *sgd;
  float* lout = nb == 1 ? loss_out : nullptr;
#define TINY_LAUNCH(A, LS)                                                                   \
  hipLaunchKernelGGL((tiny_mlp_kernel<A, LS, 0>), dim3(nb), dim3(256), smem, s, d, params, X, y, \
                     labels, rows, inv_count, gout, slab, numel, loss_part, loss_scale, lout, sg)
  const bool ref_shape = d.n_layers == 2 && d.widths[0] == 2 && d.widths[1] == 3 && d.widths[2] == 1;
  if (ref_shape && d.loss == LOSS_MSE && d.act == ACT_RELU) {
    hipLaunchKernelGGL((tiny_mlp_kernel<ACT_RELU, LOSS_MSE, 1>), dim3(nb), dim3(256), smem, s, d,
                       params, X, y, labels, rows, inv_count, gout, slab, numel, loss_part,
                       loss_scale, lout, sg);
  } else if (d.loss == LOSS_XENT) {
    if (d.act == ACT_TANH) TINY_LAUNCH(ACT_TANH, LOSS_XENT);
    else TINY_LAUNCH(ACT_RELU, LOSS_XENT);
  } else {
    if (d.act == ACT_TANH) TINY_LAUNCH(ACT_TANH, LOSS_MSE);
    else TINY_LAUNCH(ACT_RELU, LOSS_MSE);
  }
#undef TINY_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (nb > 1) {
    if (sgd) return hipErrorInvalidValue;   // the optimizer fusion needs the single-block form
    return splitk_reduce(slabs, nb, numel, 1, numel, grad + base, numel, nullptr, 0, nullptr,
                         loss_part, nb, loss_scale, loss_out, s);
  }
  return hipSuccess;
}

bool tiny_mlp_can_fuse_sgd(int rows) { return tiny_blocks(rows) == 1; }

}  // namespace nnmpi
