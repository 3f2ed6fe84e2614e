// Output layer + loss for heads of ANY shape (the reference's last Linear generalised: ref.py:44,
// MSELoss / softmax cross-entropy ref.py:94,173,176) -- the path for heads the skinny head.hip
// kernels do not take (out > 16, or an fp32 weight image over 64 KiB of LDS: e.g. 8192 -> 10
// cross-entropy, 8192 -> 3 regression, 1024 -> 100 classes).
//
// bf16 activations with in % 256 == 0 and out <= 128 take the matrix-core path of head.hip
// (head_general_mfma); everything else runs the four fp32 VALU launches below (fixed summation
// order, deterministic):
//   1. logits[r][o] = b[o] + sum_k a[r][k] W[o][k]          64x64 register-tiled SGEMM (LDS, K
//                                                             chunks of 32, 4x4 outputs/thread)
//   2. per row: loss, dl = dL/dlogits * inv_count (in place) one wave per row, any width
//   3. dZ[r][k] = (sum_o dl[r][o] W[o][k]) * act'(a[r][k])   64x64 tiles over (rows, features)
//   4. gW partials over row splits (+ gb, loss) -> a reducer that sums them in split order
// The weights stay the fp32 master (as in the skinny head), activations bf16 or fp32.
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace nnmpi {

constexpr int HG_T = 64;       // output tile edge
constexpr int HG_KC = 32;      // K chunk staged in LDS
constexpr int HG_THREADS = 256;
constexpr int HG_LOSS_ROWS = 4;   // rows (= waves) per loss block

template <typename TA>
__device__ __forceinline__ float ld_act(const TA* p) {
  return static_cast<float>(*p);
}

// C[m][n] = sum_k A(m,k) * B(n,k), A(m,k) = A[m*lda + k], B(n,k) = B[n*ldb + k]; 64x64 tile.
// Every output accumulates k = 0..K-1 in order.
template <typename TA, typename TB>
__device__ __forceinline__ void tile_nt(const TA* __restrict__ A, int lda, int M, const TB* __restrict__ B,
                                        int ldb, int N, int K, int m0, int n0, float (&acc)[4][4],
                                        float (*As)[HG_T + 1], float (*Bs)[HG_T + 1]) {
  const int t = threadIdx.x, tm = t % 16, tn = t / 16;
  for (int k0 = 0; k0 < K; k0 += HG_KC) {
    // stage A[m0..+64][k0..+32] and B[n0..+64][k0..+32] transposed ([k][m]) into LDS
    for (int i = t; i < HG_T * HG_KC; i += HG_THREADS) {
      const int r = i / HG_KC, k = i % HG_KC;
      const int gm = m0 + r, gn = n0 + r, gk = k0 + k;
      As[k][r] = (gm < M && gk < K) ? ld_act(A + (long long)gm * lda + gk) : 0.f;
      Bs[k][r] = (gn < N && gk < K) ? static_cast<float>(B[(long long)gn * ldb + gk]) : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < HG_KC; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[k][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[k][tn + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
}

template <typename TA>
__global__ void __launch_bounds__(HG_THREADS) hg_logits_kernel(const TA* __restrict__ a, int rows, int in,
                                                                const float* __restrict__ W,
                                                                const float* __restrict__ b, int out,
                                                                float* __restrict__ logits) {
  __shared__ float As[HG_KC][HG_T + 1], Bs[HG_KC][HG_T + 1];
  const int m0 = blockIdx.x * HG_T, n0 = blockIdx.y * HG_T;
  float acc[4][4] = {};
  tile_nt(a, in, rows, W, in, out, in, m0, n0, acc, As, Bs);
  const int tm = threadIdx.x % 16, tn = threadIdx.x / 16;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = m0 + tm + 16 * i, o = n0 + tn + 16 * j;
      if (r < rows && o < out) logits[(long long)r * out + o] = acc[i][j] + b[o];
    }
}

// One wave per row.  MSE: loss = sum_o (z - y)^2, dl = 2 (z - y) inv_count.  Cross-entropy:
// loss = lse - z[label], dl = (softmax - onehot) inv_count.  dl overwrites the logits.
template <int LOSS>
__global__ void __launch_bounds__(64 * HG_LOSS_ROWS) hg_loss_kernel(float* __restrict__ z, int rows, int out,
                                                                     const float* __restrict__ y,
                                                                     const int64_t* __restrict__ labels,
                                                                     float inv_count,
                                                                     float* __restrict__ part) {
  __shared__ float wl[HG_LOSS_ROWS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x * HG_LOSS_ROWS + w;
  float loss = 0.f;
  if (r < rows) {
    float* zr = z + (long long)r * out;
    if constexpr (LOSS == LOSS_MSE) {
      const float* yr = y + (long long)r * out;
      for (int o = lane; o < out; o += 64) {
        const float d = zr[o] - yr[o];
        loss += d * d;
        zr[o] = 2.f * d * inv_count;
      }
      loss = wave_sum(loss);
    } else {
      float m = -INFINITY;
      for (int o = lane; o < out; o += 64) m = fmaxf(m, zr[o]);
      m = wave_max(m);
      const int lab = (int)labels[r];
      float s = 0.f, zlp = 0.f;
      for (int o = lane; o < out; o += 64) {
        const float v = zr[o];
        s += expf(v - m);
        zlp += (o == lab) ? v : 0.f;
      }
      s = wave_sum(s);
      const float zl = wave_sum(zlp);   // the label's logit, gathered before any rewrite
      const float lse = m + logf(s);
      for (int o = lane; o < out; o += 64) {
        const float p = expf(zr[o] - lse);
        zr[o] = (p - (o == lab ? 1.f : 0.f)) * inv_count;
      }
      loss = lse - zl;
    }
  }
  if (lane == 0) wl[w] = loss;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < HG_LOSS_ROWS; ++i) t += wl[i];
    part[blockIdx.x] = t;
  }
}

// dZ[r][k] = (sum_o dl[r][o] W[o][k]) * act'(a[r][k]): C = dl (rows x out) . W (out x in)
template <typename TA, int ACT>
__global__ void __launch_bounds__(HG_THREADS) hg_dz_kernel(const float* __restrict__ dl, int rows, int out,
                                                            const float* __restrict__ W, int in,
                                                            const TA* __restrict__ a, TA* __restrict__ dz) {
  __shared__ float As[HG_KC][HG_T + 1], Bs[HG_KC][HG_T + 1];
  const int m0 = blockIdx.x * HG_T, n0 = blockIdx.y * HG_T;
  const int t = threadIdx.x, tm = t % 16, tn = t / 16;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < out; k0 += HG_KC) {
    for (int i = t; i < HG_T * HG_KC; i += HG_THREADS) {
      // A(m,k) = dl[m][k] (k = output index), B(n,k) = W[k][n] (n = feature)
      const int r = i / HG_KC, k = i % HG_KC;
      const int gm = m0 + r, gk = k0 + k;
      As[k][r] = (gm < rows && gk < out) ? dl[(long long)gm * out + gk] : 0.f;
      const int kk = i / HG_T, nn = i % HG_T;
      const int gk2 = k0 + kk, gn = n0 + nn;
      Bs[kk][nn] = (gk2 < out && gn < in) ? W[(long long)gk2 * in + gn] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < HG_KC; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[k][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[k][tn + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = m0 + tm + 16 * i, c = n0 + tn + 16 * j;
      if (r < rows && c < in) {
        const long long idx = (long long)r * in + c;
        dz[idx] = static_cast<TA>(acc[i][j] * act_bwd_t<ACT>(ld_act(a + idx)));
      }
    }
}

// gW partial of one row split: P[s][o][k] = sum_{r in split s} dl[r][o] a[r][k]; the k-tile-0
// blocks also write gb partials sum_r dl[r][o].
template <typename TA>
__global__ void __launch_bounds__(HG_THREADS) hg_wgrad_kernel(const float* __restrict__ dl, int rows, int out,
                                                               const TA* __restrict__ a, int in,
                                                               int rows_per_split,
                                                               float* __restrict__ pw,
                                                               float* __restrict__ pb) {
  __shared__ float As[HG_KC][HG_T + 1], Bs[HG_KC][HG_T + 1];
  const int m0 = blockIdx.x * HG_T, n0 = blockIdx.y * HG_T, s = blockIdx.z;
  const int r0 = s * rows_per_split, r1 = min(rows, r0 + rows_per_split);
  const int t = threadIdx.x, tm = t % 16, tn = t / 16;
  float acc[4][4] = {};
  float bacc[4] = {};
  for (int k0 = r0; k0 < r1; k0 += HG_KC) {
    for (int i = t; i < HG_T * HG_KC; i += HG_THREADS) {
      // A(m,k) = dl[k][m] (m = output), B(n,k) = a[k][n] (n = feature); rows are contiguous in m/n
      const int kk = i / HG_T, x = i % HG_T;
      const int gk = k0 + kk;
      As[kk][x] = (gk < r1 && m0 + x < out) ? dl[(long long)gk * out + m0 + x] : 0.f;
      Bs[kk][x] = (gk < r1 && n0 + x < in) ? ld_act(a + (long long)gk * in + n0 + x) : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int k = 0; k < HG_KC; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[k][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[k][tn + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
        if (blockIdx.y == 0 && tn == 0) bacc[i] += av[i];
      }
    }
    __syncthreads();
  }
  const long long plane = (long long)out * in;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = m0 + tm + 16 * i;
    if (o >= out) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = n0 + tn + 16 * j;
      if (c < in) pw[s * plane + (long long)o * in + c] = acc[i][j];
    }
    if (blockIdx.y == 0 && tn == 0) pb[(long long)s * out + o] = bacc[i];
  }
}

// gW = sum_s P[s], gb = sum_s pb[s] (split order); block 0 also folds the loss partials.
__global__ void __launch_bounds__(256) hg_reduce_kernel(const float* __restrict__ pw, const float* __restrict__ pb,
                                                         int S, int out, int in, float* __restrict__ gW,
                                                         float* __restrict__ gb, const float* __restrict__ lpart,
                                                         int nl, float loss_scale,
                                                         float* __restrict__ loss_out) {
  const long long plane = (long long)out * in;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < plane + out;
       i += (long long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    if (i < plane) {
      for (int s = 0; s < S; ++s) acc += pw[s * plane + i];
      gW[i] = acc;
    } else {
      const int o = (int)(i - plane);
      for (int s = 0; s < S; ++s) acc += pb[(long long)s * out + o];
      gb[o] = acc;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < nl; ++i) t += lpart[i];
    loss_out[0] = t * loss_scale;
  }
}

static int hg_splits(int rows, int out, int in) {
  const int tiles = ((out + HG_T - 1) / HG_T) * ((in + HG_T - 1) / HG_T);
  int s = std::max(1, std::min(32, 1024 / std::max(tiles, 1)));
  s = std::min(s, std::max(1, rows / HG_KC));
  return s;
}

static int hg_loss_blocks(int rows) { return (rows + HG_LOSS_ROWS - 1) / HG_LOSS_ROWS; }

// 1: bf16 heads also take the VALU path below instead of head.hip's matrix-core path (A/B)
static int g_head_general_valu = 0;
void set_head_general_valu(int on) { g_head_general_valu = on; }

// workspace: logits/dl [rows*out] | loss partials | gW partials [S*out*in] | gb partials [S*out]
size_t head_general_workspace_bytes(int rows, int in, int out) {
  const int S = hg_splits(rows, out, in);
  const size_t n = (size_t)rows * out + hg_loss_blocks(rows) + 64 + (size_t)S * out * in +
                   (size_t)S * out + 64;
  // (either path: the matrix-core path of head.hip for bf16 activations, this one otherwise)
  return std::max(n * sizeof(float),
                  head_general_mfma_ok(1, in, out) ? head_general_mfma_workspace_bytes(rows, in, out)
                                                   : (size_t)0);
}

hipError_t head_general(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                        int out, const float* y, const int64_t* labels, int loss, float inv_count,
                        int act_prev, void* dz_out, float* gW, float* gb, float* dlogits_out,
                        float* ws, float loss_scale, float* loss_out, hipStream_t s) {
  if (rows <= 0 || in <= 0 || out <= 0) return hipErrorInvalidValue;
  if (head_general_mfma_ok(a_bf16, in, out) && !g_head_general_valu)
    return head_general_mfma(static_cast<const bf16*>(a), rows, in, W, b, out, y, labels, loss,
                             inv_count, act_prev, static_cast<bf16*>(dz_out), gW, gb, dlogits_out,
                             ws, loss_scale, loss_out, s);
  const int S = hg_splits(rows, out, in);
  const int nl = hg_loss_blocks(rows);
  float* z = ws;
  float* lpart = z + (size_t)rows * out;
  float* pw = lpart + nl + 64;
  float* pb = pw + (size_t)S * out * in;
  const dim3 blk(HG_THREADS);
  const dim3 g_lo((rows + HG_T - 1) / HG_T, (out + HG_T - 1) / HG_T);
  if (a_bf16)
    hipLaunchKernelGGL(hg_logits_kernel<bf16>, g_lo, blk, 0, s, (const bf16*)a, rows, in, W, b, out, z);
  else
    hipLaunchKernelGGL(hg_logits_kernel<float>, g_lo, blk, 0, s, (const float*)a, rows, in, W, b, out, z);
  if (loss == LOSS_MSE)
    hipLaunchKernelGGL(hg_loss_kernel<LOSS_MSE>, dim3(nl), dim3(64 * HG_LOSS_ROWS), 0, s, z, rows, out, y,
                       labels, inv_count, lpart);
  else
    hipLaunchKernelGGL(hg_loss_kernel<LOSS_XENT>, dim3(nl), dim3(64 * HG_LOSS_ROWS), 0, s, z, rows, out, y,
                       labels, inv_count, lpart);
  if (dz_out) {
    const dim3 g_dz((rows + HG_T - 1) / HG_T, (in + HG_T - 1) / HG_T);
#define HG_DZ(TA, ACT)                                                                             \
  hipLaunchKernelGGL((hg_dz_kernel<TA, ACT>), g_dz, blk, 0, s, z, rows, out, W, in, (const TA*)a, \
                     (TA*)dz_out)
    if (a_bf16) {
      if (act_prev == ACT_RELU) HG_DZ(bf16, ACT_RELU);
      else if (act_prev == ACT_TANH) HG_DZ(bf16, ACT_TANH);
      else HG_DZ(bf16, ACT_NONE);
    } else {
      if (act_prev == ACT_RELU) HG_DZ(float, ACT_RELU);
      else if (act_prev == ACT_TANH) HG_DZ(float, ACT_TANH);
      else HG_DZ(float, ACT_NONE);
    }
#undef HG_DZ
  }
  const int rps = (rows + S - 1) / S;
  const dim3 g_wg((out + HG_T - 1) / HG_T, (in + HG_T - 1) / HG_T, S);
  if (a_bf16)
    hipLaunchKernelGGL(hg_wgrad_kernel<bf16>, g_wg, blk, 0, s, z, rows, out, (const bf16*)a, in, rps, pw, pb);
  else
    hipLaunchKernelGGL(hg_wgrad_kernel<float>, g_wg, blk, 0, s, z, rows, out, (const float*)a, in, rps, pw,
                       pb);
  const long long n = (long long)out * in + out;
  const int rb = (int)std::min<long long>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(hg_reduce_kernel, dim3(std::max(rb, 1)), dim3(256), 0, s, pw, pb, S, out, in, gW, gb,
                     lpart, nl, loss_scale, loss_out);
  if (dlogits_out) {
    hipError_t e = hipMemcpyAsync(dlogits_out, z, (size_t)rows * out * sizeof(float),
                                  hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

}  // namespace nnmpi
