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
#include "head_common.h"

#include <algorithm>

namespace nnmpi {

static int g_head_xcd_rows = 0;
void set_head_xcd_rows(int v) { g_head_xcd_rows = v; }


// One wave per row, RPW rows per wave-iteration (their loads, targets and the RPW x OUTM
// butterfly reductions are all issued together, so no shuffle or load latency is exposed per
// row).  With FUSE (out == 1 heads) the head weights live in registers and each lane also
// accumulates the head's weight/bias gradient for its own 8*CMAX columns across all rows it
// visits; the waves are combined through LDS in wave order and every block writes one partial
// slab (gW [in], gb, loss) for the deterministic reducer.  All per-element conditions are
// expressed as predicates/clamps (no branches around loads or shuffles).
//
// HW waves per block: 16 / 8 for rows of <= 512 / 1024 features (a few rows per wave keep several
// waves on every SIMD, so the row loads of the whole chip are in flight at once), 4 for wider rows
// (their per-lane register footprint only fits at low occupancy).
template <typename TA, int CMAX, int LOSS, int ACT, bool FUSE, int RPW, int OUTM, int HW>
__global__ void __launch_bounds__(64 * HW) head_fwd_kernel(HeadArgs p, float* __restrict__ wslab,
                                                           float* __restrict__ bslab) {
  // W image [out][2][in/8][4]: element (o, k = 8c + 4h + j) at o*in + h*(in/2) + 4c + j, so the
  // 64 lanes of a wave, each owning the 8 consecutive columns of chunk c, read one half h as ONE
  // 16-byte word at consecutive addresses (the plain [out][in] image put lanes 32 B apart:
  // 8-way bank conflicts on every weight read, 58.7M of 70.3M LDS cycles of the MNIST head)
  extern __shared__ __attribute__((aligned(16))) float wl[];  // W image (+ [HW][in] if FUSE)
  constexpr int NT = 64 * HW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nW = p.out * p.in;
  const int nch8 = p.in >> 3;
  for (int i = tid; i < nW; i += NT) {
    const int o = i / p.in, k = i - o * p.in;
    wl[o * p.in + ((k >> 2) & 1) * (nch8 * 4) + (k >> 3) * 4 + (k & 3)] = p.W[i];
  }
  __shared__ float red[HW][2];
  __syncthreads();

  const int nch = p.in >> 3;
  const TA* A = reinterpret_cast<const TA*>(p.a);
  TA* DZ = reinterpret_cast<TA*>(p.dz_prev);
  const int nout = FUSE ? 1 : p.out;
  float wave_loss = 0.f;
  float gacc[CMAX][8];
  float gbacc = 0.f;
  // per-lane column validity as multiplicative masks; the chunk index is clamped for loads
  float cmask[CMAX];
  int chc[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) {
    const int ch = c * 64 + lane;
    cmask[c] = ch < nch ? 1.f : 0.f;
    chc[c] = min(ch, nch - 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) gacc[c][e] = 0.f;
  }
  // FUSE: the single output row of W in registers (masked)
  float wreg[FUSE ? CMAX : 1][8];
  if constexpr (FUSE) {
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
#pragma unroll
      for (int e = 0; e < 8; ++e) wreg[c][e] = wl[(e >> 2) * (nch8 * 4) + chc[c] * 4 + (e & 3)] * cmask[c];
  }
  float bias[OUTM];
#pragma unroll
  for (int o = 0; o < OUTM; ++o) bias[o] = p.b[min(o, nout - 1)];

  // rows of an XCD-contiguous logical block: the forward GEMM left these rows' activations in
  // the L2 of the XCD this block runs on (its tiles use the same xcd_remap), and the backward
  // launches read this block's dZ rows from there too
  const int lb = p.xcd_rows ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int gw = lb * HW + w, nwaves = gridDim.x * HW;
  for (int r0 = gw * RPW; r0 < p.rows; r0 += nwaves * RPW) {
    // Multi-output heads read W from LDS for every row: an offset the compiler cannot see
    // through keeps it from hoisting all OUTM x CMAX x 8 weights into registers across the row
    // loop (256 VGPRs + 128 spilled for out = 10, in = 1024 -> 135 us; PMC/resource-usage).
    int wo = 0;
    if constexpr (!FUSE) asm volatile("" : "+v"(wo));
    const float* wlo = wl + wo;
    float av[RPW][CMAX][8];
    float yv[RPW][OUTM];
    int labv[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int r = min(r0 + q, p.rows - 1);   // clamped: loads stay unconditional
#pragma unroll
      for (int c = 0; c < CMAX; ++c) load8<TA>(A + (long long)r * p.in + chc[c] * 8, av[q][c]);
      if constexpr (LOSS == LOSS_MSE) {
#pragma unroll
        for (int o = 0; o < OUTM; ++o) yv[q][o] = p.y[(long long)r * nout + min(o, nout - 1)];
      } else {
        labv[q] = (int)p.labels[r];
      }
    }
    // partial dot products for every (row, output), then one batched butterfly
    float part[RPW][OUTM];
#pragma unroll
    for (int q = 0; q < RPW; ++q)
#pragma unroll
      for (int o = 0; o < OUTM; ++o) {
        float sacc = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
          if constexpr (FUSE) {
#pragma unroll
            for (int e = 0; e < 8; ++e) sacc += av[q][c][e] * wreg[c][e];
          } else {
            if (o >= nout) continue;   // uniform: no work for the padding outputs
            const float* wr = wlo + o * p.in + chc[c] * 4;
            const float4 w0 = *reinterpret_cast<const float4*>(wr);
            const float4 w1 = *reinterpret_cast<const float4*>(wr + nch8 * 4);
            const float t = av[q][c][0] * w0.x + av[q][c][1] * w0.y + av[q][c][2] * w0.z +
                            av[q][c][3] * w0.w + av[q][c][4] * w1.x + av[q][c][5] * w1.y +
                            av[q][c][6] * w1.z + av[q][c][7] * w1.w;
            sacc += t * cmask[c];
          }
        }
        part[q][o] = sacc;
      }
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1)
#pragma unroll
      for (int q = 0; q < RPW; ++q)
#pragma unroll
        for (int o = 0; o < OUTM; ++o)
          if (o < nout) part[q][o] += __shfl_xor(part[q][o], sh, 64);

#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const bool valid = (r0 + q) < p.rows;
      const int r = valid ? r0 + q : p.rows - 1;
      float lg[OUTM];
#pragma unroll
      for (int o = 0; o < OUTM; ++o) lg[o] = part[q][o] + bias[o];
      float dl[OUTM];
      float row_loss = 0.f;
      if constexpr (LOSS == LOSS_MSE) {
#pragma unroll
        for (int o = 0; o < OUTM; ++o) {
          const float d = (o < nout) ? lg[o] - yv[q][o] : 0.f;
          row_loss += d * d;
          dl[o] = 2.f * d * p.inv_count;
        }
      } else {
        float mx = -INFINITY;
#pragma unroll
        for (int o = 0; o < OUTM; ++o) if (o < nout) mx = fmaxf(mx, lg[o]);
        float se = 0.f;
#pragma unroll
        for (int o = 0; o < OUTM; ++o) if (o < nout) se += __expf(lg[o] - mx);
        const float lse = mx + __logf(se);
        const int lab = labv[q];
        float lgl = 0.f;
#pragma unroll
        for (int o = 0; o < OUTM; ++o) {
          if (o == lab) lgl = lg[o];
          dl[o] = (o < nout) ? (__expf(lg[o] - lse) - (o == lab ? 1.f : 0.f)) * p.inv_count : 0.f;
        }
        row_loss = lse - lgl;
      }
      if (!valid) {
        row_loss = 0.f;
#pragma unroll
        for (int o = 0; o < OUTM; ++o) dl[o] = 0.f;
      }
      wave_loss += row_loss;
      if constexpr (FUSE) {
        gbacc += dl[0];
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
#pragma unroll
          for (int e = 0; e < 8; ++e) gacc[c][e] += dl[0] * av[q][c][e];
      } else {
        float myd = 0.f;
#pragma unroll
        for (int o = 0; o < OUTM; ++o) if (lane == o) myd = dl[o];
        if (valid && lane < nout) p.dlogits[(long long)r * nout + lane] = myd;
      }
      if (DZ != nullptr) {
#pragma unroll
        for (int c = 0; c < CMAX; ++c) {
          float g[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
          for (int o = 0; o < OUTM; ++o) {
            if constexpr (FUSE) {
#pragma unroll
              for (int e = 0; e < 8; ++e) g[e] += dl[o] * wreg[c][e];
            } else {
              if (o >= nout) continue;
              const float* wr = wlo + o * p.in + chc[c] * 4;
              const float4 w0 = *reinterpret_cast<const float4*>(wr);
              const float4 w1 = *reinterpret_cast<const float4*>(wr + nch8 * 4);
              g[0] += dl[o] * w0.x; g[1] += dl[o] * w0.y; g[2] += dl[o] * w0.z; g[3] += dl[o] * w0.w;
              g[4] += dl[o] * w1.x; g[5] += dl[o] * w1.y; g[6] += dl[o] * w1.z; g[7] += dl[o] * w1.w;
            }
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] *= act_bwd_t<ACT>(av[q][c][e]);
          if (valid && cmask[c] != 0.f) store8<TA>(DZ + (long long)r * p.in + chc[c] * 8, g);
        }
      }
    }
  }
  if (lane == 0) {
    red[w][0] = wave_loss;
    red[w][1] = gbacc;
  }
  if constexpr (FUSE) {
    // every wave parks its column partials in its own LDS row (16-B stores), then each thread
    // sums one column over the waves in wave order (one barrier, no serial wave rounds)
    float* gl = wl + nW;   // [HW][in]
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      if (cmask[c] != 0.f) {
        float* d = gl + w * p.in + chc[c] * 8;
        *reinterpret_cast<float4*>(d) = make_float4(gacc[c][0], gacc[c][1], gacc[c][2], gacc[c][3]);
        *reinterpret_cast<float4*>(d + 4) = make_float4(gacc[c][4], gacc[c][5], gacc[c][6], gacc[c][7]);
      }
    }
    __syncthreads();
    float* dst = wslab + (long long)blockIdx.x * p.in;
    for (int i = tid; i < p.in; i += NT) {
      float t = gl[i];
#pragma unroll
      for (int k = 1; k < HW; ++k) t += gl[k * p.in + i];
      dst[i] = t;
    }
  }
  __syncthreads();
  if (tid == 0) {   // wave partials in wave order
    float l = red[0][0], b = red[0][1];
#pragma unroll
    for (int k = 1; k < HW; ++k) {
      l += red[k][0];
      b += red[k][1];
    }
    p.loss_part[blockIdx.x] = l;
    if constexpr (FUSE) bslab[blockIdx.x] = b;
  }
}

// Block geometry by row width: (waves per block, rows per wave-iteration of the out == 1 heads).
// 32 / 16 / 16 / 4 rows per block: 8192 rows of <= 512 features give 256 blocks, one per CU (a
// 128-block grid left half the chip idle: 9.5 us for 16 MB of traffic, PMC-measured).  LDS per
// fused block: W row + HW gradient rows = (1 + HW) * in floats <= 64 KiB.
static int head_waves(int in) { return in / 8 <= 64 ? 16 : in / 8 <= 128 ? 8 : 4; }
static int head_rpw(int in) {
  const int nch = in / 8;
  return nch <= 64 ? 2 : nch <= 128 ? 2 : nch <= 256 ? 4 : 1;
}

// one wave-iteration per wave where possible: blocks = rows / (waves * RPW), capped at 256
// MFMA multi-output head (head_mfma_kernel): one block per CU (measured on the 8192 x 1024 x 10
// head: 512 blocks, one row group each and 2 per CU, 16.0 us; 256 blocks 15.3 us)
constexpr int MH_MAX_BLOCKS = 256;

int head_fwd_parts(int rows, int in, int out) {
  if (out > 1 && (in == 512 || in == 1024)) return std::max(1, std::min((rows + 15) / 16, MH_MAX_BLOCKS));
  const int per_block = head_waves(in) * head_rpw(in);
  return std::max(1, std::min((rows + per_block - 1) / per_block, 256));
}

template <typename TA, int CMAX, int LOSS, bool FUSE, int RPW, int OUTM, int HW>
static hipError_t head_launch_act(const HeadArgs& a, int act, int blocks, size_t smem, float* wslab,
                                  float* bslab, hipStream_t s) {
  const dim3 g(blocks), t(64 * HW);
  switch (act) {
    case ACT_RELU:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_RELU, FUSE, RPW, OUTM, HW>), g, t, smem, s, a, wslab, bslab);
      break;
    case ACT_TANH:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_TANH, FUSE, RPW, OUTM, HW>), g, t, smem, s, a, wslab, bslab);
      break;
    default:
      hipLaunchKernelGGL((head_fwd_kernel<TA, CMAX, LOSS, ACT_NONE, FUSE, RPW, OUTM, HW>), g, t, smem, s, a, wslab, bslab);
  }
  return hipGetLastError();
}

template <typename TA, int LOSS, bool FUSE, int OM>
static hipError_t head_launch_c(const HeadArgs& a, int act, int blocks, size_t smem, float* wslab,
                                float* bslab, hipStream_t s) {
  const int nch = a.in / 8;
  // fused (out == 1) heads keep several rows in flight per wave; wide heads one row (registers)
  constexpr int D = (FUSE || OM == 1) ? 1 : 16;
  if (nch <= 64) return head_launch_act<TA, 1, LOSS, FUSE, (2 / D > 0 ? 2 / D : 1), OM, 16>(a, act, blocks, smem, wslab, bslab, s);
  // multi-output heads of <= 1024 features: 4 rows per wave-iteration too (their loads and
  // 4 x out butterflies in flight together; one row at a time left the waves 53 % in s_waitcnt)
  if (nch <= 128) return head_launch_act<TA, 2, LOSS, FUSE, (FUSE || OM == 1) ? 2 : 4, OM, 8>(a, act, blocks, smem, wslab, bslab, s);
  if (nch <= 256) return head_launch_act<TA, 4, LOSS, FUSE, (4 / D > 0 ? 4 / D : 1), OM, 4>(a, act, blocks, smem, wslab, bslab, s);
  if (nch <= 1024) return head_launch_act<TA, 16, LOSS, FUSE, 1, OM, 4>(a, act, blocks, smem, wslab, bslab, s);
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------------------------------------
// Multi-output head (cross-entropy / multi-target MSE, out <= 16) on the matrix cores.
//
// One block = 4 waves = one 16-row group at a time.  The logits are a 16 (outputs, padded) x 16
// (rows) x in GEMM on v_mfma_f32_16x16x4_f32 (exact fp32 products and sums, like the VALU head
// it replaces): wave w covers the w-th quarter of the features, the 4 partial tiles are summed
// through LDS in wave order, and every wave then holds the 16 rows' logits (lane l: row l&15,
// outputs 4(l>>4)..+3), so softmax / MSE need only two cross-lane steps.  dZ_prev = (dl . W) *
// act'(a) is a second MFMA product (16 features x 16 rows, K = 16 outputs) per 16-feature tile
// of the wave's quarter; dl enters as the B operand after 16 shuffles.  W sits in LDS as fp32
// [16][in] with 16-byte chunk c of row n at c ^ (n & 15) (conflict-free for both reads).  The
// VALU head needed ~1500 VALU instructions per row (44 us for 8192 x 1024 x 10).
// ------------------------------------------------------------------------------------------
template <int ACT, int LOSS, int Q>
__global__ void __launch_bounds__(64 * MH_WAVES) head_mfma_kernel(HeadArgs p) {
  extern __shared__ __attribute__((aligned(16))) float ml[];   // W image [16][in] + partials
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int in = 4 * Q;
  const int out = p.out;
  const bf16* A = reinterpret_cast<const bf16*>(p.a);
  bf16* DZ = reinterpret_cast<bf16*>(p.dz_prev);
  const int r = lane & 15, g = lane >> 4;
  const int ngroups = (p.rows + 15) / 16;
  // software pipeline: the global loads of a block's next row group are issued before the
  // current one is computed (first group: before the W image is built)
  MhLoads<Q> cur, nxt;
  // a contiguous run of row groups per XCD-remapped block (same XCD as the forward tiles that
  // wrote these rows: L2 hits instead of Infinity-Cache reads)
  const int per = p.xcd_rows ? (ngroups + (int)gridDim.x - 1) / (int)gridDim.x : 1;
  const int g_beg = p.xcd_rows ? xcd_remap(blockIdx.x, gridDim.x) * per : (int)blockIdx.x;
  const int g_end = p.xcd_rows ? min(ngroups, g_beg + per) : ngroups;
  const int g_step = p.xcd_rows ? 1 : (int)gridDim.x;
  mh_load<Q, LOSS>(cur, p, A, min(g_beg * 16 + r, p.rows - 1), w, g);
  // W image: 16-byte loads, all issued before the first LDS store (compile-time trip count)
  constexpr int NV = 16 * in / 4 / (64 * MH_WAVES);
  f32x4 wv[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MH_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    wv[j] = n < out ? *reinterpret_cast<const f32x4*>(p.W + n * in + k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MH_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    *reinterpret_cast<f32x4*>(ml + mh_off(n, k, in)) = wv[j];
  }
  f32x4* part = reinterpret_cast<f32x4*>(ml + 16 * in);          // [4 waves][64 lanes]
  __syncthreads();
  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = (4 * g + j) < out ? p.b[4 * g + j] : 0.f;
  float block_loss = 0.f;
  for (int grp = g_beg; grp < g_end; grp += g_step) {
    const int row = grp * 16 + r;
    const bool valid = row < p.rows;
    // next group's loads (past the end: the last row again, never read back)
    mh_load<Q, LOSS>(nxt, p, A, min((grp + g_step) * 16 + r, p.rows - 1), w, g);
    __builtin_amdgcn_sched_barrier(0);
    const bf16x8* xs = cur.xs;
    // ---- logits: this wave's quarter of the features ----
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < Q / 32; ++c) {
      const int k = w * Q + c * 32 + g * 8;
      const bf16x8 xv = xs[c];
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(ml + mh_off(r, k, in));
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(ml + mh_off(r, k + 4, in));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w0[e], (float)xv[e], acc, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[e], (float)xv[e + 4], acc, 0, 0, 0);
    }
    part[w * 64 + lane] = acc;
    __syncthreads();
    f32x4 z = part[lane];
#pragma unroll
    for (int ww = 1; ww < MH_WAVES; ++ww) z += part[ww * 64 + lane];
    // ---- loss and dlogits (lane: row r, outputs 4g..4g+3) ----
    float dl[4];
    float row_loss = 0.f;
    if constexpr (LOSS == LOSS_XENT) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        z[j] += bias[j];
        if (4 * g + j < out) mx = fmaxf(mx, z[j]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) if (4 * g + j < out) se += __expf(z[j] - mx);
      se += __shfl_xor(se, 16, 64);
      se += __shfl_xor(se, 32, 64);
      const float lse = mx + __logf(se);
      const int lab = cur.lab;
      float picked = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 4 * g + j;
        if (n == lab) picked = z[j];
        dl[j] = (n < out && valid) ? (__expf(z[j] - lse) - (n == lab ? 1.f : 0.f)) * p.inv_count : 0.f;
      }
      picked += __shfl_xor(picked, 16, 64);
      picked += __shfl_xor(picked, 32, 64);
      row_loss = lse - picked;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 4 * g + j;
        z[j] += bias[j];
        const float d = n < out ? z[j] - cur.yv[j] : 0.f;
        row_loss += d * d;
        dl[j] = valid ? 2.f * d * p.inv_count : 0.f;
      }
      row_loss += __shfl_xor(row_loss, 16, 64);
      row_loss += __shfl_xor(row_loss, 32, 64);
    }
    if (w == 0) {
      if (valid && g == 0) block_loss += row_loss;
      if (p.dlogits && valid) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (4 * g + j < out) p.dlogits[(long long)row * out + 4 * g + j] = dl[j];
      }
    }
    // ---- dZ_prev for this wave's quarter: 16-feature tiles, K = 16 outputs ----
    if (DZ != nullptr) {
      float bfr[4];   // B operand of step s: dl[row r][n = 4s + g], held by lane (s, r) reg g
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int src = st * 16 + r;
        const float t0 = __shfl(dl[0], src, 64), t1 = __shfl(dl[1], src, 64);
        const float t2 = __shfl(dl[2], src, 64), t3 = __shfl(dl[3], src, 64);
        bfr[st] = g == 0 ? t0 : g == 1 ? t1 : g == 2 ? t2 : t3;
      }
      // 32 features per pair of 16x16 tiles; A-operand row i of tile half h is feature
      // f0 + 8(i>>2) + 4h + (i&3), so a lane's two accumulators are features f0 + 8g .. +7 of
      // its row: ONE 16-byte store per pair, and the activation it needs is the logits
      // operand xs[tp] already in registers
#pragma unroll
      for (int tp = 0; tp < Q / 32; ++tp) {
        const int f0 = w * Q + tp * 32;
        const int kf = f0 + 8 * (r >> 2) + (r & 3);
        const bf16x8 av = xs[tp];
        f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(ml[mh_off(4 * st + g, kf, in)], bfr[st], d0, 0, 0, 0);
          d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(ml[mh_off(4 * st + g, kf + 4, in)], bfr[st], d1, 0, 0, 0);
        }
        if (valid) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] = (bf16)(d0[j] * act_bwd_t<ACT>((float)av[j]));
            o[j + 4] = (bf16)(d1[j] * act_bwd_t<ACT>((float)av[j + 4]));
          }
          *reinterpret_cast<bf16x8*>(DZ + (long long)row * in + f0 + 8 * g) = o;
        }
      }
    }
    __syncthreads();   // the partial buffer is rewritten by the next group
    cur = nxt;
  }
  if (w == 0) {
    const float t = wave_sum(block_loss);
    if (lane == 0) p.loss_part[blockIdx.x] = t;
  }
}

// feature counts with a compiled quarter (the loads of a group are unrolled into registers)
bool head_mfma_ok(int a_bf16, int in, int out, bool fuse) {
  return !fuse && a_bf16 && out > 1 && out <= 16 && (in == 512 || in == 1024);
}

template <int Q>
static hipError_t head_mfma_launch_q(const HeadArgs& h, int act, int loss, int blocks, hipStream_t s) {
  const size_t smem = (size_t)(16 * h.in + MH_WAVES * 64 * 4) * sizeof(float);
  using Fn = void (*)(HeadArgs);
  static const Fn fns[2][3] = {
      {head_mfma_kernel<ACT_NONE, LOSS_MSE, Q>, head_mfma_kernel<ACT_RELU, LOSS_MSE, Q>, head_mfma_kernel<ACT_TANH, LOSS_MSE, Q>},
      {head_mfma_kernel<ACT_NONE, LOSS_XENT, Q>, head_mfma_kernel<ACT_RELU, LOSS_XENT, Q>, head_mfma_kernel<ACT_TANH, LOSS_XENT, Q>}};
  static bool attr[2][3] = {};
  const int li = loss == LOSS_XENT ? 1 : 0, ai = act == ACT_RELU ? 1 : act == ACT_TANH ? 2 : 0;
  if (!attr[li][ai]) {
    (void)hipFuncSetAttribute((const void*)fns[li][ai], hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr[li][ai] = true;
  }
  hipLaunchKernelGGL(fns[li][ai], dim3(blocks), dim3(64 * MH_WAVES), smem, s, h);
  return hipGetLastError();
}

static hipError_t head_mfma_launch(const HeadArgs& h, int act, int loss, int blocks, hipStream_t s) {
  return h.in == 512 ? head_mfma_launch_q<128>(h, act, loss, blocks, s)
                     : head_mfma_launch_q<256>(h, act, loss, blocks, s);
}

static hipError_t head_fwd_impl(const void* a, int a_bf16, int rows, int in, const float* W,
                                const float* b, int out, const float* y, const int64_t* labels,
                                int loss, float inv_count, int act_prev, void* dz_prev,
                                float* dlogits, float* loss_part, bool fuse, float* wslab,
                                float* bslab, hipStream_t s) {
  if (out < 1 || out > HEAD_OMAX || in % 8 != 0 || in > 8192) return hipErrorInvalidValue;
  const size_t smem = (size_t)(out * in + (fuse ? head_waves(in) * in : 0)) * sizeof(float);
  if (smem > 65536 + 32768) return hipErrorInvalidValue;
  HeadArgs h{a, rows, in, W, b, out, y, labels, inv_count, act_prev, dz_prev, dlogits, loss_part,
             g_head_xcd_rows};
  const int blocks = head_fwd_parts(rows, in, out);
  if (head_mfma_ok(a_bf16, in, out, fuse)) return head_mfma_launch(h, act_prev, loss, blocks, s);
#define HL(TA, LS, FU, OM) head_launch_c<TA, LS, FU, OM>(h, act_prev, blocks, smem, wslab, bslab, s)
  if (fuse) {
    if (loss == LOSS_XENT || out != 1) return hipErrorInvalidValue;
    return a_bf16 ? HL(bf16, LOSS_MSE, true, 1) : HL(float, LOSS_MSE, true, 1);
  }
  if (loss == LOSS_XENT) return a_bf16 ? HL(bf16, LOSS_XENT, false, HEAD_OMAX) : HL(float, LOSS_XENT, false, HEAD_OMAX);
  if (out == 1) return a_bf16 ? HL(bf16, LOSS_MSE, false, 1) : HL(float, LOSS_MSE, false, 1);
  return a_bf16 ? HL(bf16, LOSS_MSE, false, HEAD_OMAX) : HL(float, LOSS_MSE, false, HEAD_OMAX);
#undef HL
}

hipError_t head_fwd(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                    int out, const float* y, const int64_t* labels, int loss, float inv_count,
                    int act_prev, void* dz_prev, float* dlogits, float* loss_part, hipStream_t s) {
  return head_fwd_impl(a, a_bf16, rows, in, W, b, out, y, labels, loss, inv_count, act_prev, dz_prev,
                       dlogits, loss_part, false, nullptr, nullptr, s);
}

bool head_can_fuse(int out, int in, int loss) { return out == 1 && loss == LOSS_MSE && in <= 2048; }

size_t head_fused_workspace_bytes(int rows, int in) {
  const int G = head_fwd_parts(rows, in);
  return ((size_t)G * in + (size_t)((G + 3) & ~3) + 4) * sizeof(float);
}

// Whole regression head (out == 1, MSE) in two launches: fused fwd/loss/dZ/wgrad partials, then
// the deterministic slab reducer (gW, gb, loss).
hipError_t head_fused(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                      const float* y, float inv_count, int act_prev, void* dz_prev, float* gW,
                      float* gb, float* ws, float* loss_part, float loss_scale, float* loss_out,
                      hipStream_t s, const SgdFuse* sgd, SlabReduce* pending) {
  const int G = head_fwd_parts(rows, in);
  float* wslab = ws;
  float* bslab = ws + (size_t)G * in;
  hipError_t e = head_fwd_impl(a, a_bf16, rows, in, W, b, 1, y, nullptr, LOSS_MSE, inv_count, act_prev,
                               dz_prev, nullptr, loss_part, true, wslab, bslab, s);
  if (e != hipSuccess) return e;
  SlabReduce r{wslab, G, in, 1, in, gW, in, bslab, 1, gb, loss_part, G, loss_scale, loss_out, SgdFuse{}};
  if (sgd) r.sg = *sgd;
  if (pending) {
    *pending = r;
    return hipSuccess;
  }
  return slab_reduce(r, s);
}

// ---- head weight gradient: gW[o][i] = sum_r dl[r][o] a[r][i], gb[o] = sum_r dl[r][o] ----
template <typename TA, int OMAX>
__global__ void __launch_bounds__(256) head_wgrad_kernel(const TA* __restrict__ a, int rows, int in,
                                                         const float* __restrict__ dl, int out,
                                                         int rows_per_split, float* __restrict__ ws,
                                                         float* __restrict__ wsb) {
  // 4 waves per block share one (512-column, split) job: wave w takes the w-th quarter of the
  // split's rows, and the waves are combined through LDS in wave order (deterministic)
  __shared__ __attribute__((aligned(16))) float cmb[OMAX * 512 + OMAX];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c0 = blockIdx.x * 512 + lane * 8;
  const int split = blockIdx.y;
  const int s0 = split * rows_per_split;
  const int s1 = min(rows, s0 + rows_per_split);
  const int q4 = (s1 - s0 + 3) / 4;
  const int r0 = s0 + w * q4;
  const int r1 = min(s1, r0 + q4);
  float acc[OMAX][8];
  float accb[OMAX];
#pragma unroll
  for (int o = 0; o < OMAX; ++o) {
    accb[o] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[o][e] = 0.f;
  }
  const bool active = c0 < in;
  const int cc = active ? c0 : 0;   // clamped column: loads stay unconditional
  // rows in batches of RB: every load of the batch is issued before the first FMA (a single
  // row per iteration exposed one dependent L2 round trip per row: 59 us for 8192 x 1024)
  constexpr int RB = 4;
  for (int r = r0; r < r1; r += RB) {
    float av[RB][8];
    float dv[RB][OMAX];
#pragma unroll
    for (int q = 0; q < RB; ++q) {
      const int rr = min(r + q, r1 - 1);
      const float live = (r + q) < r1 ? 1.f : 0.f;
      load8<TA>(a + (long long)rr * in + cc, av[q]);
#pragma unroll
      for (int o = 0; o < OMAX; ++o) dv[q][o] = dl[(long long)rr * out + min(o, out - 1)] * live;
    }
#pragma unroll
    for (int q = 0; q < RB; ++q)
#pragma unroll
      for (int o = 0; o < OMAX; ++o) {
        if (o < out) {
          accb[o] += dv[q][o];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[o][e] += dv[q][o] * av[q][e];
        }
      }
  }
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int o = 0; o < OMAX; ++o) {
        float* d = cmb + o * 512 + lane * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = ww ? d[e] + acc[o][e] : acc[o][e];
      }
      if (lane == 0) {
#pragma unroll
        for (int o = 0; o < OMAX; ++o) cmb[OMAX * 512 + o] = ww ? cmb[OMAX * 512 + o] + accb[o] : accb[o];
      }
    }
    __syncthreads();
  }
  if (w == 0 && active) {
#pragma unroll
    for (int o = 0; o < OMAX; ++o) {
      if (o < out) {
        float* dst = ws + ((long long)split * out + o) * in + c0;
        const float* src = cmb + o * 512 + lane * 8;
        *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(src);
        *reinterpret_cast<float4*>(dst + 4) = *reinterpret_cast<const float4*>(src + 4);
      }
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
    for (int o = 0; o < OMAX; ++o) if (o < out) wsb[(long long)split * out + o] = cmb[OMAX * 512 + o];
  }
}

// ---- head weight gradient on fp32 MFMA (1 < out <= 16) ----
// gW[o][c] = sum_r dl[r][o] a[r][c] as v_mfma_f32_16x16x4_f32 products, K = 4 rows per step: lane
// l supplies A = dl[r0 + (l>>4)][o = l&15] and, for the 8 column tiles t of its block's 128
// columns, B = a[r0 + (l>>4)][c0 + 8(l&15) + t].  Column j of tile t is c0 + 8j + t, so ONE
// 16-byte activation load per lane and step feeds all 8 MFMAs of the step, and a lane's
// accumulators hold 8 consecutive columns of 4 outputs.  4 waves split the rows of the block's
// (column block, split) job; they are combined in wave order through LDS (deterministic).  The
// VALU kernel above spent 17 us on the 8192 x 1024 x 10 MNIST-shape gradient.
constexpr int HWM_WAVES = 4, HWM_BATCH = 8, HWM_COLS = 128;

template <typename TA>
__global__ void __launch_bounds__(64 * HWM_WAVES) head_wgrad_mfma_kernel(
    const TA* __restrict__ a, int rows, int in, const float* __restrict__ dl, int out,
    int rows_per_split, float* __restrict__ ws, float* __restrict__ wsb) {
  __shared__ __attribute__((aligned(16))) float cmb[HWM_WAVES * 16 * HWM_COLS];
  __shared__ float cbias[HWM_WAVES * 16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int c0 = blockIdx.x * HWM_COLS;
  const int split = blockIdx.y;
  const int o0 = blockIdx.z * 16;           // output tile (heads wider than 16 outputs)
  const int s0 = split * rows_per_split;
  const int s1 = min(rows, s0 + rows_per_split);
  const int q = (s1 - s0 + HWM_WAVES - 1) / HWM_WAVES;
  const int r0 = s0 + w * q;
  const int r1 = min(s1, r0 + q);
  const int cc = min(c0 + 8 * r, in - 8);   // clamped column group (in % 8 == 0)
  const int oc = min(o0 + r, out - 1);
  const bool o_ok = o0 + r < out;
  f32x4 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  for (int rb = r0; rb < r1; rb += 4 * HWM_BATCH) {
    float xv[HWM_BATCH][8];
    float dv[HWM_BATCH];
#pragma unroll
    for (int j = 0; j < HWM_BATCH; ++j) {   // every load of the batch before the first MFMA
      const int row = rb + 4 * j + g;
      const int rr = min(row, r1 - 1);
      load8<TA>(a + (long long)rr * in + cc, xv[j]);
      const float d = dl[(long long)rr * out + oc];
      dv[j] = (row < r1 && o_ok) ? d : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the batch's loads ahead of its MFMAs
#pragma unroll
    for (int j = 0; j < HWM_BATCH; ++j) {
      bsum += dv[j];
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[j], xv[j][t], acc[t], 0, 0, 0);
    }
  }
  bsum += __shfl_xor(bsum, 16, 64);
  bsum += __shfl_xor(bsum, 32, 64);
  float* cw = cmb + w * 16 * HWM_COLS;
#pragma unroll
  for (int e = 0; e < 4; ++e) {   // lane holds outputs 4g + e, columns 8r .. 8r + 7
    float* d = cw + (4 * g + e) * HWM_COLS + 8 * r;
    *reinterpret_cast<f32x4*>(d) = f32x4{acc[0][e], acc[1][e], acc[2][e], acc[3][e]};
    *reinterpret_cast<f32x4*>(d + 4) = f32x4{acc[4][e], acc[5][e], acc[6][e], acc[7][e]};
  }
  if (g == 0) cbias[w * 16 + r] = bsum;
  __syncthreads();
  const int o = threadIdx.x >> 4, c8 = (threadIdx.x & 15) * 8;
  if (o0 + o < out && c0 + c8 < in) {
    const float* src = cmb + o * HWM_COLS + c8;
    f32x4 t0 = *reinterpret_cast<const f32x4*>(src), t1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
    for (int ww = 1; ww < HWM_WAVES; ++ww) {
      t0 += *reinterpret_cast<const f32x4*>(src + ww * 16 * HWM_COLS);
      t1 += *reinterpret_cast<const f32x4*>(src + ww * 16 * HWM_COLS + 4);
    }
    float* dst = ws + ((long long)split * out + o0 + o) * in + c0 + c8;
    *reinterpret_cast<f32x4*>(dst) = t0;
    *reinterpret_cast<f32x4*>(dst + 4) = t1;
  }
  if (blockIdx.x == 0 && threadIdx.x < 16 && o0 + (int)threadIdx.x < out) {
    float t = cbias[threadIdx.x];
#pragma unroll
    for (int ww = 1; ww < HWM_WAVES; ++ww) t += cbias[ww * 16 + threadIdx.x];
    wsb[(long long)split * out + o0 + threadIdx.x] = t;
  }
}

static bool head_wgrad_use_mfma(int out) { return out > 1; }

static int head_splits(int rows, int in, int out) {
  const int cols = head_wgrad_use_mfma(out) ? HWM_COLS : 512;
  const int gx = (in + cols - 1) / cols * (head_wgrad_use_mfma(out) ? (out + 15) / 16 : 1);
  int s = std::max(1, 256 / gx);
  s = std::min(s, std::max(1, rows / 64));
  return s;
}

size_t head_wgrad_workspace_bytes(int rows, int in, int out) {
  const int s = head_splits(rows, in, out);
  return (size_t)s * ((size_t)out * in + out) * sizeof(float);
}


// ------------------------------------------------------------------------------------------
// General head on the matrix cores (bf16 activations, in % 256 == 0, out <= 128): the path for
// heads whose fp32 weight image does not fit the skinny kernel's LDS (e.g. 8192 -> 10) or with
// more than 16 outputs (e.g. 1024 -> 100).  Three stages instead of head_general.hip's four VALU
// launches (1332 us for 4096 x 8192 -> 10, profiles/r3_head_general_vs_skinny_vs_torch.jsonl):
//   1. head_logits_stream_kernel: logits on v_mfma_f32_16x16x4_f32 (exact fp32 products and
//      sums of the bf16 activations and the fp32 weights, fixed order), W streamed from L2
//      (every block re-reads it; a 16-row group reads NT x 16 x in floats), loss and dlogits in
//      registers -> dl (fp32, for the weight gradient) and a bf16 copy padded to outp columns;
//   2. dZ_prev = (dl . W) * act'(a): the bf16 dgrad GEMM (gemm_bf16.hip, K = out) on the bf16
//      dl copy and a bf16 image of W -- the same rounding as every hidden layer's dgrad;
//   3. gW, gb: head_wgrad's fp32 MFMA kernel in 16-output tiles + the deterministic reducer
//      (the loss partials fold in there).
// ------------------------------------------------------------------------------------------
constexpr int HS_WAVES = 4;
constexpr int HS_MAX_NT = 8;   // outputs <= 128

template <int LOSS, int NT>
__global__ void __launch_bounds__(64 * HS_WAVES) head_logits_stream_kernel(
    const bf16* __restrict__ a, int rows, int in, const float* __restrict__ W,
    const float* __restrict__ b, int out, const float* __restrict__ y,
    const int64_t* __restrict__ labels, float inv_count, float* __restrict__ dl,
    bf16* __restrict__ dl16, int outp, float* __restrict__ loss_part) {
  __shared__ f32x4 part[HS_WAVES * NT * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int Q = in / HS_WAVES;               // this wave's quarter of the features
  const int ngroups = (rows + 15) / 16;
  constexpr int U = NT <= 4 ? 2 : 1;         // 32-feature chunks per iteration (registers)
  // weight rows of this lane's A operand: n = 16 t + r (clamped, masked)
  const float* wrow[NT];
  float wmask[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    wrow[t] = W + (long long)min(16 * t + r, out - 1) * in;
    wmask[t] = (16 * t + r) < out ? 1.f : 0.f;
  }
  float block_loss = 0.f;
  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    const int row = grp * 16 + r;
    const bool valid = row < rows;
    const bf16* ar = a + (long long)min(row, rows - 1) * in + w * Q + 8 * g;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < Q; c += 32 * U) {    // every load of the step before its MFMAs
      bf16x8 xv[U];
      f32x4 wv[U][NT][2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xv[u] = *reinterpret_cast<const bf16x8*>(ar + c + 32 * u);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float* wp = wrow[t] + w * Q + c + 32 * u + 8 * g;
          wv[u][t][0] = *reinterpret_cast<const f32x4*>(wp) * wmask[t];
          wv[u][t][1] = *reinterpret_cast<const f32x4*>(wp + 4) * wmask[t];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][t][0][e], (float)xv[u][e], acc[t], 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[u][t][1][e], (float)xv[u][e + 4], acc[t], 0, 0, 0);
        }
    }
    // The LDS store below reads the accumulators the loop's last MFMA wrote.  For NT == 1 the
    // compiler (ROCm 7.2 hipcc, gfx950) placed that ds_write two instructions after the final
    // v_mfma_f32_16x16x4_f32 with no wait states, so it stored a stale partial sum (logits off by
    // a few percent at in >= 2048; NT >= 2 got its s_nops).  Pin 20 wait states between the two,
    // more than any XDL-write -> LDS-read distance needs.
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < NT; ++t) part[(w * NT + t) * 64 + lane] = acc[t];
    __syncthreads();
    if (w == 0) {
      // lane (r, g) holds the logits of row r, outputs 16 t + 4 g + j (wave order sums)
      float z[NT][4];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        f32x4 v = part[t * 64 + lane];
#pragma unroll
        for (int ww = 1; ww < HS_WAVES; ++ww) v += part[(ww * NT + t) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = 16 * t + 4 * g + j;
          z[t][j] = v[j] + (n < out ? b[n] : 0.f);
        }
      }
      float d[NT][4];
      float row_loss = 0.f;
      if constexpr (LOSS == LOSS_XENT) {
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (16 * t + 4 * g + j < out) mx = fmaxf(mx, z[t][j]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float se = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (16 * t + 4 * g + j < out) se += __expf(z[t][j] - mx);
        se += __shfl_xor(se, 16, 64);
        se += __shfl_xor(se, 32, 64);
        const float lse = mx + __logf(se);
        const int lab = (int)labels[min(row, rows - 1)];
        float picked = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 16 * t + 4 * g + j;
            if (n == lab) picked = z[t][j];
            d[t][j] = (n < out && valid) ? (__expf(z[t][j] - lse) - (n == lab ? 1.f : 0.f)) * inv_count : 0.f;
          }
        picked += __shfl_xor(picked, 16, 64);
        picked += __shfl_xor(picked, 32, 64);
        row_loss = lse - picked;
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 16 * t + 4 * g + j;
            const float dd = n < out ? z[t][j] - y[(long long)min(row, rows - 1) * out + min(n, out - 1)] : 0.f;
            row_loss += dd * dd;
            d[t][j] = valid ? 2.f * dd * inv_count : 0.f;
          }
        row_loss += __shfl_xor(row_loss, 16, 64);
        row_loss += __shfl_xor(row_loss, 32, 64);
      }
      if (valid) {
        if (g == 0) block_loss += row_loss;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = 16 * t + 4 * g + j;
            if (n < out) dl[(long long)row * out + n] = d[t][j];
            if (n < outp) dl16[(long long)row * outp + n] = (bf16)d[t][j];
          }
      }
    }
    __syncthreads();   // part[] is rewritten by the next group
  }
  if (w == 0) {
    const float t = wave_sum(block_loss);
    if (lane == 0) loss_part[blockIdx.x] = t;
  }
}

bool head_general_mfma_ok(int a_bf16, int in, int out) {
  // (each wave's quarter of the features is walked in 64-feature steps)
  return a_bf16 && in % 256 == 0 && out >= 1 && out <= 16 * HS_MAX_NT;
}

static int hs_outp(int out) { return (out + 7) / 8 * 8; }
static int hs_blocks(int rows) { return std::max(1, std::min(1024, (rows + 15) / 16)); }

// workspace (floats): dl [rows*out] | dl16 [rows*outp bf16] | W16 [outp*in bf16] | loss partials
// | head_wgrad workspace
size_t head_general_mfma_workspace_bytes(int rows, int in, int out) {
  const size_t f = (size_t)rows * out + ((size_t)rows * hs_outp(out) + 1) / 2 + 4 +
                   ((size_t)hs_outp(out) * in + 1) / 2 + 4 + hs_blocks(rows) + 4;
  return (f + 64) * sizeof(float) + head_wgrad_workspace_bytes(rows, in, out);
}

hipError_t head_general_mfma(const bf16* a, int rows, int in, const float* W, const float* b,
                             int out, const float* y, const int64_t* labels, int loss,
                             float inv_count, int act_prev, bf16* dz_out, float* gW, float* gb,
                             float* dlogits_out, float* ws, float loss_scale, float* loss_out,
                             hipStream_t s) {
  if (!head_general_mfma_ok(1, in, out) || rows < 1) return hipErrorInvalidValue;
  const int outp = hs_outp(out), nb = hs_blocks(rows);
  auto align16 = [](float* p) {
    return reinterpret_cast<float*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
  };
  float* dl = dlogits_out ? dlogits_out : ws;
  float* cur = align16(ws + (size_t)rows * out);
  bf16* dl16 = reinterpret_cast<bf16*>(cur);
  cur = align16(cur + ((size_t)rows * outp + 1) / 2);
  bf16* W16 = reinterpret_cast<bf16*>(cur);
  cur = align16(cur + ((size_t)outp * in + 1) / 2);
  float* lpart = cur;
  float* wws = align16(lpart + nb);
  // the padding columns of the bf16 dl copy stay zero (the dgrad GEMM reads 8-wide chunks)
  if (outp != out) {
    hipError_t e = hipMemsetAsync(dl16, 0, (size_t)rows * outp * sizeof(bf16), s);
    if (e != hipSuccess) return e;
  }
  const int nt = (out + 15) / 16;
#define HS_LAUNCH(L, NT)                                                                          \
  hipLaunchKernelGGL((head_logits_stream_kernel<L, NT>), dim3(nb), dim3(64 * HS_WAVES), 0, s, a, \
                     rows, in, W, b, out, y, labels, inv_count, dl, dl16, outp, lpart)
#define HS_NT(L)                                                                                  \
  switch (nt) {                                                                                   \
    case 1: HS_LAUNCH(L, 1); break;                                                               \
    case 2: HS_LAUNCH(L, 2); break;                                                               \
    case 3: HS_LAUNCH(L, 3); break;                                                               \
    case 4: HS_LAUNCH(L, 4); break;                                                               \
    case 5: HS_LAUNCH(L, 5); break;                                                               \
    case 6: HS_LAUNCH(L, 6); break;                                                               \
    case 7: HS_LAUNCH(L, 7); break;                                                               \
    default: HS_LAUNCH(L, 8); break;                                                              \
  }
  if (loss == LOSS_XENT) { HS_NT(LOSS_XENT) } else { HS_NT(LOSS_MSE) }
#undef HS_NT
#undef HS_LAUNCH
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (dz_out) {
    e = cast_f32_bf16(W, W16, (long long)out * in, s);
    if (e != hipSuccess) return e;
    // the bf16 GEMM wants K % 8 == 0: K = outp, with zero rows of W16 against dl16's zero columns
    if (outp != out) {
      e = hipMemsetAsync(W16 + (size_t)out * in, 0, (size_t)(outp - out) * in * sizeof(bf16), s);
      if (e != hipSuccess) return e;
    }
    // dZ[rows][in] = dl16[rows][outp] . W16[outp][in] * act'(a)
    e = linear_dgrad_bf16(dl16, outp, W16, in, a, in, dz_out, in, rows, in, outp, act_prev, s);
    if (e != hipSuccess) return e;
  }
  return head_wgrad(a, 1, rows, in, dl, out, gW, gb, wws, lpart, nb, loss_scale, loss_out, s,
                    nullptr, nullptr);
}

hipError_t head_wgrad(const void* a, int a_bf16, int rows, int in, const float* dlogits, int out,
                      float* gW, float* gb, float* ws, const float* loss_part, int n_loss_part,
                      float loss_scale, float* loss_out, hipStream_t s, const SgdFuse* sgd,
                      SlabReduce* pending) {
  // (more than 16 outputs: the MFMA kernel in 16-output tiles, grid z)
  if (out < 1 || (out > HEAD_OMAX && !head_wgrad_use_mfma(out)) || in % 8 != 0 || rows < 1)
    return hipErrorInvalidValue;
  const int S = head_splits(rows, in, out);
  const int rps = (rows + S - 1) / S;
  float* wsb = ws + (size_t)S * out * in;
  if (head_wgrad_use_mfma(out)) {
    const dim3 grid((in + HWM_COLS - 1) / HWM_COLS, S, (out + 15) / 16), blk(64 * HWM_WAVES);
    if (a_bf16) hipLaunchKernelGGL(head_wgrad_mfma_kernel<bf16>, grid, blk, 0, s, reinterpret_cast<const bf16*>(a), rows, in, dlogits, out, rps, ws, wsb);
    else hipLaunchKernelGGL(head_wgrad_mfma_kernel<float>, grid, blk, 0, s, reinterpret_cast<const float*>(a), rows, in, dlogits, out, rps, ws, wsb);
  } else {
    const dim3 grid((in + 511) / 512, S);
    if (a_bf16) hipLaunchKernelGGL((head_wgrad_kernel<bf16, 1>), grid, dim3(256), 0, s, reinterpret_cast<const bf16*>(a), rows, in, dlogits, out, rps, ws, wsb);
    else hipLaunchKernelGGL((head_wgrad_kernel<float, 1>), grid, dim3(256), 0, s, reinterpret_cast<const float*>(a), rows, in, dlogits, out, rps, ws, wsb);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  SlabReduce r{ws, S, (long long)out * in, out, in, gW, in, wsb, out, gb, loss_part, n_loss_part,
               loss_scale, loss_out, SgdFuse{}};
  if (sgd) r.sg = *sgd;
  if (pending) {
    *pending = r;
    return hipSuccess;
  }
  return slab_reduce(r, s);
}

}  // namespace nnmpi
