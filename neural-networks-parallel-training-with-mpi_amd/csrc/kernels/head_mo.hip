// Fused multi-output head: logits, loss, dZ_prev and the head weight gradient in one kernel
// (reference ops K3-K8, ref.py:44,94,173,176, for the MNIST-shape 1024 -> 10 cross-entropy head).
#include "head_common.h"
#include "knobs.h"

#include <algorithm>
#include <type_traits>

namespace nnmpi {

// ------------------------------------------------------------------------------------------
// Fused multi-output head (MNIST shape: cross-entropy / multi-target MSE, 1 < out <= 16,
// in = 512 / 1024, bf16 activations): head_mfma_kernel's logits, loss and dZ_prev AND the
// head's weight gradient in ONE pass (the separate head_wgrad_mfma launch re-read the 16 MB of
// activations: 16.2 + 7.2 us of the MNIST step, profiles/r3s2_final_kstats_mnist.csv).
//
// 512-thread blocks = 2 teams of 4 waves; SIMD s holds wave s of both teams.  Per iteration the
// two teams take two consecutive 16-row groups.  A team runs its group the head_mfma_kernel way
// (wave w = feature quarter; two independent 32-step logits chains, the partial tiles summed
// through LDS in wave order; softmax / MSE in registers; dZ_prev on MFMA) and publishes the
// group's dlogits (16 x 16 fp32) in LDS.  Then the weight gradient of BOTH groups is split by
// columns instead of rows: wave (t, w) accumulates gW[:, its quarter's t-th column half] over the
// 32 rows as v_mfma_f32_16x16x4_f32 products (exact fp32, K = 4 rows per step; A = dl[row][o =
// l&15] from LDS, B = a[row][c0 + 8(l&15) + tile] re-loaded from global: an L1/L2 hit, the
// team has just read these rows) -- head_wgrad_mfma's operand map.  Every gW element thus has
// ONE owner wave summing all of the block's rows in a fixed order: no team combine, and the
// accumulators are half a quarter wide (32 VGPRs at in = 1024).  The block writes one partial
// slab gW [out][in], gb [out] and its loss for the deterministic reducer (slab_reduce's deep
// form: 256 slabs).
// ------------------------------------------------------------------------------------------
constexpr int MF_TEAMS = 2, MF_WAVES = 4 * MF_TEAMS;

template <int ACT, int LOSS, int Q>
__global__ void __launch_bounds__(64 * MF_WAVES) head_mo_fused_kernel(HeadArgs p,
                                                                      float* __restrict__ gws,
                                                                      float* __restrict__ gwsb) {
  extern __shared__ __attribute__((aligned(16))) float ml[];   // W image | partials | dl | sums
  constexpr int in = 4 * Q;
  // a wave's weight-gradient columns: NT tiles of 16 x 16, column of (tile tt, lane row r) =
  // c0 + 8r + tt0 + tt; B loads of NT bf16 per lane and row
  constexpr int NT = Q == 256 ? 8 : 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2, w = wv & 3;
  const int c0 = Q == 256 ? w * Q + team * 128 : w * Q;
  const int tt0 = Q == 256 ? 0 : 4 * team;
  const int out = p.out;
  const bf16* A = reinterpret_cast<const bf16*>(p.a);
  bf16* DZ = reinterpret_cast<bf16*>(p.dz_prev);
  const int r = lane & 15, g = lane >> 4;
  const int ngroups = (p.rows + 15) / 16;
  // a contiguous run of row groups per (XCD-remapped) block: the rows the forward tiles of
  // this XCD wrote
  const int per = (ngroups + (int)gridDim.x - 1) / (int)gridDim.x;
  const int g_beg = xcd_remap(blockIdx.x, gridDim.x) * per;
  const int g_end = min(ngroups, g_beg + per);
  // W image: 16-byte loads, all issued before the first LDS store
  constexpr int NV = 16 * in / 4 / (64 * MF_WAVES);
  f32x4 wimg[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MF_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    wimg[j] = n < out ? *reinterpret_cast<const f32x4*>(p.W + n * in + k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MF_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    *reinterpret_cast<f32x4*>(ml + mh_off(n, k, in)) = wimg[j];
  }
  f32x4* part = reinterpret_cast<f32x4*>(ml + 16 * in) + team * 4 * 64;   // [team][wave][lane]
  float* dlb = ml + 16 * in + MF_WAVES * 64 * 4;                          // [team][row][out]
  float* sums = dlb + MF_TEAMS * 256;                                     // loss [team]
  __syncthreads();
  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = (4 * g + j) < out ? p.b[4 * g + j] : 0.f;
  f32x4 gacc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) gacc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f, block_loss = 0.f;
  for (int base = g_beg; base < g_end; base += MF_TEAMS) {
    const int grp = base + team;
    const int row = grp * 16 + r;
    const bool valid = grp < g_end && row < p.rows;
    MhLoads<Q> cur;
    mh_load<Q, LOSS>(cur, p, A, min(row, p.rows - 1), w, g);
    const bf16x8* xs = cur.xs;
    // ---- logits: this wave's quarter, two independent chains ----
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < Q / 32; ++c) {
      const int k = w * Q + c * 32 + g * 8;
      const bf16x8 xv = xs[c];
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(ml + mh_off(r, k, in));
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(ml + mh_off(r, k + 4, in));
#pragma unroll
      for (int e = 0; e < 4; ++e) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(w0[e], (float)xv[e], acc0, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(w1[e], (float)xv[e + 4], acc1, 0, 0, 0);
    }
    part[w * 64 + lane] = acc0 + acc1;
    __syncthreads();
    f32x4 z = part[lane];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) z += part[ww * 64 + lane];
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
      *reinterpret_cast<f32x4*>(dlb + team * 256 + r * 16 + 4 * g) = f32x4{dl[0], dl[1], dl[2], dl[3]};
    }
    // ---- dZ_prev for this wave's quarter (head_mfma_kernel's tile pairs) ----
    if (DZ != nullptr) {
      float bfr[4];
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int src = st * 16 + r;
        const float t0 = __shfl(dl[0], src, 64), t1 = __shfl(dl[1], src, 64);
        const float t2 = __shfl(dl[2], src, 64), t3 = __shfl(dl[3], src, 64);
        bfr[st] = g == 0 ? t0 : g == 1 ? t1 : g == 2 ? t2 : t3;
      }
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
    // the weight-gradient operand of both groups (rows 4s + g, NT features per lane), issued
    // after the dZ work (xs dead: no register overlap) so the loads fly across the barrier
    using BV = typename std::conditional<NT == 8, bf16x8, bf16x4>::type;
    BV xb[MF_TEAMS][4];
#pragma unroll
    for (int gg = 0; gg < MF_TEAMS; ++gg)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int rr = min((base + gg) * 16 + 4 * s + g, p.rows - 1);
        xb[gg][s] = *reinterpret_cast<const BV*>(A + (long long)rr * in + c0 + 8 * r + tt0);
      }
    __syncthreads();   // both groups' dlogits published
    // ---- gW[:, this wave's columns] += dl^T a over the 32 rows, 4 rows per step ----
#pragma unroll
    for (int gg = 0; gg < MF_TEAMS; ++gg)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float dv = dlb[gg * 256 + (4 * s + g) * 16 + r];   // dl[row 4s + g][o = r]
        if (wv == 0) bsum += dv;
#pragma unroll
        for (int t = 0; t < NT; ++t)
          gacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(dv, (float)xb[gg][s][t], gacc[t], 0, 0, 0);
      }
    __syncthreads();   // the partial and dl buffers are rewritten by the next iteration
  }
  // ---- block partials: every gW element has one owner lane ----
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int o = 4 * g + i;
    if (o < out) {
      float* dst = gws + ((long long)blockIdx.x * out + o) * in + c0 + 8 * r + tt0;
      if constexpr (NT == 8) {
        *reinterpret_cast<f32x4*>(dst) = f32x4{gacc[0][i], gacc[1][i], gacc[2][i], gacc[3][i]};
        *reinterpret_cast<f32x4*>(dst + 4) = f32x4{gacc[4][i], gacc[5][i], gacc[6][i], gacc[7][i]};
      } else {
        *reinterpret_cast<f32x4*>(dst) = f32x4{gacc[0][i], gacc[1][i], gacc[2][i], gacc[3][i]};
      }
    }
  }
  bsum += __shfl_xor(bsum, 16, 64);
  bsum += __shfl_xor(bsum, 32, 64);
  if (w == 0) {
    const float t = wave_sum(block_loss);
    if (lane == 0) sums[team] = t;
  }
  if (wv == 0 && g == 0 && r < out) gwsb[(long long)blockIdx.x * out + r] = bsum;
  __syncthreads();
  if (tid == 0) p.loss_part[blockIdx.x] = sums[0] + sums[1];
}

static int g_head_fused_mo = -1;   // NNMPI_HEAD_FUSED=0: separate head + head_wgrad launches (A/B)
void set_head_fused(int on) { g_head_fused_mo = on; }   // -1: re-read the environment
static bool head_fused_mo_on() {
  if (g_head_fused_mo < 0) {
    const char* e = knob_env("NNMPI_HEAD_FUSED");
    g_head_fused_mo = (e && e[0] == '0') ? 0 : 1;
  }
  return g_head_fused_mo == 1;
}

static int head_mo_blocks(int rows) {
  return std::max(1, std::min(256, ((rows + 15) / 16 + MF_TEAMS - 1) / MF_TEAMS));
}

bool head_mo_fused_ok(int a_bf16, int rows, int in, int out, int loss) {
  return head_fused_mo_on() && a_bf16 && rows >= 1 && out > 1 && out <= 16 &&
         (in == 512 || in == 1024) && (loss == LOSS_XENT || loss == LOSS_MSE);
}

size_t head_mo_workspace_bytes(int rows, int in, int out) {
  return (size_t)head_mo_blocks(rows) * ((size_t)out * in + out) * sizeof(float);
}

template <int Q>
static hipError_t head_mo_launch_q(const HeadArgs& h, int act, int loss, int blocks, float* gws,
                                   float* gwsb, hipStream_t s) {
  const size_t smem = (size_t)(16 * h.in + MF_WAVES * 64 * 4 + MF_TEAMS * 256 + 16) * sizeof(float);
  using Fn = void (*)(HeadArgs, float*, float*);
  static const Fn fns[2][3] = {
      {head_mo_fused_kernel<ACT_NONE, LOSS_MSE, Q>, head_mo_fused_kernel<ACT_RELU, LOSS_MSE, Q>, head_mo_fused_kernel<ACT_TANH, LOSS_MSE, Q>},
      {head_mo_fused_kernel<ACT_NONE, LOSS_XENT, Q>, head_mo_fused_kernel<ACT_RELU, LOSS_XENT, Q>, head_mo_fused_kernel<ACT_TANH, LOSS_XENT, Q>}};
  static bool attr[2][3] = {};
  const int li = loss == LOSS_XENT ? 1 : 0, ai = act == ACT_RELU ? 1 : act == ACT_TANH ? 2 : 0;
  if (!attr[li][ai]) {
    (void)hipFuncSetAttribute((const void*)fns[li][ai], hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr[li][ai] = true;
  }
  hipLaunchKernelGGL(fns[li][ai], dim3(blocks), dim3(64 * MF_WAVES), smem, s, h, gws, gwsb);
  return hipGetLastError();
}

// Whole multi-output head in two launches: the fused kernel, then the deterministic combine
// (gW, gb, loss; optionally the optimizer update) -- or the combine returned as pending for the
// next grouped backward launch.  loss_part needs head_fwd_parts(rows, in, out) entries; ws
// head_mo_workspace_bytes.
hipError_t head_mo_fused(const bf16* a, int rows, int in, const float* W, const float* b, int out,
                         const float* y, const int64_t* labels, int loss, float inv_count,
                         int act_prev, void* dz_prev, float* gW, float* gb, float* ws,
                         float* loss_part, float loss_scale, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd, SlabReduce* pending) {
  if (!head_mo_fused_ok(1, rows, in, out, loss)) return hipErrorInvalidValue;
  if ((loss == LOSS_XENT && !labels) || (loss == LOSS_MSE && !y)) return hipErrorInvalidValue;
  const int G = head_mo_blocks(rows);
  float* gws = ws;
  float* gwsb = ws + (size_t)G * out * in;
  HeadArgs h{a, rows, in, W, b, out, y, labels, inv_count, act_prev, dz_prev, nullptr, loss_part, 1};
  hipError_t e = in == 512 ? head_mo_launch_q<128>(h, act_prev, loss, G, gws, gwsb, s)
                           : head_mo_launch_q<256>(h, act_prev, loss, G, gws, gwsb, s);
  if (e != hipSuccess) return e;
  SlabReduce r{gws, G, (long long)out * in, out, in, gW, in, gwsb, out, gb, loss_part, G, loss_scale,
               loss_out, SgdFuse{}};
  if (sgd) r.sg = *sgd;
  if (pending) {
    *pending = r;
    return hipSuccess;
  }
  return slab_reduce(r, s);
}

}  // namespace nnmpi
