// Fused multi-output head: logits, loss, dZ_prev and the head weight gradient in one kernel
// (reference ops K3-K8, ref.py:44,94,173,176, for the MNIST-shape 1024 -> 10 cross-entropy head).
#include "head_common.h"
#include "knobs.h"

#include <algorithm>
#include <cstdlib>

namespace nnmpi {

// ------------------------------------------------------------------------------------------
// Fused multi-output head (MNIST shape: cross-entropy / multi-target MSE, 1 < out <= 16,
// in = 512 / 1024, bf16 activations): logits, loss, dZ_prev AND the head's weight gradient in
// ONE pass over the activations, every product on the bf16 matrix cores
// (v_mfma_f32_16x16x32_bf16, 1/8 the issue cycles of the fp32 v_mfma_f32_16x16x4_f32 per FLOP).
// The two launches it replaces (head_mfma_kernel + head_wgrad_mfma_kernel, fp32 MFMA) took
// 16.2 + 7.2 us of the MNIST step (profiles/r3s2_final_kstats_mnist.csv).
//
// Precision (the fp32 reference's products, to the bits that matter):
//   logits  = a . (W_hi + W_lo)^T   W split into two bf16 terms (16 significant bits), a is bf16:
//             every product exact in fp32, fp32 accumulation -> logits to ~2^-16 relative;
//   dZ_prev = (bf16(dl) . W_hi) * act'(a), stored as bf16 -- the rounding of every hidden layer's
//             dgrad GEMM (bf16 operands, fp32 accumulation), inside test_head's bound;
//   gW      = (dl_hi + dl_lo)^T . a, gb = sum dl (fp32) -- dl split like W: ~2^-16 relative.
//
// Block: 512 threads = 2 teams x 4 waves; each iteration the teams take two consecutive 16-row
// groups.  Wave (t, w) owns feature quarter w of its team's group for the logits (B operand =
// its 16-byte activation loads, lane (row l&15, 8 features)) and dZ; the partial logit tiles
// are summed through LDS in wave order.  The weight gradient needs K = rows: the two groups'
// activations are staged through LDS as a [32 rows][512 columns] image read back transposed
// (ds_read_b64_tr_b16), one 512-column phase at a time, and every wave owns 4 column tiles of a
// phase -- each gW element has one owner summing the block's rows in a fixed order.  LDS:
// W_hi / W_lo [16][in + 8] bf16 (padded rows: conflict-free 16-byte reads), W_hi^T [in][16],
// the a stage, logit partials, dlogits: 141 KB at in = 1024.  The block writes ONE partial slab
// gW [out][in], gb [out] and its loss for the deterministic reducer (slab_reduce's deep form).
// ------------------------------------------------------------------------------------------
constexpr int MF_TEAMS = 2, MF_WAVES = 4 * MF_TEAMS;
constexpr int MF_PH = 512;   // columns per weight-gradient phase
// dlogits staging [team][16 rows][16 outputs] fp32 with padded strides: the weight gradient's
// A-operand reads (lane: output r, rows 8g .. 8g+7 of the two groups) put lanes of different g at
// bank offsets 0 / 32 / 16 / 48 instead of all at 0 (4-way conflicts with a 16-float row stride)
constexpr int MF_DLB_ROW = 20, MF_DLB_TEAM = 336;   // (336 = 16 x 20 + 16: the team offset is 16 banks)
// the block's gW partial image [16][in] fp32 in LDS: row stride in + 4 (rows 4g + i of the
// writing lanes land 16 banks apart)
constexpr int MF_GROW_PAD = 4;

template <int IN>
struct MfLds {
  static constexpr int WROW = IN + 8;                       // padded W_hi / W_lo row (bf16)
  static constexpr int WHI = 0;
  static constexpr int WLO = WHI + 16 * WROW * 2;
  static constexpr int WT = WLO + 16 * WROW * 2;            // [IN][16] bf16
  static constexpr int STAGE = WT + IN * 16 * 2;            // [32][MF_PH] bf16, swizzled
  static constexpr int PART = STAGE + 32 * MF_PH * 2;       // [waves][64] f32x4
  static constexpr int DLB = PART + MF_WAVES * 64 * 16;     // [team][16 rows][16 outs] fp32 (padded)
  static constexpr int SUMS = DLB + MF_TEAMS * MF_DLB_TEAM * 4;   // loss [team]
  static constexpr int BYTES = SUMS + 64;
};

// W_hi^T image: row f (16 outputs, 32 B) stored at row f ^ (bit 3 of f -> bit 2) with its two
// 16-byte halves swapped when bit 4 of f is set: the 16 lanes of a dZ A-operand read (rows
// f0 + 8(m >> 2) + 4h + (m & 3), one half) then hit 16 distinct 16-byte slots of a 256-byte bank
// row (plain 32-byte rows: 4-way conflicts)
__device__ __forceinline__ int mf_wt_off(int f, int half) {
  return (f ^ (((f >> 3) & 1) << 2)) * 16 + ((half ^ ((f >> 4) & 1)) << 3);
}

// a-stage image: row k (0..31) of MF_PH bf16, 16-byte chunk c of row k at c ^ swz(k)
__device__ __forceinline__ int mf_stage_off(int k, int x) {
  const int swz = ((k & 3) | ((k >> 1) & 4)) << 1;
  return k * (MF_PH * 2) + ((((x >> 3) ^ swz)) << 4) + ((x & 7) << 1);
}

// B operand (k = row 8(l>>4) + j, n = column xb + (l&15)) of the staged activations
__device__ __forceinline__ bf16x8 mf_stage_frag(const char* stage, int xb, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int k = 8 * (lane >> 4) + q;
  const int x = xb + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(stage + mf_stage_off(k, x)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(stage + mf_stage_off(k + 4, x)));
  typedef __attribute__((ext_vector_type(8))) short s16x8;
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int ACT, int LOSS, int Q>
__global__ void __launch_bounds__(64 * MF_WAVES) head_mo_fused_kernel(HeadArgs p,
                                                                      float* __restrict__ gws,
                                                                      float* __restrict__ gwsb,
                                                                      unsigned long long* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // diagnostic phase stamps (st != null: scripts/r4_head_stamps.py): 100 MHz real-time counter
  // at 8 points of the first iteration, written by thread 0
  const auto stamp = [&](int i) {
    if (st && threadIdx.x == 0) st[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  constexpr int in = 4 * Q;
  using L = MfLds<in>;
  constexpr int NPH = in / MF_PH;           // weight-gradient phases
  constexpr int QPP = MF_PH / Q;            // feature quarters per phase
  bf16* whi = reinterpret_cast<bf16*>(smem + L::WHI);
  bf16* wlo = reinterpret_cast<bf16*>(smem + L::WLO);
  bf16* wt = reinterpret_cast<bf16*>(smem + L::WT);
  char* stage = smem + L::STAGE;
  f32x4* part_all = reinterpret_cast<f32x4*>(smem + L::PART);
  float* dlb = reinterpret_cast<float*>(smem + L::DLB);
  float* sums = reinterpret_cast<float*>(smem + L::SUMS);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int team = wv >> 2, w = wv & 3;
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
  // the first row group's activations and labels: independent of the W images, so their loads
  // are issued first and fly during the image build
  MhLoads<Q> cur, nxt;
  mh_load<Q, LOSS>(cur, p, A, min((g_beg + team) * 16 + r, p.rows - 1), w, g);
  // ---- W images: W = W_hi + W_lo (bf16 each) from 16-byte row loads; W_hi^T from W_hi in LDS
  // after a barrier (a second, column-wise read of W from L2 by all 256 blocks cost ~4 us; a
  // 2-byte transpose store from the row pass puts 64 lanes on two banks)
  constexpr int NV = 16 * in / 4 / (64 * MF_WAVES);
  constexpr int NC = in / (64 * MF_WAVES);   // W^T rows per thread
  f32x4 wimg[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MF_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    wimg[j] = n < out ? *reinterpret_cast<const f32x4*>(p.W + n * in + k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int i4 = j * 64 * MF_WAVES + tid, n = i4 / (in / 4), k = (i4 % (in / 4)) * 4;
    bf16x4 h, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      h[e] = (bf16)wimg[j][e];
      l[e] = (bf16)(wimg[j][e] - (float)h[e]);
    }
    *reinterpret_cast<bf16x4*>(whi + n * L::WROW + k) = h;
    *reinterpret_cast<bf16x4*>(wlo + n * L::WROW + k) = l;
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int kk = c * 64 * MF_WAVES + tid;
    bf16x8 t0, t1;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      t0[n] = whi[n * L::WROW + kk];
      t1[n] = whi[(n + 8) * L::WROW + kk];
    }
    *reinterpret_cast<bf16x8*>(wt + mf_wt_off(kk, 0)) = t0;
    *reinterpret_cast<bf16x8*>(wt + mf_wt_off(kk, 1)) = t1;
  }
  f32x4* part = part_all + team * 4 * 64;
  __syncthreads();
  stamp(1);
  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = (4 * g + j) < out ? p.b[4 * g + j] : 0.f;
  f32x4 gacc[NPH][4];
#pragma unroll
  for (int ph = 0; ph < NPH; ++ph)
#pragma unroll
    for (int t = 0; t < 4; ++t) gacc[ph][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f, block_loss = 0.f;
  const bf16x8 zero8 = {};
  for (int base = g_beg; base < g_end; base += MF_TEAMS) {
    const int grp = base + team;
    const int row = grp * 16 + r;
    const bool valid = grp < g_end && row < p.rows;
    const bf16x8* xs = cur.xs;
    // ---- logits: this wave's quarter, W_hi and W_lo terms in two chains ----
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < Q / 32; ++c) {
      const int k = w * Q + c * 32 + g * 8;
      const bf16x8 wh = *reinterpret_cast<const bf16x8*>(whi + r * L::WROW + k);
      const bf16x8 wl = *reinterpret_cast<const bf16x8*>(wlo + r * L::WROW + k);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xs[c], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xs[c], acc1, 0, 0, 0);
    }
    part[w * 64 + lane] = acc0 + acc1;
    __syncthreads();
    if (base == g_beg) stamp(2);
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
      *reinterpret_cast<f32x4*>(dlb + team * MF_DLB_TEAM + r * MF_DLB_ROW + 4 * g) = f32x4{dl[0], dl[1], dl[2], dl[3]};
    }
    __syncthreads();   // both groups' dlogits published
    if (base == g_beg) stamp(3);
    // ---- dZ_prev for this wave's quarter: K = outputs (16, zero-padded to 32) ----
    if (DZ != nullptr) {
      bf16x8 bdl = zero8;   // B operand: dl[row r][outputs 8g .. 8g+7] in bf16
      if (g < 2) {
        const f32x4 d0 = *reinterpret_cast<const f32x4*>(dlb + team * MF_DLB_TEAM + r * MF_DLB_ROW + 8 * g);
        const f32x4 d1 = *reinterpret_cast<const f32x4*>(dlb + team * MF_DLB_TEAM + r * MF_DLB_ROW + 8 * g + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { bdl[e] = (bf16)d0[e]; bdl[e + 4] = (bf16)d1[e]; }
      }
#pragma unroll
      for (int tp = 0; tp < Q / 32; ++tp) {
        const int f0 = w * Q + tp * 32;
        const bf16x8 av = xs[tp];
        f32x4 d[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          // A row m = lane & 15 of tile half h is feature f0 + 8(m >> 2) + 4h + (m & 3): the
          // lane's two accumulators are features f0 + 8g .. +7 of its row (one 16-byte store)
          const int f = f0 + 8 * (r >> 2) + 4 * h + (r & 3);
          const bf16x8 wa = g < 2 ? *reinterpret_cast<const bf16x8*>(wt + mf_wt_off(f, g)) : zero8;
          d[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bdl, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
        if (valid) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            o[j] = (bf16)(d[0][j] * act_bwd_t<ACT>((float)av[j]));
            o[j + 4] = (bf16)(d[1][j] * act_bwd_t<ACT>((float)av[j + 4]));
          }
          *reinterpret_cast<bf16x8*>(DZ + (long long)row * in + f0 + 8 * g) = o;
        }
      }
    }
    if (base == g_beg) stamp(4);
    // the next iteration's activations (xs stays live for the stage writes below)
    const bool more = base + MF_TEAMS < g_end;
    if (more) mh_load<Q, LOSS>(nxt, p, A, min((base + MF_TEAMS + team) * 16 + r, p.rows - 1), w, g);
    // ---- weight gradient: A = dl[rows 8g .. 8g+7 of the 32][o = r] as hi + lo ----
    bf16x8 ahi, alo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * g + e;   // block row 0..31: group k >> 4, row k & 15
      const float v = dlb[(k >> 4) * MF_DLB_TEAM + (k & 15) * MF_DLB_ROW + r];
      if (wv == 0) bsum += v;
      ahi[e] = (bf16)v;
      alo[e] = (bf16)(v - (float)ahi[e]);
    }
#pragma unroll
    for (int ph = 0; ph < NPH; ++ph) {
      // stage the two groups' activations of this phase's columns (the waves whose quarter
      // lies in it): row k = 16 t + r, columns of xs[c]
      if (w / QPP == ph) {
#pragma unroll
        for (int c = 0; c < Q / 32; ++c) {
          const int x = (w % QPP) * Q + c * 32 + 8 * g;
          *reinterpret_cast<bf16x8*>(stage + mf_stage_off(team * 16 + r, x)) = xs[c];
        }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 bv = mf_stage_frag(stage, (wv * 4 + t) * 16, lane);
        gacc[ph][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bv, gacc[ph][t], 0, 0, 0);
        gacc[ph][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bv, gacc[ph][t], 0, 0, 0);
      }
      __syncthreads();   // the stage / partial / dl buffers are rewritten next
      if (base == g_beg) stamp(5 + ph);
    }
    if (more) cur = nxt;
  }
  // ---- block partials: every gW element has one owner lane (o = 4g + i, column l & 15).  The
  // accumulators go through LDS (the W images are dead: the loop ended on a barrier) as a
  // [16][in] fp32 image, then every thread stores whole 16-byte row pieces: 5 coalesced stores
  // per thread at in = 1024, out = 10 instead of 32 scattered 4-byte ones per lane ----
  float* gimg = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int ph = 0; ph < NPH; ++ph)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        gimg[(4 * g + i) * (in + MF_GROW_PAD) + ph * MF_PH + (wv * 4 + t) * 16 + r] = gacc[ph][t][i];
  __syncthreads();
  {
    const int n4 = out * in / 4, r4 = in / 4;
    float* dst = gws + (long long)blockIdx.x * out * in;
    for (int v = tid; v < n4; v += 64 * MF_WAVES)
      reinterpret_cast<f32x4*>(dst)[v] =
          *reinterpret_cast<const f32x4*>(gimg + (v / r4) * (in + MF_GROW_PAD) + 4 * (v % r4));
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
  stamp(7);
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

// blocks of the fused head: one 2-group iteration per block up to a cap; the cap trades the
// partial-slab volume (out x in fp32 per block, written here and read by the combine) and the
// per-block W image build against parallelism (NNMPI_HEAD_BLOCKS, experiments)
static int head_mo_cap() {
  static int cap = -1;
  if (cap < 0) {
    const char* e = knob_env("NNMPI_HEAD_BLOCKS");
    // (clamped to the loss-partial count head_fwd_parts sizes the workspace for, MH_MAX_BLOCKS:
    // a larger cap would write loss partials past it, into the weight-gradient slabs)
    cap = (e && atoi(e) > 0) ? std::min(atoi(e), 256) : 256;
  }
  return cap;
}

static int head_mo_blocks(int rows) {
  return std::max(1, std::min(head_mo_cap(), ((rows + 15) / 16 + MF_TEAMS - 1) / MF_TEAMS));
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
                                   float* gwsb, unsigned long long* st, hipStream_t s) {
  const size_t smem = (size_t)MfLds<4 * Q>::BYTES;
  using Fn = void (*)(HeadArgs, float*, float*, unsigned long long*);
  static const Fn fns[2][3] = {
      {head_mo_fused_kernel<ACT_NONE, LOSS_MSE, Q>, head_mo_fused_kernel<ACT_RELU, LOSS_MSE, Q>, head_mo_fused_kernel<ACT_TANH, LOSS_MSE, Q>},
      {head_mo_fused_kernel<ACT_NONE, LOSS_XENT, Q>, head_mo_fused_kernel<ACT_RELU, LOSS_XENT, Q>, head_mo_fused_kernel<ACT_TANH, LOSS_XENT, Q>}};
  static bool attr[2][3] = {};
  const int li = loss == LOSS_XENT ? 1 : 0, ai = act == ACT_RELU ? 1 : act == ACT_TANH ? 2 : 0;
  if (!attr[li][ai]) {
    (void)hipFuncSetAttribute((const void*)fns[li][ai], hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr[li][ai] = true;
  }
  hipLaunchKernelGGL(fns[li][ai], dim3(blocks), dim3(64 * MF_WAVES), smem, s, h, gws, gwsb, st);
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
                         const SgdFuse* sgd, SlabReduce* pending, unsigned long long* stamps) {
  if (!head_mo_fused_ok(1, rows, in, out, loss)) return hipErrorInvalidValue;
  if ((loss == LOSS_XENT && !labels) || (loss == LOSS_MSE && !y)) return hipErrorInvalidValue;
  const int G = head_mo_blocks(rows);
  float* gws = ws;
  float* gwsb = ws + (size_t)G * out * in;
  HeadArgs h{a, rows, in, W, b, out, y, labels, inv_count, act_prev, dz_prev, nullptr, loss_part, 1};
  hipError_t e = in == 512 ? head_mo_launch_q<128>(h, act_prev, loss, G, gws, gwsb, stamps, s)
                           : head_mo_launch_q<256>(h, act_prev, loss, G, gws, gwsb, stamps, s);
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
