// bf16 MFMA GEMM for gfx950 with fused MLP epilogues.
//
//   C[m][n] = sum_k A(m,k) * B(k,n)      (bf16 inputs, fp32 accumulation)
//
// Operand storage is a template parameter per operand:
//   KMAJ : element (x,k) at base[x*ld + k]   (k contiguous)       -> LDS [x][64k], ds_read_b128
//   XMAJ : element (x,k) at base[k*ld + x]   (x contiguous)       -> LDS [64k][x], ds_read_b64_tr_b16
// which covers the three MLP orientations without materialising transposes:
//   forward  Z  = X  . W^T   A=X  KMAJ, B=W  KMAJ   epilogue act(acc + bias) -> bf16
//   dgrad    dX = dZ . W     A=dZ KMAJ, B=W  XMAJ   epilogue acc * act'(a_prev) -> bf16
//   wgrad    dW = dZ^T . X   A=dZ XMAJ, B=X  XMAJ   epilogue fp32 split-K slab (+ bias grad)
//
// Reference ops replaced: K1/K2 (addmm+relu), K8/K9 (mm+threshold_backward),
// K6/K7/K10 (mm(dZ^T,X) + sum(dZ,0)) of ref.py:170,176.
//
// Design (cdna_hip_programming.md §3, §5): 256 threads = 4 waves in a 2x2 grid, each wave owns
// a (BM/2)x(BN/2) sub-tile of 16x16 MFMA tiles (v_mfma_f32_16x16x32_bf16).  The MFMA is issued
// with swapped operands (B fragment first) so each lane ends with 4 CONSECUTIVE n values of one
// row: 8-byte bf16 / 16-byte fp32 epilogue stores.  BK = 64, two LDS stages, register-staged
// global->LDS copies issued one tile ahead.  LDS images are XOR-swizzled at 16-byte granularity
// (conflict-free for the b128 row reads and the tr_b16 transposed reads; checked with the §LDS
// bank model).  Blocks are remapped so consecutive tiles share an XCD (T1).  The wgrad bias
// gradient (row sums of dZ^T) rides on the same A fragments through one extra MFMA against a
// ones operand in the n-tile-0 blocks.
#include "gemm_tiles.h"
#include "knobs.h"

namespace nnmpi {

static int g_stage_epi = -1;   // NNMPI_STAGE_EPI=1: LDS-staged 256x256 forward epilogue (A/B)
void set_stage_epi(int on) { g_stage_epi = on; }   // -1: re-read the environment
static int stage_epi() {
  if (g_stage_epi < 0) {
    const char* e = knob_env("NNMPI_STAGE_EPI");
    g_stage_epi = (e && e[0] == '1') ? 1 : 0;
  }
  return g_stage_epi;
}
static int g_sgd_serial = -1;   // NNMPI_SGD_SERIAL=<form> (experiments)
void set_sgd_epilogue(int form) { g_sgd_serial = form; }   // -1: re-read the environment
static int sgd_serial() {
  if (g_sgd_serial < 0) {
    const char* e = knob_env("NNMPI_SGD_SERIAL");
    g_sgd_serial = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 0;
  }
  return g_sgd_serial;
}
static int g_store_pol = 0;   // host: store16 policy the launches put in GemmParams (0 plain)

// Deterministic split-K / partial-slab combine (the three jobs a backward needs), 512-thread
// blocks (8 waves):
//   main blocks   out[m][n] = sum_z ws[z][m][n]     (float4 columns)
//   bias blocks   bout[m]   = sum_z bws[z][m]
//   one more block (optional)   *loss_out = loss_scale * sum_i loss_part[i]
// WS "virtual" waves split the S partials of a column group (virtual wave v sums z = v, v+WS,
// ... in order; WS is picked so that each lane issues ~8 independent loads) and are combined in
// order through LDS.  WS < 8: a block holds 8/WS column groups of 64; WS = 16: each physical
// wave runs two virtual waves.  Bitwise reproducible for a given (S, WS); the standalone launch
// and the grouped backward launch run this same body.
constexpr int SLAB_NW = 8;
constexpr int SLAB_THREADS = 64 * SLAB_NW;

template <int WS>
struct SlabShape {
  static constexpr int VPW = WS > SLAB_NW ? WS / SLAB_NW : 1;   // virtual waves per wave
  static constexpr int CG = WS >= SLAB_NW ? 1 : SLAB_NW / WS;   // column groups per block
  static constexpr int COLS = 64 * CG;                         // columns (float4 / scalars) per block
};

template <int WS>
__device__ __forceinline__ void slab_reduce_block(const SlabReduce& r, int b, int nb_main, int nb_bias,
                                                  f32x4* part) {
  using SS = SlabShape<WS>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cg = WS >= SLAB_NW ? 0 : w / WS;
  const int w0 = WS >= SLAB_NW ? w : w % WS;
  const bool combiner = (w0 == 0);
  if (b < nb_main) {
    const int N = r.N, nv = N >> 2;
    const long long nvec = (long long)r.M * nv;
    const long long v = ((long long)b * SS::CG + cg) * 64 + lane;
    long long m = 0, n = 0;
    if (v < nvec) {
      m = v / nv;
      n = (v % nv) * 4;
    }
    const float* p = r.ws + m * N + n;
    float* o = r.out + m * r.ldo + n;
    // the combiner's optimizer operands are loaded first, beside the slab loads
    const bool upd = combiner && v < nvec && r.sg.g_base && r.sgd_serial != 1;
    SgdPre4 pre{};
    if (upd) pre = sgd_pre4(r.sg, o);
#pragma unroll
    for (int j = 0; j < SS::VPW; ++j) {
      const int vw = w0 + j * SLAB_NW;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (v < nvec) {
#pragma unroll 8
        for (int z = vw; z < r.S; z += WS) acc += *reinterpret_cast<const f32x4*>(p + z * r.stride);
      }
      part[(cg * WS + vw) * 64 + lane] = acc;
    }
    __syncthreads();
    // The transposed weight image (pkd) wants 8 consecutive ROWS per 16 B; a lane holds 4
    // consecutive columns of one row.  When the block's columns are R whole rows (R = 2 / 4 / 8),
    // the new values go through LDS (after the partials: [R][N] bf16) and every thread stores
    // one R x 2-byte run per column, instead of 4 scattered 2-byte stores per lane.
    const int R = (SS::COLS * 4) / N;
    const bool pk_lds = r.pkd && r.sg.g_base && WS < SLAB_NW && (R == 2 || R == 4 || R == 8) &&
                        R * N == SS::COLS * 4 && N <= 2 * SLAB_THREADS;
    bf16* stash = reinterpret_cast<bf16*>(part + SLAB_NW * 64);
    if (combiner && v < nvec) {
      f32x4 t = part[cg * WS * 64 + lane];
#pragma unroll
      for (int k = 1; k < WS; ++k) t += part[(cg * WS + k) * 64 + lane];
      if (r.sg.g_base) {
        const f32x4 pn = upd ? sgd_apply4(r.sg, pre, t) : sgd_fused_store4(r.sg, o, t);
        if (r.pkf || (r.pkd && !pk_lds)) rb_pack_store4(r.pkf, pk_lds ? nullptr : r.pkd, (int)m, (int)n, r.M, r.N, pn);
        if (pk_lds) {
          bf16x4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = (bf16)pn[e];
          *reinterpret_cast<bf16x4*>(stash + (m % R) * N + n) = h;
        }
      } else {
        *reinterpret_cast<f32x4*>(o) = t;
      }
    }
    if (pk_lds) {
      __syncthreads();
      const long long m0 = (long long)b * SS::COLS * 4 / N;
      for (int c = threadIdx.x; c < N; c += SLAB_THREADS) {
        if (m0 >= r.M) break;
        bf16 col[8];
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) col[rr] = rr < R ? stash[rr * N + c] : (bf16)0.f;
        bf16* d = r.pkd + rb_pk_off(c, (int)m0, r.M);
        if (R == 8) *reinterpret_cast<bf16x8*>(d) = bf16x8{col[0], col[1], col[2], col[3], col[4], col[5], col[6], col[7]};
        else if (R == 4) *reinterpret_cast<bf16x4*>(d) = bf16x4{col[0], col[1], col[2], col[3]};
        else *reinterpret_cast<bf16x2*>(d) = bf16x2{col[0], col[1]};
      }
    }
    return;
  }
  float* ps = reinterpret_cast<float*>(part);
  if (b < nb_main + nb_bias) {
    const long long m = ((long long)(b - nb_main) * SS::CG + cg) * 64 + lane;
#pragma unroll
    for (int j = 0; j < SS::VPW; ++j) {
      const int vw = w0 + j * SLAB_NW;
      float acc = 0.f;
      if (m < r.M) {
#pragma unroll 8
        for (int z = vw; z < r.S; z += WS) acc += r.bws[z * r.bstride + m];
      }
      ps[(cg * WS + vw) * 64 + lane] = acc;
    }
    __syncthreads();
    if (combiner && m < r.M) {
      float t = ps[cg * WS * 64 + lane];
#pragma unroll
      for (int k = 1; k < WS; ++k) t += ps[(cg * WS + k) * 64 + lane];
      if (r.sg.g_base) sgd_fused_store(r.sg, r.bout + m, t);
      else r.bout[m] = t;
    }
    return;
  }
  // loss partials: strided per-thread sums, wave sums, then a fixed-order combine
  float acc = 0.f;
  for (int i = threadIdx.x; i < r.n_loss_part; i += SLAB_THREADS) acc += r.loss_part[i];
  acc = wave_sum(acc);
  if (lane == 0) ps[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < SLAB_NW; ++k) t += ps[k];
    *r.loss_out = t * r.loss_scale;
  }
}

// Deep combine (S > 64 partials: one per row band / per head block): a block sums DEEP_COLS
// columns over DEEP_Q lane groups (group q sums z = q, q + DEEP_Q, ... in order; the groups are
// then combined in order through LDS).  A block reads S x 16 x 16 B (64 KiB at S = 256) instead
// of the 64-column form's 256 KiB, so the combine spreads over 16x more blocks (the 256-slab
// head combine ran on 40 blocks).  Selected by slab_ws() == SLAB_DEEP; bitwise reproducible.
constexpr int SLAB_DEEP = 32, DEEP_COLS = 16, DEEP_Q = SLAB_THREADS / DEEP_COLS;

__device__ __forceinline__ void slab_reduce_deep_block(const SlabReduce& r, int b, int nb_main,
                                                       int nb_bias, f32x4* part) {
  const int c = threadIdx.x % DEEP_COLS, q = threadIdx.x / DEEP_COLS;
  if (b < nb_main) {
    const int nv = r.N >> 2;
    const long long nvec = (long long)r.M * nv;
    const long long v = (long long)b * DEEP_COLS + c;
    const bool live = v < nvec;
    const long long m = live ? v / nv : 0, n = live ? (v % nv) * 4 : 0;
    const float* p = r.ws + m * r.N + n;
    float* o = r.out + m * r.ldo + n;
    const bool upd = q == 0 && live && r.sg.g_base;
    SgdPre4 pre{};
    if (upd) pre = sgd_pre4(r.sg, o);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (live) {
#pragma unroll 8
      for (int z = q; z < r.S; z += DEEP_Q) acc += *reinterpret_cast<const f32x4*>(p + z * r.stride);
    }
    part[q * DEEP_COLS + c] = acc;
    __syncthreads();
    if (q == 0 && live) {
      f32x4 t = part[c];
#pragma unroll 8
      for (int k = 1; k < DEEP_Q; ++k) t += part[k * DEEP_COLS + c];
      if (upd) {
        const f32x4 pn = sgd_apply4(r.sg, pre, t);
        if (r.pkf || r.pkd) rb_pack_store4(r.pkf, r.pkd, (int)m, (int)n, r.M, r.N, pn);
      } else {
        *reinterpret_cast<f32x4*>(o) = t;
      }
    }
    return;
  }
  float* ps = reinterpret_cast<float*>(part);
  if (b < nb_main + nb_bias) {
    const long long m = (long long)(b - nb_main) * DEEP_COLS + c;
    float acc = 0.f;
    if (m < r.M) {
#pragma unroll 8
      for (int z = q; z < r.S; z += DEEP_Q) acc += r.bws[z * r.bstride + m];
    }
    ps[q * DEEP_COLS + c] = acc;
    __syncthreads();
    if (q == 0 && m < r.M) {
      float t = ps[c];
#pragma unroll 8
      for (int k = 1; k < DEEP_Q; ++k) t += ps[k * DEEP_COLS + c];
      if (r.sg.g_base) sgd_fused_store(r.sg, r.bout + m, t);
      else r.bout[m] = t;
    }
    return;
  }
  // loss partials: the same fixed-order form as slab_reduce_block's
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (int i = threadIdx.x; i < r.n_loss_part; i += SLAB_THREADS) acc += r.loss_part[i];
  acc = wave_sum(acc);
  if (lane == 0) ps[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < SLAB_NW; ++k) t += ps[k];
    *r.loss_out = t * r.loss_scale;
  }
}

constexpr int SLAB_PART_BYTES = 16 * 64 * 16;   // max(WS, NW) x 64 lanes x f32x4

template <int WS>
__global__ void __launch_bounds__(SLAB_THREADS) slab_reduce_kernel(SlabReduce r, int nb_main, int nb_bias) {
  __shared__ f32x4 part[SLAB_PART_BYTES / 16];
  if constexpr (WS == SLAB_DEEP) slab_reduce_deep_block(r, blockIdx.x, nb_main, nb_bias, part);
  else slab_reduce_block<WS>(r, blockIdx.x, nb_main, nb_bias, part);
}

__device__ __forceinline__ void slab_reduce_any(int ws, const SlabReduce& r, int b, int nb_main,
                                                int nb_bias, f32x4* part) {
  switch (ws) {
    case 1: slab_reduce_block<1>(r, b, nb_main, nb_bias, part); break;
    case 2: slab_reduce_block<2>(r, b, nb_main, nb_bias, part); break;
    case 4: slab_reduce_block<4>(r, b, nb_main, nb_bias, part); break;
    case 8: slab_reduce_block<8>(r, b, nb_main, nb_bias, part); break;
    case 16: slab_reduce_block<16>(r, b, nb_main, nb_bias, part); break;
    default: slab_reduce_deep_block(r, b, nb_main, nb_bias, part); break;
  }
}

// Grouped backward launch (see bwd_group): dgrad tiles, then wgrad (tile, split) blocks, then
// the previous layer's combine blocks.  GEMM segments are padded to multiples of 8 blocks so the
// XCD remap inside each segment sees the hardware's round-robin XCD assignment.
struct BwdGroupParams {
  GemmParams dg;
  int dg_gx, dg_n, dg_blocks;
  GemmParams wg;
  int wg_gx, wg_tiles, wg_n, wg_blocks;
  SlabReduce red;
  int red_ws, nb_main, nb_bias;
};

constexpr int GRP_BM = 128, GRP_BN = 128, GRP_WGM = 2, GRP_WGN = 4, GRP_NS = 2;
constexpr int GRP_THREADS = 64 * GRP_WGM * GRP_WGN;
constexpr int GRP_SMEM = GRP_NS * (GRP_BM + GRP_BN) * GEMM_BK * 2;

// GA: LDS read mode of the two GEMM jobs (dma_gemm_tile ASYNC_TR).  Two 64 KiB / 512-thread
// blocks per CU (4 waves per SIMD) is what lets one block's DMA wait hide behind the other's
// MFMAs, so the register budget is pinned to 128 VGPRs (launch bound: 4 waves per SIMD).
template <int ACT, int GA>
__global__ void __launch_bounds__(GRP_THREADS, 4) bwd_group_kernel(BwdGroupParams g) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  int bid = blockIdx.x;
  if (bid < g.dg_blocks) {
    const int l = xcd_remap(bid, g.dg_blocks);
    if (l >= g.dg_n) return;
    dma_gemm_tile<GRP_BM, GRP_BN, GRP_WGM, GRP_WGN, KMAJ, XMAJ, EPI_DACT, ACT, false, GRP_NS, GA>(
        g.dg, smem, l % g.dg_gx, l / g.dg_gx, 0);
    return;
  }
  bid -= g.dg_blocks;
  if (bid < g.wg_blocks) {
    const int l = xcd_remap(bid, g.wg_blocks);
    if (l >= g.wg_n) return;
    const int split = l / g.wg_tiles, t = l % g.wg_tiles;
    dma_gemm_tile<GRP_BM, GRP_BN, GRP_WGM, GRP_WGN, XMAJ, XMAJ, EPI_F32, ACT_NONE, true, GRP_NS, GA>(
        g.wg, smem, t % g.wg_gx, t / g.wg_gx, split);
    return;
  }
  bid -= g.wg_blocks;
  slab_reduce_any(g.red_ws, g.red, bid, g.nb_main, g.nb_bias, reinterpret_cast<f32x4*>(smem));
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static int g_gemm_impl = -1;

static int gemm_impl() {
  if (g_gemm_impl < 0) {
    const char* e = knob_env("NNMPI_GEMM");
    g_gemm_impl = (e && e[0] == '1') ? 1 : 2;   // 2 = LDS-DMA ring (default), 1 = register-staged
  }
  return g_gemm_impl;
}

void set_gemm_impl(int impl) { g_gemm_impl = impl; }
int get_gemm_impl() { return gemm_impl(); }


template <int BM, int BN, int WGM, int WGN, int NS, int LA, int LB, int EPI, int ACT, bool BG>
static hipError_t launch_dma(GemmParams p, int splits, hipStream_t s) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, splits);
  constexpr int smem = NS * (BM + BN) * GEMM_BK * 2;
  set_extents<LA, LB>(p);
  p.store_pol = g_store_pol;
  auto kfn = gemm_bf16_dma_kernel<BM, BN, WGM, WGN, LA, LB, EPI, ACT, BG, NS>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(64 * WGM * WGN), smem, s, p);
  return hipGetLastError();
}

// DMA-path variants (experiments select one with set_gemm_variant; 0 = default).
static int g_variant = 0;
void set_gemm_variant(int v) { g_variant = v; }
// 256x256 ping-pong kernel per epilogue (index into its kernel table: 0 GM 4, 1 row-major,
// 2 GM 4 + one DMA half per phase, 3 row-major + one half per phase): forward, dgrad, wgrad
static int g_pp_order[3] = {0, 0, 1};
void set_pp256_order(int epi, int idx) {
  if (epi >= 0 && epi < 3 && idx >= 0 && idx < 4) g_pp_order[epi] = idx;
}

// Prefetch of the fused SGD update's operands in the 256x256 weight gradient (pp256_tile PF):
// 0 off, 1 default cache policy, 2 nt.  NNMPI_PP_PREFETCH (experiments) / set_pp_prefetch A/B.
static int g_pp_prefetch = -2;
constexpr int PP_PREFETCH_DEFAULT = 0;
void set_pp_prefetch(int v) { g_pp_prefetch = (v >= 0 && v <= 2) ? v : -1; }
static int pp_prefetch() {
  if (g_pp_prefetch == -2) {
    const char* e = knob_env("NNMPI_PP_PREFETCH");
    g_pp_prefetch = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : -1;
  }
  return g_pp_prefetch >= 0 ? g_pp_prefetch : PP_PREFETCH_DEFAULT;
}

// Kernel-selection knobs of the training step (scripts/step_ab.py A/Bs them; -1 / 0 = default).
static int g_fwd_variant = -1;    // forward GEMM main-loop variant (launch_t's switch)
static int g_group_async = -1;    // grouped-backward LDS read mode (dma_gemm_tile ASYNC_TR)
static int g_wgrad_splits = 0;    // > 0: upper bound on the weight-gradient split-K factor
constexpr int FWD_VARIANT_DEFAULT = 0;
constexpr int GROUP_ASYNC_DEFAULT = 2;   // measured: 102.3 -> 97.9 us/step (proxy512, step_ab)
constexpr int WGM_ASYNC_DEFAULT = 2;     // wgrad_multi (row-band step); 3 = pipelined k-halves
void set_fwd_variant(int v) { g_fwd_variant = v; }
void set_group_async(int m) { g_group_async = m; }
void set_wgrad_splits(int s) { g_wgrad_splits = s; }
void set_store_policy(int p) { g_store_pol = p; }
// Store policy of the split-K weight-gradient slabs alone in the grouped backward (A/B,
// NNMPI_SLAB_STORE=<0|1|2>; -1 = the general policy above).  The slabs are read back by the NEXT
// launch's combine from every XCD, so their dirty lines are written back at the launch boundary
// ("boundary" row, MI355X_MICROARCH.md: + B / 6 TB/s); write-through (2 = sc1) moves that
// traffic into the epilogue, where other CUs' main loops may hide it.
static int g_slab_store_pol = -2;
void set_slab_store_policy(int p) { g_slab_store_pol = p; }
static int slab_store_pol() {
  if (g_slab_store_pol == -2) {
    const char* e = knob_env("NNMPI_SLAB_STORE");
    g_slab_store_pol = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : -1;
  }
  return g_slab_store_pol >= 0 ? g_slab_store_pol : g_store_pol;
}

template <int BM, int BN, int LA, int LB, int EPI, int ACT, bool BG>
static hipError_t launch_t(GemmParams p, int splits, hipStream_t s, int variant = -1) {
  if (variant < 0) variant = g_variant;
  if constexpr (BM == 256 && BN == 256) {
    // large shapes: 256x256 tile, 8 waves (each 128x64), 128 KiB LDS, 1 block/CU
    if (variant == 9) return launch_dma<256, 256, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
    dim3 grid((p.N + 255) / 256, (p.M + 255) / 256, splits);
    set_extents<LA, LB>(p);
    // default: reads retired after the barrier, grouped tile order GM 4 (forward, dgrad) or
    // row-major (weight gradient: XMAJ x XMAJ, 4 waves of tiles at 8192 wide, measured 2-3 %
    // faster that way: profiles/gemm_wide8192_pp256_variants.json); each also with one DMA
    // half per phase (ISSUE 1).  Table index = set_pp256_order idx; variants 15..18 pick one.
    using K = void (*)(GemmParams);
    static const K kfns[4] = {gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 4, 0>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 1, 0>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 4, 1>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 1, 1>};
    const int dflt = g_pp_order[EPI];
    static bool attr = false;
    if (!attr) {
      for (K f : kfns)
        (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_SMEM);
      attr = true;
    }
    if (variant >= 19 && variant <= 24) {
      // the deep-ring twin lives in csrc/experiments (NNMPI_BUILD_EXPERIMENTS=1 builds)
      if (!exp_pp256_ring) return hipErrorNotSupported;
      return exp_pp256_ring(variant, LA, LB, EPI, ACT, BG, p, grid, s);
    }
    if constexpr (EPI == EPI_F32) {
      // weight gradient + fused SGD: the update operands prefetched during the main loop
      const int pf = pp_prefetch();
      if (pf > 0 && variant == 0 && dflt == 1 && p.sg.g_base && !p.c16 && p.sgd_serial == 0) {
        static const K pfns[2] = {gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 1, 0, 1>,
                                  gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 1, 0, 2>};
        static bool pattr = false;
        if (!pattr) {
          for (K f : pfns)
            (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      PP_PF_SMEM);
          pattr = true;
        }
        hipLaunchKernelGGL(pfns[pf - 1], grid, dim3(PP_THREADS), PP_PF_SMEM, s, p);
        return hipGetLastError();
      }
    }
    const K kfn = kfns[(variant >= 15 && variant <= 18) ? variant - 15 : dflt];
    hipLaunchKernelGGL(kfn, grid, dim3(PP_THREADS), PP_SMEM, s, p);
    return hipGetLastError();
  } else {
  if (gemm_impl() == 2) {
    if constexpr (BM == 128 && BN == 128) {
      switch (variant) {
        case 1: return launch_dma<128, 128, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 2: return launch_dma<128, 128, 2, 4, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 3: return launch_dma<128, 128, 4, 2, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 4: return launch_dma<128, 128, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 5: return launch_dma<64, 128, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);  // 2 blocks/CU
        case 6: return launch_dma<128, 64, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 7: return launch_dma<64, 128, 2, 4, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 8: return launch_dma<128, 128, 2, 2, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
        // rectangular tiles (0.75x the L2->LDS bytes per FLOP of 128x128) for shapes with
        // >= 256 of them
        case 10: return launch_dma<256, 128, 4, 2, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 11: return launch_dma<128, 256, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 12: return launch_dma<256, 128, 4, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 13: return launch_dma<128, 256, 2, 4, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        default: return launch_dma<128, 128, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);  // = variant 4
      }
    } else {
      return launch_dma<BM, BN, 2, 2, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
    }
  }
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, splits);
  constexpr int smem = 2 * (BM + BN) * GEMM_BK * 2;
  auto kfn = gemm_bf16_kernel<BM, BN, LA, LB, EPI, ACT, BG>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(GEMM_THREADS), smem, s, p);
  return hipGetLastError();
  }
}

template <int BM, int BN, int LA, int LB, int EPI, bool BG>
static hipError_t launch_act(const GemmParams& p, int act, int splits, hipStream_t s,
                             int variant = -1) {
  const int v = variant >= 0 ? variant : g_variant;
  switch (act) {
    case ACT_RELU: return launch_t<BM, BN, LA, LB, EPI, ACT_RELU, BG>(p, splits, s, v);
    case ACT_TANH: return launch_t<BM, BN, LA, LB, EPI, ACT_TANH, BG>(p, splits, s, v);
    default: return launch_t<BM, BN, LA, LB, EPI, ACT_NONE, BG>(p, splits, s, v);
  }
}

static int g_force_tile = 0;  // 0 = heuristic; 64 / 128 force a tile edge (experiments)
void set_gemm_tile(int t) { g_force_tile = t; }
bool gemm_host::default_path() { return gemm_impl() == 2 && g_force_tile == 0 && g_variant == 0; }
using gemm_host::make_wgrad;
using gemm_host::pick_tile;
using gemm_host::wgrad_tile;

int gemm_host::pick_tile(int M, int N) {
  if (g_force_tile) return g_force_tile;
  // 256x256 once that alone fills the chip, 128x128 when that yields ~a full wave of blocks,
  // else 64x64.
  const long long t256 = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if (t256 >= 256 && gemm_impl() == 2) return 256;
  const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128);
  return t128 >= 192 ? 128 : 64;
}

hipError_t linear_fwd_bf16(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                           bf16* Y, int ldy, int M, int N, int K, int act, hipStream_t s) {
  GemmParams p{};
  p.A = X; p.lda = ldx; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = Y; p.ldc = ldy; p.bias = bias;
  const int t = pick_tile(M, N);
  p.stage_epi = stage_epi();
  if (t == 256) return launch_act<256, 256, KMAJ, KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s);
  if (t == 128) {
    const int v = g_variant != 0 ? g_variant : g_fwd_variant >= 0 ? g_fwd_variant : FWD_VARIANT_DEFAULT;
    return launch_act<128, 128, KMAJ, KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s, v);
  }
  return launch_act<64, 64, KMAJ, KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s);
}

hipError_t linear_dgrad_bf16(const bf16* dZ, int lddz, const bf16* W, int ldw, const bf16* Aprev,
                             int lda_prev, bf16* dX, int lddx, int M, int N, int K, int act,
                             hipStream_t s) {
  GemmParams p{};
  p.A = dZ; p.lda = lddz; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = dX; p.ldc = lddx; p.aux = Aprev; p.ldaux = lda_prev;
  const int t = pick_tile(M, N);
  if (t == 256) return launch_act<256, 256, KMAJ, XMAJ, EPI_DACT, false>(p, act, 1, s);
  if (t == 128) return launch_act<128, 128, KMAJ, XMAJ, EPI_DACT, false>(p, act, 1, s);
  return launch_act<64, 64, KMAJ, XMAJ, EPI_DACT, false>(p, act, 1, s);
}

int gemm_host::wgrad_tile(int M, int N) {
  if (g_force_tile) return g_force_tile;
  const long long t256 = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if (t256 >= 256 && gemm_impl() == 2) return 256;
  return (M >= 128 && N >= 128) ? 128 : 64;
}

int wgrad_splits(int M, int N, int K) {
  // split the (long) batch reduction until ~one block per CU; keep >= 4 k-steps per split
  const int t = wgrad_tile(M, N);
  const int tiles = ((M + t - 1) / t) * ((N + t - 1) / t);
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  int s = 1;
  while (tiles * s < 256 && ksteps / (s * 2) >= 4 && s < 64) s *= 2;
  if (g_wgrad_splits > 0 && g_wgrad_splits < s) s = g_wgrad_splits;  // experiments: fewer slabs
  return s;
}

size_t wgrad_workspace_bytes(int M, int N, int K) {
  const int s = wgrad_splits(M, N, K);
  if (s == 1) return 0;
  return (size_t)s * ((size_t)M * N + M) * sizeof(float);
}

// GEMM parameters of a weight gradient and the split-K combine it needs (pending.S == 0: the
// GEMM writes dW / db directly).
static int make_wgrad_s(const WgradArgs& a, GemmParams& p, SlabReduce& pending, int want) {
  // dW[M=out][N=in] = sum_k dZ[k][m] X[k][n]; db[m] = sum_k dZ[k][m].
  const int M = a.M, N = a.N, K = a.K;
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  // (the split count actually used: every split holds k_per_split k-steps, the last one fewer)
  const int kps = (ksteps + want - 1) / want;
  const int splits = std::max(1, (ksteps + kps - 1) / kps);
  p = GemmParams{};
  p.sgd_serial = sgd_serial();
  p.A = a.dZ; p.lda = a.lddz; p.B = a.X; p.ldb = a.ldx; p.M = M; p.N = N; p.K = K;
  p.k_per_split = kps * GEMM_BK;
  pending = SlabReduce{};
  if (splits == 1) {
    p.C = a.dW; p.ldc = N; p.c_split_stride = 0;
    p.bias_grad = a.db; p.bg_split_stride = 0;
    p.sg = a.sg;          // (g_base null: plain gradient store)
    p.c16 = a.dW16; p.bg16 = a.db16;
    return splits;
  }
  p.C = a.ws; p.ldc = N; p.c_split_stride = (long long)M * N;
  float* bws = a.ws + (size_t)splits * M * N;
  p.bias_grad = a.db ? bws : nullptr; p.bg_split_stride = M;
  pending.ws = a.ws; pending.S = splits; pending.stride = (long long)M * N; pending.M = M;
  pending.N = N; pending.out = a.dW; pending.ldo = N;
  if (a.db) { pending.bws = bws; pending.bstride = M; pending.bout = a.db; }
  pending.sg = a.sg;
  return splits;
}

int gemm_host::make_wgrad(const WgradArgs& a, GemmParams& p, SlabReduce& pending) {
  return make_wgrad_s(a, p, pending, wgrad_splits(a.M, a.N, a.K));
}

hipError_t linear_wgrad_bf16_deferred(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                                      float* db, int M, int N, int K, float* ws, hipStream_t s,
                                      const SgdFuse* sgd, SlabReduce* pending) {
  return linear_wgrad_bf16_ex(dZ, lddz, X, ldx, dW, db, M, N, K, ws, s, sgd, pending, nullptr,
                              nullptr);
}

hipError_t linear_wgrad_bf16_ex(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                                float* db, int M, int N, int K, float* ws, hipStream_t s,
                                const SgdFuse* sgd, SlabReduce* pending, bf16* dW16, bf16* db16) {
  WgradArgs a{dZ, lddz, X, ldx, dW, db, M, N, K, ws, SgdFuse{}, dW16, db16};
  if (sgd) a.sg = *sgd;
  if (dW16 && (sgd || wgrad_splits(M, N, K) > 1)) return hipErrorInvalidValue;
  GemmParams p;
  SlabReduce r;
  const int splits = make_wgrad(a, p, r);
  if (splits > 1 && ws == nullptr) return hipErrorInvalidValue;
  hipError_t e;
  const int wt = wgrad_tile(M, N);
  const bool bg = db != nullptr || db16 != nullptr;
  if (wt == 256) e = bg ? launch_t<256, 256, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, splits, s)
                        : launch_t<256, 256, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, splits, s);
  else if (wt == 128) e = bg ? launch_t<128, 128, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, splits, s)
                             : launch_t<128, 128, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, splits, s);
  else e = bg ? launch_t<64, 64, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, splits, s)
              : launch_t<64, 64, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, splits, s);
  if (e != hipSuccess) return e;
  if (pending) {
    *pending = r;
    return hipSuccess;
  }
  return r.S > 0 ? slab_reduce(r, s) : hipSuccess;
}

bool wgrad_defer_ok(int M, int N, int K) {
  return gemm_impl() == 2 && g_force_tile == 0 && g_variant == 0 && sgd_serial() == 0 &&
         wgrad_tile(M, N) == 256 && M % 256 == 0 && N % 256 == 0 && wgrad_splits(M, N, K) == 1;
}

hipError_t linear_wgrad_bf16_out16_defer(const bf16* dZ, int lddz, const bf16* X, int ldx, bf16* dW16,
                                         bf16* db16, int M, int N, int K, const SgdFuse& other,
                                         const bf16* g16o, hipStream_t s) {
  if (!wgrad_defer_ok(M, N, K) || !dW16 || !db16 || !g16o || !other.p_base) return hipErrorInvalidValue;
  WgradArgs a{dZ, lddz, X, ldx, nullptr, nullptr, M, N, K, nullptr, SgdFuse{}, dW16, db16};
  GemmParams p;
  SlabReduce r;
  make_wgrad(a, p, r);
  p.sg2 = other;
  p.g16o = g16o;
  return launch_t<256, 256, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, 1, s);
}

hipError_t linear_wgrad_bf16(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                             float* db, int M, int N, int K, float* ws, hipStream_t s,
                             const SgdFuse* sgd) {
  return linear_wgrad_bf16_deferred(dZ, lddz, X, ldx, dW, db, M, N, K, ws, s, sgd, nullptr);
}

hipError_t gemm_bf16_generic(const bf16* A, int lda, int la, const bf16* B, int ldb, int lb,
                             int M, int N, int K, float* C, int ldc, hipStream_t s);

hipError_t gemm_bf16_generic_tile(const bf16* A, int lda, int la, const bf16* B, int ldb, int lb,
                                  int M, int N, int K, float* C, int ldc, int tile, hipStream_t s) {
  // The same plain GEMM through the 256x256 ping-pong kernel (tile 256) or the 128x128 DMA
  // kernel (tile 128): operand-layout experiments on the production tiles.
  if (tile != 256 && tile != 128) return gemm_bf16_generic(A, lda, la, B, ldb, lb, M, N, K, C, ldc, s);
  GemmParams p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = C; p.ldc = ldc;
#define NNMPI_GT(T)                                                                              \
  if (la == KMAJ && lb == KMAJ) return launch_t<T, T, KMAJ, KMAJ, EPI_F32, ACT_NONE, false>(p, 1, s); \
  if (la == KMAJ && lb == XMAJ) return launch_t<T, T, KMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, 1, s); \
  if (la == XMAJ && lb == KMAJ) return launch_t<T, T, XMAJ, KMAJ, EPI_F32, ACT_NONE, false>(p, 1, s); \
  return launch_t<T, T, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, 1, s);
  if (tile == 256) { NNMPI_GT(256) }
  NNMPI_GT(128)
#undef NNMPI_GT
}

hipError_t gemm_bf16_generic(const bf16* A, int lda, int la, const bf16* B, int ldb, int lb,
                             int M, int N, int K, float* C, int ldc, hipStream_t s) {
  // Plain fp32-output GEMM in any of the four layout combinations (testing / utility).
  GemmParams p{};
  p.A = A; p.lda = lda; p.B = B; p.ldb = ldb; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = C; p.ldc = ldc;
  if (la == KMAJ && lb == KMAJ) return launch_t<64, 64, KMAJ, KMAJ, EPI_F32, ACT_NONE, false>(p, 1, s);
  if (la == KMAJ && lb == XMAJ) return launch_t<64, 64, KMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, 1, s);
  if (la == XMAJ && lb == KMAJ) return launch_t<64, 64, XMAJ, KMAJ, EPI_F32, ACT_NONE, false>(p, 1, s);
  return launch_t<64, 64, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, 1, s);
}

static int slab_ws(const SlabReduce& r) {
  // more than 64 partials: the deep 16-column form
  if (r.S > 64) return SLAB_DEEP;
  // ~8 independent loads per lane: WS = S / 8 rounded up to a power of two, in [1, 16]
  int ws = 1;
  while (ws < 16 && ws * 8 < r.S) ws *= 2;
  return ws;
}

static int slab_cols(int ws) {
  return ws == SLAB_DEEP ? DEEP_COLS : ws >= SLAB_NW ? 64 : 64 * (SLAB_NW / ws);
}

static void slab_blocks(const SlabReduce& r, int& nb_main, int& nb_bias, int& nb) {
  const int cols = slab_cols(slab_ws(r));
  const long long nvec = (r.ws && r.out && r.S > 0) ? (long long)r.M * (r.N / 4) : 0;
  nb_main = (int)((nvec + cols - 1) / cols);
  nb_bias = (r.bws && r.bout && r.S > 0) ? (r.M + cols - 1) / cols : 0;
  nb = nb_main + nb_bias + (r.loss_out ? 1 : 0);
}

hipError_t slab_reduce(const SlabReduce& r0, hipStream_t s) {
  SlabReduce r = r0;
  r.sgd_serial = sgd_serial();
  int nb_main, nb_bias, nb;
  slab_blocks(r, nb_main, nb_bias, nb);
  if (nb == 0) return hipSuccess;
  const dim3 g(nb), t(SLAB_THREADS);
  switch (slab_ws(r)) {
    case 1: hipLaunchKernelGGL(slab_reduce_kernel<1>, g, t, 0, s, r, nb_main, nb_bias); break;
    case 2: hipLaunchKernelGGL(slab_reduce_kernel<2>, g, t, 0, s, r, nb_main, nb_bias); break;
    case 4: hipLaunchKernelGGL(slab_reduce_kernel<4>, g, t, 0, s, r, nb_main, nb_bias); break;
    case 8: hipLaunchKernelGGL(slab_reduce_kernel<8>, g, t, 0, s, r, nb_main, nb_bias); break;
    case 16: hipLaunchKernelGGL(slab_reduce_kernel<16>, g, t, 0, s, r, nb_main, nb_bias); break;
    default: hipLaunchKernelGGL(slab_reduce_kernel<SLAB_DEEP>, g, t, 0, s, r, nb_main, nb_bias); break;
  }
  return hipGetLastError();
}

hipError_t splitk_reduce(const float* ws, int S, long long stride, int M, int N, float* out, int ldo,
                         const float* bws, long long bstride, float* bout, const float* loss_part,
                         int n_loss_part, float loss_scale, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd) {
  SlabReduce r{ws, S, stride, M, N, out, ldo, bws, bstride, bout, loss_part, n_loss_part, loss_scale,
               loss_out, SgdFuse{}};
  if (sgd) r.sg = *sgd;
  return slab_reduce(r, s);
}

static int g_group = -1;   // grouped backward launch: 1 on (default), 0 off (NNMPI_GROUP=0)
void set_bwd_group(int on) { g_group = on; }
static bool group_enabled() {
  if (g_group < 0) {
    const char* e = knob_env("NNMPI_GROUP");
    g_group = (e && e[0] == '0') ? 0 : 1;
  }
  return g_group == 1;
}

bool bwd_group_supported(int rows, int out_f, int in_f) {
  // the grouped kernel covers the 128x128 tile shapes of the default DMA main loop
  // (small batches, whose standalone dgrad would take 64x64 tiles, run grouped too: the grouped
  // launch saves two launch boundaries per layer, which is what a small-batch step is made of;
  // the accumulation order does not depend on the tile, so results are identical)
  return group_enabled() && gemm_impl() == 2 && g_variant == 0 && pick_tile(rows, in_f) != 256 &&
         wgrad_tile(out_f, in_f) == 128;
}

hipError_t bwd_group(const DgradArgs* dg, const WgradArgs* wg, const SlabReduce* red,
                     SlabReduce* wg_pending, hipStream_t s) {
  if (wg_pending) *wg_pending = SlabReduce{};
  int nb_main = 0, nb_bias = 0, nbr = 0;
  if (red) slab_blocks(*red, nb_main, nb_bias, nbr);
  GemmParams pw{};
  SlabReduce pend{};
  int splits = 0;
  if (wg) splits = make_wgrad(*wg, pw, pend);
  // an un-split wgrad would apply the optimizer in its epilogue while dgrad_i (same launch, or
  // earlier in the fallback) still reads W_i: refuse instead of racing
  if (dg && wg && splits == 1 && wg->sg.g_base) return hipErrorInvalidValue;
  // the grouped kernel covers the 128x128 tile shapes of the default DMA main loop
  bool ok = group_enabled() && gemm_impl() == 2 && g_variant == 0;
  if (dg) ok = ok && pick_tile(dg->M, dg->N) != 256;
  if (wg) ok = ok && wgrad_tile(wg->M, wg->N) == 128 && wg->db != nullptr &&
               (splits == 1 || wg->ws != nullptr);
  if (!ok) {
    hipError_t e = hipSuccess;
    if (red && nbr) e = slab_reduce(*red, s);
    if (e == hipSuccess && dg)
      e = linear_dgrad_bf16(dg->dZ, dg->lddz, dg->W, dg->ldw, dg->Aprev, dg->lda_prev, dg->dX,
                            dg->lddx, dg->M, dg->N, dg->K, dg->act, s);
    if (e == hipSuccess && wg)
      e = linear_wgrad_bf16_deferred(wg->dZ, wg->lddz, wg->X, wg->ldx, wg->dW, wg->db, wg->M, wg->N,
                                     wg->K, wg->ws, s, &wg->sg, wg_pending);
    return e;
  }
  BwdGroupParams g{};
  if (dg) {
    GemmParams& p = g.dg;
    p.A = dg->dZ; p.lda = dg->lddz; p.B = dg->W; p.ldb = dg->ldw;
    p.M = dg->M; p.N = dg->N; p.K = dg->K;
    p.k_per_split = ((dg->K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
    p.C = dg->dX; p.ldc = dg->lddx; p.aux = dg->Aprev; p.ldaux = dg->lda_prev;
    set_extents<KMAJ, XMAJ>(p);
    g.dg_gx = (p.N + GRP_BN - 1) / GRP_BN;
    g.dg_n = g.dg_gx * ((p.M + GRP_BM - 1) / GRP_BM);
    g.dg_blocks = (g.dg_n + 7) & ~7;
  }
  if (wg) {
    set_extents<XMAJ, XMAJ>(pw);
    g.wg = pw;
    g.wg_gx = (pw.N + GRP_BN - 1) / GRP_BN;
    g.wg_tiles = g.wg_gx * ((pw.M + GRP_BM - 1) / GRP_BM);
    g.wg_n = g.wg_tiles * splits;
    g.wg_blocks = (g.wg_n + 7) & ~7;
    if (wg_pending) *wg_pending = pend;
  }
  if (red) {
    g.red = *red;
    g.red.sgd_serial = sgd_serial();
    g.red_ws = slab_ws(*red);
    g.nb_main = nb_main;
    g.nb_bias = nb_bias;
  }
  g.dg.store_pol = g_store_pol;
  g.wg.store_pol = splits > 1 ? slab_store_pol() : g_store_pol;
  const int nb = g.dg_blocks + g.wg_blocks + nbr;
  if (nb == 0) return hipSuccess;
  const int act = dg ? dg->act : ACT_NONE;
  const int ga = g_group_async >= 0 ? std::min(g_group_async, 2) : GROUP_ASYNC_DEFAULT;
  using GrpFn = void (*)(BwdGroupParams);
  static const GrpFn fns[3][3] = {
      {bwd_group_kernel<ACT_RELU, 0>, bwd_group_kernel<ACT_RELU, 1>, bwd_group_kernel<ACT_RELU, 2>},
      {bwd_group_kernel<ACT_TANH, 0>, bwd_group_kernel<ACT_TANH, 1>, bwd_group_kernel<ACT_TANH, 2>},
      {bwd_group_kernel<ACT_NONE, 0>, bwd_group_kernel<ACT_NONE, 1>, bwd_group_kernel<ACT_NONE, 2>}};
  static bool attr[3][3] = {};
  const int ai = act == ACT_RELU ? 0 : act == ACT_TANH ? 1 : 2;
  const GrpFn kfn = fns[ai][ga];
  if (!attr[ai][ga]) {
    (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, GRP_SMEM);
    attr[ai][ga] = true;
  }
  hipLaunchKernelGGL(kfn, dim3(nb), dim3(GRP_THREADS), GRP_SMEM, s, g);
  if (!wg_pending && wg && pend.S > 0) {   // caller does not defer: combine right away
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return slab_reduce(pend, s);
  }
  return hipGetLastError();
}

// ---- row-band step: all weight gradients in one launch, all combines in one launch -------
// (rowband.hip).  The weight-gradient jobs are the grouped backward's 128x128 split-K tiles
// (same tile body, same slab layout as the standalone launch); jobs follow each other in block
// order, each padded to a multiple of 8 blocks so its XCD remap sees the round-robin XCD
// assignment.
// In-launch split-K fixup of one job (FIX): the split that arrives LAST at a tile sums the S
// partial slabs in split order and applies the update (or stores the gradient).
struct WgmFix {
  float* out;    // dW [M][N] (ld N): the gradient's arena position (SGD: the update's operand)
  float* bout;   // db [M]
  SgdFuse sg;    // g_base set: apply SGD-momentum at those positions, else store the gradient
  bf16* pkf;     // with sg: the row-band v2 images of the updated W and W^T (null: none)
  bf16* pkd;
  int* cnt;      // one arrival counter per tile: zero between launches (the last arrival resets it)
  int S;         // splits
};

struct WgradMultiParams {
  GemmParams wg[RB_MAXL];
  int gx[RB_MAXL], tiles[RB_MAXL], n[RB_MAXL], blocks[RB_MAXL];
  int nj;
  unsigned long long* stamps;   // diagnostic: per block {start, end, XCC id, HW id} (null: off)
  WgmFix fix[RB_MAXL];          // FIX kernels only
  int gemm_blocks;              // FIX: blocks past this one run the extra combine `tail`
  SlabReduce tail;              // (the row-band head's per-band partials)
  int tail_ws, tail_nb_main, tail_nb_bias;
  const bf16* kA[RB_MAXL];      // wgrad_small's image path: K-major fragment images of dZ (A)
  const bf16* kB[RB_MAXL];      // and of the layer input (B); kbands bands
  int kbands;
  int gm;                       // image path: tile rows of an XCD's patch (grouped_tile)
};
// diagnostic (scripts/r5_wg_stamps.py): every later wgrad_multi launch records per-block stamps
// (the stamped twins are compiled into the experiments library only)
static unsigned long long* g_wgm_stamps = nullptr;
#if NNMPI_EXPERIMENTS_BUILD
void set_wgrad_multi_stamps(unsigned long long* buf) { g_wgm_stamps = buf; }
#endif

// NS: LDS stages of the DMA ring.  The launch holds about one block per CU (3 jobs x 16 tiles x 5
// splits = 240 blocks on the proxy step), so no second block hides a k-step's DMA wait; a
// 4-stage ring (128 KiB, three stages in flight) was built to test whether the L2 round trip
// bounds it: measured equal (proxy step 0.0737 / 0.0739 / 0.0749 ms with 4 stages vs 0.0733 /
// 0.0731 / 0.0742 with 2, wgrad_multi 26.2 us either way: profiles/r4_wgrad_multi_stages_ab.txt),
// so the default stays 2 (NNMPI_WG_STAGES=4 selects the deep ring).
constexpr int WGM_NS = 4;
constexpr int WGM_SMEM = WGM_NS * (GRP_BM + GRP_BN) * GEMM_BK * 2;
static int g_wgm_ns = -1;
static int wgm_stages() {   // 0: register-staged operands (NNMPI_WG_REG=1, A/B)
  if (g_wgm_ns < 0) {
    const char* e = knob_env("NNMPI_WG_STAGES");
    const char* r = knob_env("NNMPI_WG_REG");
    g_wgm_ns = (r && r[0] == '1') ? 0 : (e && e[0] == '4') ? WGM_NS : (e && e[0] == '3') ? 3 : 2;
  }
  return g_wgm_ns;
}

// Register-staged twin of the grouped weight-gradient tile (A/B, NNMPI_WG_REG=1): global ->
// VGPR -> ds_write with the operands of k-steps t+1 and t+2 in registers while k-step t
// computes, instead of LDS-DMA.  The row-band step's own weight stream reaches ~67 GB/s per CU
// through VGPR loads where the DMA ring of this launch moves ~33 (838 KB per block in 25 us).
// Same MFMA, same operand order, same k order: bitwise the dma_gemm_tile results.
struct WgRegLoad {   // one XMAJ operand stage: [64 k][128 x] bf16, 2 chunks of 16 B per thread
  uint4 r[2];
  __device__ __forceinline__ void load(const bf16* __restrict__ base, int ld, int x0, int X, int k0,
                                       int kend, int tid) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int c = tid + it * GRP_THREADS, k = k0 + c / 16, x = x0 + (c % 16) * 8;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (x < X && k < kend) v = *reinterpret_cast<const uint4*>(base + (long long)k * ld + x);
      r[it] = v;
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int c = tid + it * GRP_THREADS, k = c / 16, ch = c % 16;
      *reinterpret_cast<uint4*>(lds + k * 256 + ((ch ^ swz_x<128>(k)) << 4)) = r[it];
    }
  }
};

__device__ __forceinline__ void wg_reg_tile(const GemmParams& p, char* smem, int tx, int ty, int split) {
  constexpr int BM = GRP_BM, BN = GRP_BN, BK = GEMM_BK, WGN = GRP_WGN;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int WM = BM / GRP_WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int m0 = ty * BM, n0 = tx * BN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bg = tx == 0 && wn == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
  WgRegLoad a[2], b[2];   // operands of k-steps t+1 (slot (t+1) & 1) and t+2
  if (nt > 0) {
    a[0].load(p.A, p.lda, m0, p.M, kbeg, kend, tid);
    b[0].load(p.B, p.ldb, n0, p.N, kbeg, kend, tid);
    a[0].store(smem, tid);
    b[0].store(smem + A_BYTES, tid);
    a[1].load(p.A, p.lda, m0, p.M, kbeg + BK, kend, tid);
    b[1].load(p.B, p.ldb, n0, p.N, kbeg + BK, kend, tid);
    a[0].load(p.A, p.lda, m0, p.M, kbeg + 2 * BK, kend, tid);
    b[0].load(p.B, p.ldb, n0, p.N, kbeg + 2 * BK, kend, tid);
    __syncthreads();
  }
  auto step = [&](int t, WgRegLoad& an, WgRegLoad& bn) {
    const char* cur = smem + (t & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = read_frag_async<BM, XMAJ>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = read_frag_async<BN, XMAJ>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      if (do_bg) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
          accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[i], accb[i], 0, 0, 0);
      }
    }
    // k-step t+1 into the other stage (last read at step t-1: every wave is past the barrier
    // that ended it), then its registers take k-step t+3
    if (t + 1 < nt) {
      char* nxt = smem + ((t + 1) & 1) * STAGE;
      an.store(nxt, tid);
      bn.store(nxt + A_BYTES, tid);
      an.load(p.A, p.lda, m0, p.M, kbeg + (t + 3) * BK, kend, tid);
      bn.load(p.B, p.ldb, n0, p.N, kbeg + (t + 3) * BK, kend, tid);
    }
    __syncthreads();
  };
  for (int t = 0; t < nt; t += 2) {
    step(t, a[1], b[1]);
    if (t + 1 < nt) step(t + 1, a[0], b[0]);
  }
  if (lepi_ok<EPI_F32>(p)) {
    lds_epilogue<GRP_WGM, GRP_WGN, EPI_F32, ACT_NONE>(p, acc, smem, m0, n0, wm, wn, w, lane, split);
    if (do_bg && (lane >> 4) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * WM + i * 16 + (lane & 15);
        if (m >= p.M) continue;
        float* gb = p.bias_grad + split * p.bg_split_stride + m;
        if (p.sg.g_base) sgd_fused_store(p.sg, gb, accb[i][0]);
        else *gb = accb[i][0];
      }
    }
    return;
  }
  gemm_epilogue<BM, BN, GRP_WGM, GRP_WGN, EPI_F32, ACT_NONE, true>(p, acc, accb, do_bg, m0, n0, wm, wn,
                                                                     lane, split, nullptr);
}

// In-launch split-K fixup of a wgrad_multi tile (the grouped tile: 8 waves as 2 x 4, 64 x 32
// accumulators each, BM = BN = 128), cooperative and deadlock-free:
//  1. every split publishes its partial slab (LDS-staged rows, write-through stores) and counts
//     in at the tile's arrival counter (MI355X_MICROARCH.md "Valid forms" row 1: every store and
//     load of the slab bytes sc1, each storing wave drains vmcnt before the workgroup barrier, one
//     lane's agent-scope atomic signals);
//  2. the tile's rows are cut into S portions of whole 8-row groups; portion p belongs to split
//     p, taken by CAS on its claim word.  The LAST arrival (its add returned S - 1) never waits:
//     it takes its own portion and then every portion still unclaimed.  An earlier split polls the
//     counter (bounded, with s_sleep) and, once all S have arrived, claims its own portion; on
//     timeout it leaves the portion to the last arrival.  So no block ever depends on another
//     being resident, and each portion is combined exactly once;
//  3. a portion sums its rows of the S slabs in slab_multi's order (WS interleaved partials from
//     zero: bitwise the combine launch's result), then applies SGD-momentum (master, momentum,
//     bf16 shadow, the forward image; the transposed image from the portion restaged through LDS,
//     one 16-byte piece per lane) or stores the gradient; tiles of the first column also combine
//     the bias rows of the portion.
// The counters and claim words (WGM_CW per tile) are zeroed by the row-band launch before every
// weight-gradient launch (RowbandArgs::zero_words).
// slab_multi's virtual-wave count for S partial slabs (slab_ws, S <= 64)
__host__ __device__ __forceinline__ int slab_ws_n(int S) {
  int ws = 1;
  while (ws < 16 && ws * 8 < S) ws *= 2;
  return ws;
}
constexpr int WGM_MAXS = 16;       // most splits the fixup takes (more: the combine launch)
constexpr int WGM_CW = 32;         // counter words per tile: [0] arrivals, [1 + p] portion claims
constexpr int WGM_SPIN = 400;      // polls of an early split (x ~0.2 us) before it gives up

__device__ __forceinline__ void wgm_portion(const GemmParams& p, const WgmFix& f, char* smem, int tx,
                                            int ty, int portion) {
  const int tid = threadIdx.x;
  const int m0 = ty * GRP_BM, n0 = tx * GRP_BN, M = p.M, N = p.N, S = f.S, WS = slab_ws_n(S);
  const int g0 = (GRP_BM / 8) * portion / S, g1 = (GRP_BM / 8) * (portion + 1) / S;   // 8-row groups
  const int r0 = 8 * g0, nr = 8 * (g1 - g0);
  const long long ss = (long long)M * N;
  const float* slab = reinterpret_cast<const float*>(p.C);
  bf16* tb = reinterpret_cast<bf16*>(smem);   // the portion's updated rows, bf16 [nr][128]
  constexpr int IT = 32 * (GRP_BN / 4) / GRP_THREADS;   // float4 items per thread per 32 rows
  const bool upd = f.sg.g_base != nullptr;
  for (int c0 = 0; c0 < nr; c0 += 32) {   // (32-row chunks: one for S >= 4)
  // every split's values of this thread's items in flight at once, then the sums
  f32x4 u[IT][WGM_MAXS];
  int gm[IT], gn[IT];
  bool ok[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int e = c0 * (GRP_BN / 4) + tid + k * GRP_THREADS, row = r0 + e / (GRP_BN / 4);
    gm[k] = m0 + row;
    gn[k] = n0 + 4 * (e % (GRP_BN / 4));
    ok[k] = e < nr * (GRP_BN / 4) && gm[k] < M && gn[k] < N;
#pragma unroll
    for (int z = 0; z < WGM_MAXS; ++z)
      if (ok[k] && z < S) u[k][z] = ld_sc1(slab + z * ss + (long long)gm[k] * N + gn[k]);
  }
  SgdPre4 pre[IT];
  if (upd) {
#pragma unroll
    for (int k = 0; k < IT; ++k)
      if (ok[k]) pre[k] = sgd_pre4(f.sg, f.out + (long long)gm[k] * N + gn[k]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < IT; ++k) {
#pragma unroll
    for (int z = 0; z < WGM_MAXS; ++z) asm volatile("" : "+v"(u[k][z]));
    if (!ok[k]) continue;
    f32x4 t = {0.f, 0.f, 0.f, 0.f};
    for (int vw = 0; vw < WS; ++vw) {
      f32x4 pv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int z = 0; z < WGM_MAXS; ++z)
        if (z < S && z % WS == vw) pv += u[k][z];
      t = vw == 0 ? pv : t + pv;
    }
    float* o = f.out + (long long)gm[k] * N + gn[k];
    if (upd) {
      const f32x4 pn = sgd_apply4(f.sg, pre[k], t);
      bf16x4 hv;
#pragma unroll
      for (int e = 0; e < 4; ++e) hv[e] = (bf16)pn[e];
      if (f.pkf) *reinterpret_cast<bf16x4*>(f.pkf + rb_pk_off(gm[k], gn[k], N)) = hv;
      if (f.pkd) *reinterpret_cast<bf16x4*>(tb + (gm[k] - m0 - r0) * GRP_BN + (gn[k] - n0)) = hv;
    } else {
      *reinterpret_cast<f32x4*>(o) = t;
    }
  }
  }
  // bias rows of the portion (the tiles of the first column hold them)
  if (p.bias_grad && tx == 0 && tid < nr && m0 + r0 + tid < M) {
    const int m = m0 + r0 + tid;
    float bz[WGM_MAXS];
#pragma unroll
    for (int z = 0; z < WGM_MAXS; ++z)
      if (z < S) bz[z] = ld_sc1_f(p.bias_grad + z * p.bg_split_stride + m);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int z = 0; z < WGM_MAXS; ++z) asm volatile("" : "+v"(bz[z]));
    float b = 0.f;
    for (int vw = 0; vw < WS; ++vw) {
      float pb = 0.f;
#pragma unroll
      for (int z = 0; z < WGM_MAXS; ++z)
        if (z < S && z % WS == vw) pb += bz[z];
      b = vw == 0 ? pb : b + pb;
    }
    if (upd) sgd_fused_store(f.sg, f.bout + m, b);
    else f.bout[m] = b;
  }
  if (upd && f.pkd) {
    // W^T image pieces: column n, rows m .. m+7 of one 8-row group -> 16 contiguous bytes
    __syncthreads();
    for (int e = tid; e < (nr / 8) * GRP_BN; e += GRP_THREADS) {
      const int gi = e / GRP_BN, c = e % GRP_BN, n = n0 + c, m = m0 + r0 + 8 * gi;
      if (n >= N || m >= M) continue;
      bf16x8 col;
#pragma unroll
      for (int r = 0; r < 8; ++r) col[r] = tb[(8 * gi + r) * GRP_BN + c];
      *reinterpret_cast<bf16x8*>(f.pkd + rb_pk_off(n, m, M)) = col;
    }
  }
  __syncthreads();   // (the LDS rows may be reused by the next portion)
}

__device__ __forceinline__ void wgm_fixup(const GemmParams& p, const WgmFix& f, char* smem, int tx,
                                          int ty, int split, int tile, const f32x4* acc,
                                          const f32x4* accb) {
  constexpr int NW = GRP_WGM * GRP_WGN, WM = GRP_BM / GRP_WGM, WN = GRP_BN / GRP_WGN;
  constexpr int MI = WM / 16, NJ = WN / 16, ITER = GRP_BM / (NW * LEPI_ROWS);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w / GRP_WGN, wn = w % GRP_WGN;
  const int m0 = ty * GRP_BM, n0 = tx * GRP_BN, M = p.M, N = p.N, S = f.S;
  float* img = reinterpret_cast<float*>(smem);
  // ---- 1. publish this split's slab ----
  __builtin_amdgcn_s_barrier();   // every wave is past its last read of the DMA ring
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wm * WM + i * 16 + (lane & 15);
      const int c4 = (wn * WN + j * 16) / 4 + (lane >> 4);
      *reinterpret_cast<f32x4*>(img + lepi_off(r, c4)) = acc[i * NJ + j];
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int q = lane & 15, gn = n0 + q * 8;
  float* slab = reinterpret_cast<float*>(p.C) + split * (long long)M * N;
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int r = (it * NW + w) * LEPI_ROWS + (lane >> 4), gm = m0 + r;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(img + lepi_off(r, 2 * q));
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(img + lepi_off(r, 2 * q + 1));
    if (gm < M && gn < N) {
      float* o = slab + (long long)gm * N + gn;
      st_sc1(o, v0);
      st_sc1(o + 4, v1);
    }
  }
  if (p.bias_grad && tx == 0 && wn == 0 && (lane >> 4) == 0) {   // the row-sum lanes
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
      if (m < M) st_sc1_f(p.bias_grad + split * p.bg_split_stride + m, accb[i][0]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave's slab stores are complete; the LDS image is free
  // ---- 2. arrive; the last arrival never waits ----
  int* cw = f.cnt + tile * WGM_CW;   // [0] arrivals, [1 + p] claim of portion p
  int* flag = reinterpret_cast<int*>(smem + 60 * 1024);
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(cw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int mode = 0;   // 0: leave, 1: own portion, 2: last arrival
    if (old == S - 1) {
      mode = 2;
    } else {
      int polls = 0;
      while (ld_sc1_i(cw) < S && ++polls < WGM_SPIN) __builtin_amdgcn_s_sleep(8);
      if (polls < WGM_SPIN &&
          __hip_atomic_fetch_add(cw + 1 + split, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        mode = 1;
    }
    if (mode == 2)
      mode = __hip_atomic_fetch_add(cw + 1 + split, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 ? 2 : 3;
    flag[0] = mode;
  }
  __syncthreads();
  const int mode = flag[0];
  __syncthreads();
  if (mode == 0) return;
  // ---- 3. combine ----
  if (mode == 1 || mode == 2) wgm_portion(p, f, smem, tx, ty, split);
  if (mode >= 2) {
    for (int o = 1; o < S; ++o) {
      const int pp = (split + o) % S;
      if (tid == 0)
        flag[0] = __hip_atomic_fetch_add(cw + 1 + pp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
      __syncthreads();
      const int mine = flag[0];
      __syncthreads();
      if (mine) wgm_portion(p, f, smem, tx, ty, pp);
    }
  }
}

// ST: diagnostic per-block stamps (set_wgrad_multi_stamps); the job loop breaks instead of
// returning so both forms share one body (ST = false is the production kernel, unchanged code)
template <int GA, int NS, bool ST = false, bool FIX = false>
__global__ void __launch_bounds__(GRP_THREADS, (NS == 0 || GA >= 3 || FIX || ST) ? 2 : 4) wgrad_multi_kernel(WgradMultiParams g) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  if constexpr (FIX) {
    if ((int)blockIdx.x >= g.gemm_blocks) {   // the extra combine (row-band head partials)
      slab_reduce_any(g.tail_ws, g.tail, blockIdx.x - g.gemm_blocks, g.tail_nb_main, g.tail_nb_bias,
                      reinterpret_cast<f32x4*>(smem));
      return;
    }
  }
  if constexpr (ST) {
    if (threadIdx.x == 0) {
      g.stamps[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memrealtime();
      g.stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC id
      g.stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW id
    }
  }
  int bid = blockIdx.x;
#pragma unroll
  for (int j = 0; j < RB_MAXL; ++j) {
    if (j >= g.nj) break;
    if (bid < g.blocks[j]) {
      const int l = xcd_remap(bid, g.blocks[j]);
      if (l >= g.n[j]) break;
      const int split = l / g.tiles[j], t = l % g.tiles[j];
      unsigned long long* kst = ST ? g.stamps + 1024 * 4 + (long long)blockIdx.x * 128 : nullptr;
      if constexpr (FIX) {
        constexpr int MI = GRP_BM / GRP_WGM / 16, NJ = GRP_BN / GRP_WGN / 16;
        f32x4 acc[MI * NJ], accb[MI];
        dma_gemm_tile<GRP_BM, GRP_BN, GRP_WGM, GRP_WGN, XMAJ, XMAJ, EPI_F32, ACT_NONE, true, NS, GA, ST,
                      true>(g.wg[j], smem, t % g.gx[j], t / g.gx[j], split, kst, acc, accb);
        wgm_fixup(g.wg[j], g.fix[j], smem, t % g.gx[j], t / g.gx[j], split, t, acc, accb);
      } else if constexpr (NS == 0) {   // register-staged operands (A/B)
        wg_reg_tile(g.wg[j], smem, t % g.gx[j], t / g.gx[j], split);
      } else {
        dma_gemm_tile<GRP_BM, GRP_BN, GRP_WGM, GRP_WGN, XMAJ, XMAJ, EPI_F32, ACT_NONE, true, NS, GA, ST>(
            g.wg[j], smem, t % g.gx[j], t / g.gx[j], split, kst);
      }
      break;
    }
    bid -= g.blocks[j];
  }
  if constexpr (ST) {
    __syncthreads();
    if (threadIdx.x == 0) g.stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// Half-width tile of the grouped weight gradient (NNMPI_WGM_TILE=1): 128 (M) x 64 (N), 4 waves
// of 64 x 32 -- the same per-wave work as the 128 x 128 tile, twice the blocks, so two blocks
// share each CU and one's DMA / LDS phase runs beside the other's MFMAs (per-k-step stamps of the
// 128 x 128 tile at one block per CU: wait 320 + barrier 88 + DMA issue 412 + reads and MFMAs
// 892 cycles, in lockstep -- profiles/r5_wgrad_kstep_stamps.txt).  Same K split, same slab
// layout, same per-element accumulation order: bitwise the 128 x 128 tile's slabs.
#if NNMPI_EXPERIMENTS_BUILD
constexpr int WGH_BM = 128, WGH_BN = 64, WGH_WGM = 2, WGH_WGN = 2;
constexpr int WGH_THREADS = 64 * WGH_WGM * WGH_WGN;
constexpr int WGH_SMEM = 2 * (WGH_BM + WGH_BN) * GEMM_BK * 2;

template <int GA>
__global__ void __launch_bounds__(WGH_THREADS, 2) wgrad_multi_h_kernel(WgradMultiParams g) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  int bid = blockIdx.x;
#pragma unroll
  for (int j = 0; j < RB_MAXL; ++j) {
    if (j >= g.nj) break;
    if (bid < g.blocks[j]) {
      const int l = xcd_remap(bid, g.blocks[j]);
      if (l >= g.n[j]) break;
      const int split = l / g.tiles[j], t = l % g.tiles[j];
      dma_gemm_tile<WGH_BM, WGH_BN, WGH_WGM, WGH_WGN, XMAJ, XMAJ, EPI_F32, ACT_NONE, true, 2, GA>(
          g.wg[j], smem, t % g.gx[j], t / g.gx[j], split);
      break;
    }
    bid -= g.blocks[j];
  }
}

static int g_wgm_tile = -1;
void set_wgm_tile(int t) { g_wgm_tile = t; }   // -1: re-read NNMPI_WGM_TILE
static int wgm_tile() {
  if (g_wgm_tile < 0) {
    const char* e = knob_env("NNMPI_WGM_TILE");
    g_wgm_tile = (e && e[0] == '1') ? 1 : 0;
  }
  return g_wgm_tile;
}
#else
static constexpr int wgm_tile() { return 0; }
#endif

// Kernel variant of a wgrad_multi launch: DMA ring stages (NNMPI_WG_STAGES 2 / 3 / 4, or 0 =
// register-staged, NNMPI_WG_REG=1), LDS read mode (dma_gemm_tile ASYNC_TR; NNMPI_WGM_ASYNC or
// set_group_async), in-launch fixup, diagnostic stamps.
template <int GA, int NS>
static void* wgm_fn(bool fix, bool st) {
#if NNMPI_EXPERIMENTS_BUILD
  if (fix) return st ? (void*)wgrad_multi_kernel<GA, NS, true, true> : (void*)wgrad_multi_kernel<GA, NS, false, true>;
  return st ? (void*)wgrad_multi_kernel<GA, NS, true, false> : (void*)wgrad_multi_kernel<GA, NS, false, false>;
#else
  // (the production library: neither the in-launch fixup nor the stamped twin)
  return (fix || st) ? nullptr : (void*)wgrad_multi_kernel<GA, NS, false, false>;
#endif
}

static hipError_t wgm_launch(const WgradMultiParams& g, int nb, bool fix, hipStream_t s) {
  static const int env_ga = [] {
    const char* e = knob_env("NNMPI_WGM_ASYNC");
    return (e && e[0] >= '0' && e[0] <= '4') ? e[0] - '0' : -1;
  }();
  int ga = g_group_async >= 0 ? std::min(g_group_async, 4) : env_ga >= 0 ? env_ga : WGM_ASYNC_DEFAULT;
  int ns = wgm_stages();
  if (fix && ns == 0) ns = 2;          // (the fixup takes the DMA tile only)
  if (ga < 2) ga = 2;                  // (the compiler-scheduled / whole-stage read modes retired)
  const bool st = g.stamps != nullptr;
  void* f = nullptr;
#if NNMPI_EXPERIMENTS_BUILD
  if (ns == 0) f = st ? (void*)wgrad_multi_kernel<2, 0, true> : (void*)wgrad_multi_kernel<2, 0>;
#else
  if (ns == 0) f = st ? nullptr : (void*)wgrad_multi_kernel<2, 0>;
#endif
  else if (ns == 3) f = ga == 2 ? wgm_fn<2, 3>(fix, st) : ga == 3 ? wgm_fn<3, 3>(fix, st) : wgm_fn<4, 3>(fix, st);
  else if (ns == WGM_NS) f = ga == 2 ? wgm_fn<2, WGM_NS>(fix, st) : ga == 3 ? wgm_fn<3, WGM_NS>(fix, st)
                                                                   : wgm_fn<4, WGM_NS>(fix, st);
  else f = ga == 2 ? wgm_fn<2, 2>(fix, st) : ga == 3 ? wgm_fn<3, 2>(fix, st) : wgm_fn<4, 2>(fix, st);
  if (!f) return hipErrorNotSupported;
  const int smem = (ns == 0 ? 2 : ns) * (GRP_BM + GRP_BN) * GEMM_BK * 2;
  static void* attr_done[64] = {};
  bool seen = false;
  for (void*& a : attr_done) {
    if (a == f) { seen = true; break; }
    if (!a) { a = f; break; }
  }
  if (!seen) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hipLaunchKernelGGL(reinterpret_cast<void (*)(WgradMultiParams)>(f), dim3(nb), dim3(GRP_THREADS), smem, s, g);
  return hipGetLastError();
}

int wgrad_multi_splits(int nj, int M, int N, int K) {
  const int tiles = ((M + GRP_BM - 1) / GRP_BM) * ((N + GRP_BN - 1) / GRP_BN);
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  // one 512-thread block per CU: measured on the proxy step (3 jobs of 16 tiles, K = 8192), 5
  // splits 25.2 + 8.6 us (grouped weight gradients + combines) vs 10 splits 23.7 + 11.9 and 16
  // splits 27.2 + 14.3 (profiles/r3s2_rowband_splits_ab.txt): fewer slabs, less combine traffic
  int s = std::max(1, 256 / std::max(1, nj * tiles));
  s = std::min(s, std::max(1, ksteps / 4));   // >= 4 k-steps per split
  if (g_wgrad_splits > 0 && g_wgrad_splits < s) s = g_wgrad_splits;
  return s;
}

hipError_t wgrad_multi(const WgradArgs* jobs, int nj, const int* splits, SlabReduce* pending,
                       hipStream_t s) {
  if (nj < 1 || nj > RB_MAXL) return hipErrorInvalidValue;
  WgradMultiParams g{};
  g.nj = nj;
  int nb = 0;
  for (int j = 0; j < nj; ++j) {
    const WgradArgs& a = jobs[j];
    if (wgrad_tile(a.M, a.N) != 128 || a.db == nullptr || a.ws == nullptr || a.dW16 != nullptr)
      return hipErrorInvalidValue;
    const int want = (splits && splits[j] > 0) ? splits[j] : wgrad_multi_splits(nj, a.M, a.N, a.K);
    GemmParams p;
    const int sp = make_wgrad_s(a, p, pending[j], want);
    if (sp == 1) {   // un-split: the combine would have nothing to do -- keep the slab form
      p.C = a.ws; p.c_split_stride = (long long)a.M * a.N; p.sg = SgdFuse{};
      p.bias_grad = a.ws + (size_t)a.M * a.N; p.bg_split_stride = a.M;
      p.c16 = nullptr; p.bg16 = nullptr;
      pending[j] = SlabReduce{a.ws, 1, (long long)a.M * a.N, a.M, a.N, a.dW, a.N,
                              a.ws + (size_t)a.M * a.N, a.M, a.db, nullptr, 0, 0.f, nullptr, a.sg};
    }
    set_extents<XMAJ, XMAJ>(p);
    p.store_pol = slab_store_pol();
    g.wg[j] = p;
#if NNMPI_EXPERIMENTS_BUILD
    const int bn = wgm_tile() == 1 ? WGH_BN : GRP_BN;
#else
    const int bn = GRP_BN;
#endif
    g.gx[j] = (p.N + bn - 1) / bn;
    g.tiles[j] = g.gx[j] * ((p.M + GRP_BM - 1) / GRP_BM);
    g.n[j] = g.tiles[j] * sp;
    g.blocks[j] = (g.n[j] + 7) & ~7;
    nb += g.blocks[j];
  }
#if NNMPI_EXPERIMENTS_BUILD
  if (wgm_tile() == 1) {
    static const int env_ga = [] {
      const char* e = knob_env("NNMPI_WGM_ASYNC");
      return (e && e[0] >= '2' && e[0] <= '4') ? e[0] - '0' : -1;
    }();
    const int ga = env_ga == 3 ? 3 : env_ga == 4 ? 4 : 2;
    void* f = ga == 3 ? (void*)wgrad_multi_h_kernel<3> : ga == 4 ? (void*)wgrad_multi_h_kernel<4>
                                                               : (void*)wgrad_multi_h_kernel<2>;
    static void* attr_done[4] = {};
    bool seen = false;
    for (void*& a : attr_done) {
      if (a == f) { seen = true; break; }
      if (!a) { a = f; break; }
    }
    if (!seen) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, WGH_SMEM);
    hipLaunchKernelGGL(reinterpret_cast<void (*)(WgradMultiParams)>(f), dim3(nb), dim3(WGH_THREADS),
                       WGH_SMEM, s, g);
    return hipGetLastError();
  }
#endif
  g.stamps = g_wgm_stamps;
  return wgm_launch(g, nb, false, s);
}

#if NNMPI_EXPERIMENTS_BUILD
int wgrad_fix_counters(int M, int N) {
  return ((M + GRP_BM - 1) / GRP_BM) * ((N + GRP_BN - 1) / GRP_BN) * WGM_CW;
}
#endif

// The row-band step's weight gradients with the in-launch fixup (one launch, no combine launch):
// jobs as wgrad_multi; fix[j] says where job j's result goes (its out / bout / sg / images; cnt =
// its tile counters, zero); `tail` (may have S == 0 / null loss): an extra combine run by blocks
// appended to the grid (the head's per-band partials).
#if NNMPI_EXPERIMENTS_BUILD
hipError_t wgrad_multi_fix(const WgradArgs* jobs, int nj, const int* splits, const WgOut* fix,
                           const SlabReduce* tail, hipStream_t s) {
  if (nj < 1 || nj > RB_MAXL) return hipErrorInvalidValue;
  WgradMultiParams g{};
  g.nj = nj;
  int nb = 0;
  for (int j = 0; j < nj; ++j) {
    const WgradArgs& a = jobs[j];
    if (wgrad_tile(a.M, a.N) != 128 || a.db == nullptr || a.ws == nullptr || a.dW16 != nullptr ||
        !fix[j].cnt)
      return hipErrorInvalidValue;
    const int want = (splits && splits[j] > 0) ? splits[j] : wgrad_multi_splits(nj, a.M, a.N, a.K);
    GemmParams p;
    SlabReduce pend;
    const int sp = make_wgrad_s(a, p, pend, want);
    if (sp > WGM_MAXS) return hipErrorNotSupported;
    // every split writes its slab (even S == 1: the fixup reads the partial from registers)
    p.C = a.ws; p.c_split_stride = (long long)a.M * a.N; p.sg = SgdFuse{};
    p.bias_grad = a.ws + (size_t)sp * a.M * a.N; p.bg_split_stride = a.M;
    p.c16 = nullptr; p.bg16 = nullptr;
    set_extents<XMAJ, XMAJ>(p);
    g.wg[j] = p;
    g.gx[j] = (p.N + GRP_BN - 1) / GRP_BN;
    g.tiles[j] = g.gx[j] * ((p.M + GRP_BM - 1) / GRP_BM);
    g.n[j] = g.tiles[j] * sp;
    g.blocks[j] = (g.n[j] + 7) & ~7;
    g.fix[j] = WgmFix{a.dW, a.db, a.sg, fix[j].pkf, fix[j].pkd, fix[j].cnt, sp};
    nb += g.blocks[j];
  }
  g.gemm_blocks = nb;
  if (tail && tail->ws && tail->S > 0) {
    g.tail = *tail;
    g.tail.sgd_serial = sgd_serial();
    g.tail_ws = slab_ws(*tail);
    int nbt = 0;
    slab_blocks(*tail, g.tail_nb_main, g.tail_nb_bias, nbt);
    nb += nbt;
  }
  g.stamps = g_wgm_stamps;
  return wgm_launch(g, nb, true, s);
}
#endif

// ---- Small-batch weight gradients, update in the epilogue (the column-split row-band step) ----
// At <= 4,096 rows wgrad_multi's split-K slabs (5 per layer at 1,024 rows) and their combine
// launch cost more than the product: 9.8 + 8.8 us for 1.6 GFLOP on the proxy at 1,024 rows
// (profiles/r5_rowband_split_bench.txt).  Here every layer's 64 x 64 tiles (3 x 64 = 192 blocks
// on the proxy) reduce the whole K = rows un-split, and the epilogue applies SGD-momentum from
// registers and rewrites the v2 weight images (one rank), or stores the gradient (several ranks);
// extra blocks combine the head's per-band partials (the row-band head_red).  One launch where
// the slab form takes two, and no slab round trip.
//
// Image path (KPW > 0; the split kernel wrote the operands as K-major MFMA fragments, RowbandArgs
// ka / kz): no LDS operand stage at all.  Each of the 8 waves takes KPW = kbands / 8 consecutive
// 32-row k-blocks and computes the whole 64 x 64 tile over them -- 4 + 4 one-KiB fragments per
// k-block, each a single 16-byte load per lane straight into an MFMA operand, DEP k-blocks in
// flight -- then the 8 partial tiles are summed in wave order through LDS into the LDS-DMA
// path's register layout, and the same epilogue runs.  (The LDS-DMA tile streams its operands
// at ~38 GB/s per CU, profiles/r5_wgrad_small_ab.txt.)
template <int KPW>
__device__ __forceinline__ void wgs_kimg_tile(const bf16* __restrict__ za, const bf16* __restrict__ xb,
                                              int nkb, int gm0, int gn0, bool bias, char* smem,
                                              f32x4 (&acc)[2], f32x4 (&accb)[2]) {
  constexpr int DEP = KPW <= 4 ? KPW : 3;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kb0 = w * KPW;
  f32x4 pa[4][4], pb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) pa[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;
  const bf16x8* fa = reinterpret_cast<const bf16x8*>(za) + lane;
  const bf16x8* fb = reinterpret_cast<const bf16x8*>(xb) + lane;
  bf16x8 ra[DEP][4], rb[DEP][4];
  auto load = [&](int t, int sl) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[sl][i] = fa[((long long)(gm0 + i) * nkb + kb0 + t) * 64];
      rb[sl][i] = fb[((long long)(gn0 + i) * nkb + kb0 + t) * 64];
    }
  };
#pragma unroll
  for (int t = 0; t < DEP; ++t) load(t, t);
#pragma unroll
  for (int t = 0; t < KPW; ++t) {
    const int sl = t % DEP;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) pa[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[sl][j], ra[sl][i], pa[i][j], 0, 0, 0);
    if (bias) {
#pragma unroll
      for (int i = 0; i < 4; ++i) pb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, ra[sl][i], pb[i], 0, 0, 0);
    }
    // (sched_barrier: the refill stays behind this k-block's MFMAs -- the compiler would hoist
    // every load of the unrolled loop and spill past 4 k-blocks in flight)
    __builtin_amdgcn_sched_barrier(0);
    if (t + DEP < KPW) load(t + DEP, sl);
    __builtin_amdgcn_sched_barrier(0);
  }
  // the partial tiles in wave order: part[w][i][j][lane], bias partials bp[w][i][16]
  f32x4* part = reinterpret_cast<f32x4*>(smem);
  float* bp = reinterpret_cast<float*>(part + 8 * 16 * 64);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[((w * 4 + i) * 4 + j) * 64 + lane] = pa[i][j];
  if (bias && lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bp[(w * 4 + i) * 16 + lane] = pb[i][0];
  }
  __syncthreads();
  // the LDS-DMA tile's layout: wave (wm, wn) = (w >> 2, w & 3) holds m-groups 2 wm + i, n-group wn
  const int wm = w >> 2, wn = w & 3;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 t = part[((0 * 4 + 2 * wm + i) * 4 + wn) * 64 + lane];
#pragma unroll
    for (int v = 1; v < 8; ++v) t += part[((v * 4 + 2 * wm + i) * 4 + wn) * 64 + lane];
    acc[i] = t;
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias && lane < 16) {
      float b = bp[(0 * 4 + 2 * wm + i) * 16 + lane];
#pragma unroll
      for (int v = 1; v < 8; ++v) b += bp[(v * 4 + 2 * wm + i) * 16 + lane];
      accb[i][0] = b;
    }
  }
}
constexpr int WGS_KIMG_SMEM = 8 * 16 * 64 * 16 + 8 * 4 * 16 * 4;
constexpr int WGS_KIMG_MAXB = 128;   // bands (4,096 rows): up to 16 k-blocks per wave

template <int GA, int NS, int KPW = 0>
__global__ void __launch_bounds__(SLAB_THREADS) wgrad_small_kernel(WgradMultiParams g) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  // diagnostic (set_wgrad_multi_stamps, scripts/r5_wgs_stamps.py): per block the real-time
  // counter at entry, after the GEMM, at exit
  unsigned long long* stp = (NNMPI_EXPERIMENTS_BUILD && g.stamps) ? g.stamps + blockIdx.x * 4 : nullptr;
  if (stp && threadIdx.x == 0) stp[0] = __builtin_amdgcn_s_memrealtime();
  if ((int)blockIdx.x >= g.gemm_blocks) {   // the head's combine
    slab_reduce_any(g.tail_ws, g.tail, blockIdx.x - g.gemm_blocks, g.tail_nb_main, g.tail_nb_bias,
                    reinterpret_cast<f32x4*>(smem));
    if (stp) {
      __syncthreads();
      if (threadIdx.x == 0) stp[2] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  constexpr int MI = 2, NJ = 1;   // 64 x 64 tile, 2 x 4 waves of 32 x 16 (512 threads: the
                                  // combine blocks' shape)
  int bid = blockIdx.x;
#pragma unroll
  for (int j = 0; j < RB_MAXL; ++j) {
    if (j >= g.nj) break;
    if (bid < g.blocks[j]) {
      const int t = xcd_remap(bid, g.blocks[j]);
      if (t >= g.n[j]) break;
      // (image path: an XCD's 8 consecutive tiles as a 2 x 4 patch -- 2 dZ + 4 input panels
      // through its L2 instead of 1 + 8 for a row of tiles; the main loop streams at the chip's
      // fetch rate, profiles/r6_wgrad_small_kimg.txt)
      int tx, ty;
      grouped_tile(t, g.gx[j], g.tiles[j] / g.gx[j], KPW > 0 ? g.gm : 1, tx, ty);
      const WgmFix& f = g.fix[j];
      const int M = g.wg[j].M, N = g.wg[j].N;
      const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 2, wn = w & 3;
      const int m0 = ty * 64, n0 = tx * 64;
      const bool upd = f.sg.g_base != nullptr;
      int mm[MI * NJ], nn[MI * NJ];
      bool ok[MI * NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) {
          const int k = i * NJ + jj;
          mm[k] = m0 + wm * 32 + i * 16 + (lane & 15);
          nn[k] = n0 + wn * 16 + jj * 16 + (lane >> 4) * 4;
          ok[k] = mm[k] < M && nn[k] < N;
        }
      // Every operand of the update -- the weights' and the biases' master / momentum values --
      // is loaded BEFORE the main loop (the oldest loads: the ring's counted vmcnt waits retire
      // them first), so the epilogue has no dependent round trip left (per-block stamps: the
      // epilogue was 3.4 us of a 10.3 us block with the loads after the GEMM and the bias update
      // one more round trip behind them; scripts/r5_wgs_stamps.py)
      const bool dob = tx == 0 && wn == 0 && (lane >> 4) == 0;   // the bias lanes
      SgdPre4 pre[MI * NJ];
      float bp[MI], bm[MI];
      long long boff[MI];
      if (upd) {
#pragma unroll
        for (int k = 0; k < MI * NJ; ++k)
          if (ok[k]) pre[k] = sgd_pre4(f.sg, f.out + (long long)mm[k] * N + nn[k]);
        if (dob) {
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int m = m0 + wm * 32 + i * 16 + lane;
            boff[i] = (f.bout + min(m, M - 1)) - f.sg.g_base;
            bp[i] = f.sg.p_base[boff[i]];
            bm[i] = f.sg.m_base[boff[i]];
          }
        }
      }
      f32x4 acc[MI * NJ], accb[MI];
      if constexpr (KPW > 0) {
        wgs_kimg_tile<KPW>(g.kA[j], g.kB[j], g.kbands, ty * 4, tx * 4, tx == 0, smem, acc, accb);
      } else {
        dma_gemm_tile<64, 64, 2, 4, XMAJ, XMAJ, EPI_F32, ACT_NONE, true, NS, GA, false, true>(
            g.wg[j], smem, tx, ty, 0, nullptr, acc, accb);
      }
      if (stp && threadIdx.x == 0) stp[1] = __builtin_amdgcn_s_memrealtime();
      if (upd) {
        // the updates; the transposed image through LDS as 16-byte pieces (8 rows of a column)
        bf16* tb = reinterpret_cast<bf16*>(smem);   // [64][64] new weights of the tile
        __syncthreads();   // (every wave is past its last read of the DMA ring)
#pragma unroll
        for (int k = 0; k < MI * NJ; ++k) {
          if (!ok[k]) continue;
          const f32x4 pn = sgd_apply4(f.sg, pre[k], acc[k]);
          rb_pack_store4(f.pkf, nullptr, mm[k], nn[k], M, N, pn);
          bf16x4 hv;
#pragma unroll
          for (int e = 0; e < 4; ++e) hv[e] = (bf16)pn[e];
          *reinterpret_cast<bf16x4*>(tb + (mm[k] - m0) * 64 + (nn[k] - n0)) = hv;
        }
        if (f.pkd) {
          __syncthreads();
          const int c = tid & 63, g8 = tid >> 6, n = n0 + c, m = m0 + 8 * g8;
          if (n < N && m < M) {
            bf16x8 col;
#pragma unroll
            for (int r = 0; r < 8; ++r) col[r] = tb[(8 * g8 + r) * 64 + c];
            *reinterpret_cast<bf16x8*>(f.pkd + rb_pk_off(n, m, M)) = col;
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < MI * NJ; ++k)
          if (ok[k]) *reinterpret_cast<f32x4*>(f.out + (long long)mm[k] * N + nn[k]) = acc[k];
      }
      if (dob) {   // the bias gradient: the row sums (sgd_fused_store's arithmetic, operands early)
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0 + wm * 32 + i * 16 + lane;
          if (m >= M) continue;
          if (upd) {
            float bb = bm[i];
            const float pn = sgd_elem(bp[i], accb[i][0], bb, f.sg.hp[0], f.sg.hp[1], f.sg.hp[2], f.sg.hp[3],
                                      f.sg.hp[4], f.sg.nesterov != 0, f.sg.first != 0);
            f.sg.p_base[boff[i]] = pn;
            if (f.sg.hp[1] != 0.f) f.sg.m_base[boff[i]] = bb;
            if (f.sg.s_base) f.sg.s_base[boff[i]] = (bf16)pn;
          } else {
            f.bout[m] = accb[i][0];
          }
        }
      }
      break;
    }
    bid -= g.blocks[j];
  }
  if (stp) {
    __syncthreads();
    if (threadIdx.x == 0) stp[2] = __builtin_amdgcn_s_memrealtime();
  }
}

// The image path (NNMPI_WGS_KIMG=0: the LDS-DMA tiles, A/B): whole 8-band groups, <= 4,096 rows
static int g_wgs_kimg = -1;
void set_wgs_kimg(int v) { g_wgs_kimg = v; }
bool wgrad_kimg_ok(int rows) {
  if (g_wgs_kimg < 0) {
    const char* e = knob_env("NNMPI_WGS_KIMG");
    g_wgs_kimg = (e && e[0] == '0') ? 0 : 1;
  }
  const int nb = (rows + 31) / 32;
  return g_wgs_kimg == 1 && rows > 0 && nb % 8 == 0 && nb <= WGS_KIMG_MAXB;
}

hipError_t wgrad_small(const WgradArgs* jobs, int nj, const WgOut* img, const SlabReduce* tail,
                       hipStream_t s, int kbands) {
  if (nj < 1 || nj > RB_MAXL) return hipErrorInvalidValue;
  WgradMultiParams g{};
  g.nj = nj;
  // the image path when every job has both images and the bands split evenly over 8 waves
  bool kimg = kbands > 0 && kbands % 8 == 0 && kbands <= WGS_KIMG_MAXB && img != nullptr;
  for (int j = 0; kimg && j < nj; ++j) {
    kimg = img[j].kA && img[j].kB && jobs[j].M % 64 == 0 && jobs[j].N % 64 == 0 &&
           jobs[j].K <= kbands * 32 && jobs[j].K > (kbands - 1) * 32;
    g.kA[j] = img[j].kA;
    g.kB[j] = img[j].kB;
  }
  g.kbands = kbands;
  static const int gm = [] {   // (NNMPI_WGS_GM 1 / 2 / 4, A/B)
    const char* e = knob_env("NNMPI_WGS_GM");
    return (e && (e[0] == '1' || e[0] == '2' || e[0] == '4')) ? e[0] - '0' : 2;
  }();
  g.gm = gm;
  int nb = 0;
  for (int j = 0; j < nj; ++j) {
    const WgradArgs& a = jobs[j];
    if (a.db == nullptr || a.dW16 != nullptr || a.M % 32 || a.N % 32) return hipErrorInvalidValue;
    GemmParams p;
    SlabReduce pend;
    make_wgrad_s(a, p, pend, 1);
    p.sg = SgdFuse{};
    p.c16 = nullptr; p.bg16 = nullptr;
    set_extents<XMAJ, XMAJ>(p);
    g.wg[j] = p;
    g.gx[j] = (p.N + 63) / 64;
    g.tiles[j] = g.gx[j] * ((p.M + 63) / 64);
    g.n[j] = g.tiles[j];
    g.blocks[j] = (g.n[j] + 7) & ~7;
    g.fix[j] = WgmFix{a.dW, a.db, a.sg, img ? img[j].pkf : nullptr, img ? img[j].pkd : nullptr, nullptr, 1};
    nb += g.blocks[j];
  }
  g.gemm_blocks = nb;
  if (tail && tail->ws && tail->S > 0) {
    g.tail = *tail;
    g.tail.sgd_serial = sgd_serial();
    g.tail_ws = slab_ws(*tail);
    int nbt = 0;
    slab_blocks(*tail, g.tail_nb_main, g.tail_nb_bias, nbt);
    nb += nbt;
  }
  g.stamps = g_wgm_stamps;
  // DMA ring stages (NNMPI_WGS_STAGES 2 / 3 / 4 / 6 / 8; default 4).  One 64 x 64 tile per CU
  // streams its whole K at ~0.43 us per 16 KiB k-step (per-block stamps), but deeper rings do not
  // help -- 6 / 8 stages 14.5 / 14.8 us vs 14.0 at 1,024 rows (profiles/r5_wgrad_small_ab.txt):
  // the per-CU LDS-DMA fill rate (MI355X_MICROARCH.md "ldsdma-fill", ~25 GB/s per loader wave),
  // not the round trip, bounds it
  static const int ns = [] {
    const char* e = knob_env("NNMPI_WGS_STAGES");
    const int v = (e && e[0] >= '2' && e[0] <= '8') ? e[0] - '0' : 4;
    return (v == 5 || v == 7) ? v + 1 : v;
  }();
  const int smem = std::max(ns * (64 + 64) * GEMM_BK * 2, SLAB_PART_BYTES);
  // LDS read mode of the tile (dma_gemm_tile ASYNC_TR, NNMPI_WGS_ASYNC 2 / 3 / 4): 4 -- the
  // refill's DMA pieces issued between the k-halves' MFMAs -- measured 13.4 vs 14.2 us (mode 2)
  // at 1,024 rows and 18.7 vs 19.6 us at 2,048 (profiles/r5_wgrad_small_ab.txt)
  static const int ga = [] {
    const char* e = knob_env("NNMPI_WGS_ASYNC");
    return (e && (e[0] == '2' || e[0] == '3')) ? e[0] - '0' : 4;
  }();
  auto* f = ns == 2 ? wgrad_small_kernel<2, 2> : ns == 3 ? wgrad_small_kernel<2, 3>
          : ns == 4 ? (ga == 3 ? wgrad_small_kernel<3, 4> : ga == 4 ? wgrad_small_kernel<4, 4> : wgrad_small_kernel<2, 4>)
          : ns == 6 ? wgrad_small_kernel<2, 6> : wgrad_small_kernel<2, 8>;
  static bool attr = false;
  if (!attr) {
    for (auto* k : {wgrad_small_kernel<2, 4>, wgrad_small_kernel<3, 4>, wgrad_small_kernel<4, 4>,
                    wgrad_small_kernel<2, 6>, wgrad_small_kernel<2, 8>})
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  if (kimg) {
    using Fn = void (*)(WgradMultiParams);
    static const Fn kf[16] = {wgrad_small_kernel<4, 4, 1>,  wgrad_small_kernel<4, 4, 2>,  wgrad_small_kernel<4, 4, 3>,
                              wgrad_small_kernel<4, 4, 4>,  wgrad_small_kernel<4, 4, 5>,  wgrad_small_kernel<4, 4, 6>,
                              wgrad_small_kernel<4, 4, 7>,  wgrad_small_kernel<4, 4, 8>,  wgrad_small_kernel<4, 4, 9>,
                              wgrad_small_kernel<4, 4, 10>, wgrad_small_kernel<4, 4, 11>, wgrad_small_kernel<4, 4, 12>,
                              wgrad_small_kernel<4, 4, 13>, wgrad_small_kernel<4, 4, 14>, wgrad_small_kernel<4, 4, 15>,
                              wgrad_small_kernel<4, 4, 16>};
    static bool kattr = false;
    if (!kattr) {
      for (Fn k : kf) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      kattr = true;
    }
    hipLaunchKernelGGL(kf[kbands / 8 - 1], dim3(nb), dim3(SLAB_THREADS), std::max(WGS_KIMG_SMEM, SLAB_PART_BYTES),
                       s, g);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(f, dim3(nb), dim3(SLAB_THREADS), smem, s, g);
  return hipGetLastError();
}

struct SlabMultiParams {
  SlabReduce r[RB_MAXL + 1];
  int ws[RB_MAXL + 1], nb_main[RB_MAXL + 1], nb_bias[RB_MAXL + 1], nb[RB_MAXL + 1];
  int nr;
};

__global__ void __launch_bounds__(SLAB_THREADS) slab_multi_kernel(SlabMultiParams g) {
  __shared__ f32x4 part[SLAB_PART_BYTES / 16];
  int bid = blockIdx.x;
#pragma unroll
  for (int j = 0; j < RB_MAXL + 1; ++j) {
    if (j >= g.nr) return;
    if (bid < g.nb[j]) {
      slab_reduce_any(g.ws[j], g.r[j], bid, g.nb_main[j], g.nb_bias[j], part);
      return;
    }
    bid -= g.nb[j];
  }
}

hipError_t slab_reduce_multi(const SlabReduce* r, int nr, hipStream_t s) {
  if (nr < 1 || nr > RB_MAXL + 1) return hipErrorInvalidValue;
  SlabMultiParams g{};
  g.nr = nr;
  int nb = 0;
  for (int j = 0; j < nr; ++j) {
    g.r[j] = r[j];
    g.r[j].sgd_serial = sgd_serial();
    g.ws[j] = slab_ws(r[j]);
    slab_blocks(r[j], g.nb_main[j], g.nb_bias[j], g.nb[j]);
    nb += g.nb[j];
  }
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(slab_multi_kernel, dim3(nb), dim3(SLAB_THREADS), 0, s, g);
  return hipGetLastError();
}

// ---- wide backward pairs (csrc/experiments/gemm_experiments.hip) ------------------------
// Off by default and built only on request: measured on the 8192-wide step (3 interleaved
// rounds, one box) 5.575 ms paired vs 5.540 separate (profiles/r2s2_wide_sgd_epilogue_pair_ab.txt).
// Without the experiments translation unit every pair is refused, so the engine launches the
// jobs separately.
void set_wide_pair(int on) {
  if (exp_set_wide_pair) exp_set_wide_pair(on);
}
bool wide_pair_wgrad_ok(int rows, int out_f, int in_f) {
  return exp_wide_pair_wgrad_ok && exp_wide_pair_wgrad_ok(rows, out_f, in_f);
}
bool wide_pair_dgrad_ok(int rows, int out_f, int in_f) {
  return exp_wide_pair_dgrad_ok && exp_wide_pair_dgrad_ok(rows, out_f, in_f);
}
hipError_t wide_pair(const WgradArgs& w1, const DgradArgs* dg, const WgradArgs* w2, hipStream_t s) {
  if (!exp_wide_pair) return hipErrorNotSupported;
  return exp_wide_pair(w1, dg, w2, s);
}

#if NNMPI_EXPERIMENTS_BUILD
// diagnostic: the 128x128 forward with per-block stamps (experiments translation unit)
hipError_t linear_fwd_bf16_stamped(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                                   bf16* Y, int ldy, int M, int N, int K, unsigned long long* stamps,
                                   hipStream_t s) {
  if (!exp_fwd_stamped) return hipErrorNotSupported;
  return exp_fwd_stamped(X, ldx, W, ldw, bias, Y, ldy, M, N, K, stamps, s);
}
#endif

bool experiments_built() { return exp_wide_pair != nullptr; }

}  // namespace nnmpi
