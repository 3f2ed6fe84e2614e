// Experiment kernels, built into the native library only with NNMPI_EXPERIMENTS=1 (_build.py).
// None of them is on the training path: each was built and measured against the production
// kernels and kept for re-measurement (docs/PERF.md §4, profiles/r2s2_*):
//   * gemm_bf16_pp256_ring_kernel  -- deep DMA ring twin of the 256x256 ping-pong kernel
//                                     (bench.py --gemm_variant 19..24): 3-10 % slower;
//   * gemm_bf16_pp256_pair_kernel  -- wgrad + SGD epilogue beside dgrad in one launch
//                                     (NNMPI_PAIR=1): 0.6 % slower on the wide step;
//   * gemm_bf16_dma_stamp_kernel   -- per-block entry/exit stamps of the 128x128 forward
//                                     (scripts/stamp_fwd.py).
// The production file reaches them through the weak references declared in gemm_tiles.h.
#include "kernels/gemm_tiles.h"
#include "knobs.h"

namespace nnmpi {

// Diagnostic twin of gemm_bf16_dma_kernel: every block records the constant 100 MHz real-time
// counter at entry and after its last store has retired (per-lane vector stores of two lanes,
// never a scalar store), so dispatch skew, per-block span and the launch's own overhead can be
// separated (scripts/stamp_fwd.py).  Not used by the training step.
template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int ACT, bool BIASGRAD, int NS>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_bf16_dma_stamp_kernel(GemmParams p,
                                                                           unsigned long long* st) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int gx = gridDim.x, gy = gridDim.y;
  const int lin = blockIdx.y * gx + blockIdx.x;
  const int bid = xcd_remap(lin, gx * gy);
  dma_gemm_tile<BM, BN, WGM, WGN, LA, LB, EPI, ACT, BIASGRAD, NS>(p, smem, bid % gx, bid / gx, blockIdx.z);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x < 2) st[2 * lin + threadIdx.x] = threadIdx.x ? t1 : t0;
}

hipError_t exp_fwd_stamped(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                                   bf16* Y, int ldy, int M, int N, int K, unsigned long long* stamps,
                                   hipStream_t s) {
  GemmParams p{};
  p.A = X; p.lda = ldx; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = Y; p.ldc = ldy; p.bias = bias;
  const long long a = (long long)(p.M - 1) * p.lda + p.K, b = (long long)(p.N - 1) * p.ldb + p.K;
  p.a_bytes = (unsigned)std::min<long long>(a * 2, DMA_OOB - 16);
  p.b_bytes = (unsigned)std::min<long long>(b * 2, DMA_OOB - 16);
  constexpr int smem = 2 * (128 + 128) * GEMM_BK * 2;
  auto kfn = gemm_bf16_dma_stamp_kernel<128, 128, 2, 4, KMAJ, KMAJ, EPI_BIAS_ACT, ACT_RELU, false, 2>;
  (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hipLaunchKernelGGL(kfn, dim3((N + 127) / 128, (M + 127) / 128, 1), dim3(512), smem, s, p, stamps);
  return hipGetLastError();
}


// Two independent 256x256 GEMMs in ONE launch (the wide model's backward: the weight gradient of
// layer i with its SGD epilogue beside the dgrad of layer i-1).  A weight-gradient tile ends in a
// memory-bound SGD epilogue (~18 B per parameter: master, momentum, bf16 shadow), a dgrad tile is
// compute-bound with a light epilogue; as separate launches every CU runs its SGD epilogues at
// the same time and HBM idles during the main loops.  Here the two jobs' blocks are interleaved
// in groups of 8 (one per XCD), so while some CUs stream an SGD epilogue others run MFMA main
// loops, and the launch boundary between them is gone.  Each job keeps its own tile order: job
// block j of n lands on XCD j % 8 exactly as in its own launch (n1, n2 multiples of 8), so
// xcd_remap / grouped_tile see the same ids.  Bitwise identical to the two launches.
template <int LA1, int LB1, int EPI1, int ACT1, bool BG1, int GM1,
          int LA2, int LB2, int EPI2, int ACT2, bool BG2, int GM2>
__global__ void __launch_bounds__(PP_THREADS) gemm_bf16_pp256_pair_kernel(GemmParams p1, GemmParams p2,
                                                                          int gx1, int gy1, int gx2,
                                                                          int gy2) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int n1 = gx1 * gy1, n2 = gx2 * gy2, m = min(n1, n2);
  const int b = blockIdx.x;
  int job, j;
  if (b < 2 * m) {
    job = (b >> 3) & 1;
    j = ((b >> 4) << 3) | (b & 7);
  } else {
    job = n1 > n2 ? 0 : 1;
    j = m + (b - 2 * m);
  }
  if (job == 0) pp256_tile<LA1, LB1, EPI1, ACT1, BG1, true, GM1>(p1, smem, xcd_remap(j, n1), gx1, gy1, 0);
  else pp256_tile<LA2, LB2, EPI2, ACT2, BG2, true, GM2>(p2, smem, xcd_remap(j, n2), gx2, gy2, 0);
}


// ------------------------------------------------------------------------------------------
// Deep-ring twin of gemm_bf16_pp256_kernel: the same tile, waves, phases, fragment reads and
// MFMA sections, but the LDS holds a RING of PP_RING = 10 half images (160 KiB, all of it)
// instead of 2 K-tile buffers (8 halves), and DMA issue is uniform: the phase that reads half
// q (read order q = 4t + ph: A0(t), B1(t), A1(t), B0(t+1); B0(0) is q = -1) issues half q + 8.
//   slot(q) = (q + 1) mod 10;  slot(q + 8) == slot(q - 2): a half is restaged two phases after
//   its read (the WAR margin of the 8-slot kernel, see LATE_LGKM above);
//   before phase q's first barrier a counted vmcnt(14) retires half q + 1 (7 newer halves x 2
//   DMA instructions per wave stay in flight), read in phase q + 1 (RAW, as above).
// So 7-8 halves (112-128 KiB) are in flight per CU instead of 5-6: the L2/MALL -> LDS stream of
// a 256x256 tile needs ~75 GB/s per CU at the MFMA rate, and the deeper issue-ahead is the
// lever docs/PERF.md §4 names for the gap to hipBLASLt.
// ------------------------------------------------------------------------------------------
constexpr int PP_RING = 10;
constexpr int PP_RING_SMEM = PP_RING * PP_HALF;   // 160 KiB (the R = 8 forms use 128 KiB of it)

// MODE 0: one half per phase, half q + D (D = R - 2) in phase q;  MODE 1: two halves in each
// light phase (P2, P4: 4 fragment reads), q + D - 1 and q + D, none in P1 / P3 (8 reads each).
// Either way the slot of the newest half is the slot of half q - 2 (WAR margin 2 phases) and the
// vmcnt before phase q's barrier leaves (newest issued - (q + 1)) halves x 2 instructions.
template <int LA, int LB, int EPI, int ACT, bool BIASGRAD, int R = 10, int MODE = 0, int GM = 4>
__global__ void __launch_bounds__(PP_THREADS) gemm_bf16_pp256_ring_kernel(GemmParams p) {
  static_assert(R == 6 || R == 8 || R == 10, "ring of 6, 8 or 10 half images");
  constexpr int D = R - 2;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr int BK = GEMM_BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int gx = gridDim.x, gy = gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
  int tx, ty;
  grouped_tile(bid, gx, gy, GM, tx, ty);
  const int split = blockIdx.z;
  const int m0 = ty * 256, n0 = tx * 256;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)p.b_bytes, 0x00020000);
  DmaPlan<128, LA, 8> pa0, pa1;
  DmaPlan<128, LB, 8> pb0, pb1;
  pa0.init(w, lane, m0, p.M, p.lda);
  pa1.init(w, lane, m0 + 128, p.M, p.lda);
  pb0.init(w, lane, n0, p.N, p.ldb);
  pb1.init(w, lane, n0 + 128, p.N, p.ldb);
  auto slot = [&](int q) { return smem + ((q + 1 + R) % R) * PP_HALF; };
  auto kof = [&](int t) { return kbeg + t * BK; };
  // issue half q of the read order (its type is q & 3; q = -1 is B0(0))
  auto issue = [&](int q) {
    const int r = q & 3, t = q >> 2;   // arithmetic shift: q = -1 -> r 3, t -1 -> B0(0)
    char* dst = slot(q);
    if (r == 0) pa0.issue(rsA, dst, w, kof(t), kend);
    else if (r == 1) pb1.issue(rsB, dst, w, kof(t), kend);
    else if (r == 2) pa1.issue(rsA, dst, w, kof(t), kend);
    else pb0.issue(rsB, dst, w, kof(t + 1), kend);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsum[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rsum[i] = 0.f;
  const bool do_bg = BIASGRAD && tx == 0 && wn == 0;

  // prologue: halves -1 .. D - 1; retire -1 and 0
#pragma unroll
  for (int q = -1; q < D; ++q) issue(q);
  wait_vm<2 * (D - 1)>();
  __builtin_amdgcn_s_barrier();

  bf16x8 af[4][2], b0f[2][2], b0n[2][2], b1f[2][2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) b0n[jj][kk] = read_frag_async<128, LB>(slot(-1), wn * 32 + jj * 16, kk, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (wm == 1) __builtin_amdgcn_s_barrier();   // wave row 1 runs one barrier behind

  for (int t = 0; t < nt; ++t) {
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int q = 4 * t + ph;
      const char* cur = slot(q);
      if (ph == 0 || ph == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag_async<128, LA>(cur, wm * 64 + i * 16, kk, lane);
      }
      if (ph == 0) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0f[jj][kk] = b0n[jj][kk];
      } else if (ph == 1) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b1f[jj][kk] = read_frag_async<128, LB>(cur, wn * 32 + jj * 16, kk, lane);
      } else if (ph == 3) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0n[jj][kk] = read_frag_async<128, LB>(cur, wn * 32 + jj * 16, kk, lane);
      }
      // newest half(s) (types compile-time per phase) into the slot(s) of halves q - 3, q - 2
      if constexpr (MODE == 0) {
        issue(q + D);
      } else if (ph & 1) {
        issue(q + D - 1);
        issue(q + D);
      }
      // half q + 1 has landed (this wave's part): (newest - (q + 1)) halves stay in flight
      if (MODE == 0 || (ph & 1)) wait_vm<2 * (D - 1)>();
      else wait_vm<2 * (D - 2)>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int hA = ph >> 1;
      const int hB = (ph == 1 || ph == 2) ? 1 : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            acc[hA * 4 + i][hB * 2 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                hB ? b1f[jj][kk] : b0f[jj][kk], af[i][kk], acc[hA * 4 + i][hB * 2 + jj], 0, 0, 0);
      if constexpr (BIASGRAD) {
        if (do_bg && (ph == 0 || ph == 2)) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
              for (int e = 0; e < 8; ++e) rsum[hA * 4 + i] += (float)af[i][kk][e];
        }
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();   // balance the stagger
  wait_vm<0>();                                  // trailing out-of-range DMAs
  f32x4 accb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float v = rsum[i];
    if constexpr (BIASGRAD) {
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
    }
    accb[i] = f32x4{v, v, v, v};
  }
  int mrow[8], ncol[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) mrow[i] = m0 + (i >> 2) * 128 + wm * 64 + (i & 3) * 16 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) ncol[j] = n0 + (j >> 1) * 128 + wn * 32 + (j & 1) * 16 + (lane >> 4) * 4;
  epilogue_store<8, 4, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, mrow, ncol, lane, split);
}

// ---- host side -------------------------------------------------------------------------------
hipError_t exp_pp256_ring(int variant, int la, int lb, int epi, int act, int bg, GemmParams p,
                          dim3 grid, hipStream_t s) {
  // 19..24: 10 slots / 8 slots, one half per phase; 10 / 8 slots, two halves in each light
  // phase; 6 slots, one / two (all GM 4)
  if (variant < 19 || variant > 24) return hipErrorInvalidValue;
  const int smem = variant >= 23 ? 6 * PP_HALF : (variant & 1) ? PP_RING_SMEM : PP_SMEM;
  using K = void (*)(GemmParams);
  K kfn = nullptr;
#define NNMPI_RING(LA, LB, EPI, ACT, BG)                                                        \
  if (la == LA && lb == LB && epi == EPI && act == ACT && bg == (int)BG) {                     \
    static const K f[6] = {gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 10, 0>,           \
                           gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 8, 0>,            \
                           gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 10, 1>,           \
                           gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 8, 1>,            \
                           gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 6, 0>,            \
                           gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 6, 1>};           \
    kfn = f[variant - 19];                                                                     \
  }
  NNMPI_RING(KMAJ, KMAJ, EPI_BIAS_ACT, ACT_RELU, false)
  NNMPI_RING(KMAJ, KMAJ, EPI_BIAS_ACT, ACT_TANH, false)
  NNMPI_RING(KMAJ, KMAJ, EPI_BIAS_ACT, ACT_NONE, false)
  NNMPI_RING(KMAJ, XMAJ, EPI_DACT, ACT_RELU, false)
  NNMPI_RING(KMAJ, XMAJ, EPI_DACT, ACT_TANH, false)
  NNMPI_RING(KMAJ, XMAJ, EPI_DACT, ACT_NONE, false)
  NNMPI_RING(XMAJ, XMAJ, EPI_F32, ACT_NONE, true)
  NNMPI_RING(XMAJ, XMAJ, EPI_F32, ACT_NONE, false)
  NNMPI_RING(KMAJ, KMAJ, EPI_F32, ACT_NONE, false)
  NNMPI_RING(KMAJ, XMAJ, EPI_F32, ACT_NONE, false)
  NNMPI_RING(XMAJ, KMAJ, EPI_F32, ACT_NONE, false)
#undef NNMPI_RING
  if (!kfn) return hipErrorNotSupported;
  (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
  hipLaunchKernelGGL(kfn, grid, dim3(PP_THREADS), smem, s, p);
  return hipGetLastError();
}

static int g_pair = -1;   // 1 on, 0 off (default; NNMPI_PAIR=1 / set_wide_pair)
void exp_set_wide_pair(int on) { g_pair = on; }
static bool pair_enabled() {
  if (g_pair < 0) {
    const char* e = knob_env("NNMPI_PAIR");
    g_pair = (e && e[0] == '1') ? 1 : 0;
  }
  return g_pair == 1 && gemm_host::default_path();
}
static bool tiles256_x8(int M, int N) {
  const long long t = (long long)((M + 255) / 256) * ((N + 255) / 256);
  return t >= 256 && t % 8 == 0;
}
bool exp_wide_pair_wgrad_ok(int rows, int out_f, int in_f) {
  return pair_enabled() && gemm_host::wgrad_tile(out_f, in_f) == 256 && tiles256_x8(out_f, in_f) &&
         wgrad_splits(out_f, in_f, rows) == 1;
}
bool exp_wide_pair_dgrad_ok(int rows, int out_f, int in_f) {
  // dgrad output: rows x in_f
  return pair_enabled() && gemm_host::pick_tile(rows, in_f) == 256 && tiles256_x8(rows, in_f);
}

template <typename F>
static void pp_attr_once(F f) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_SMEM);
    done = true;
  }
}

hipError_t exp_wide_pair(const WgradArgs& w1, const DgradArgs* dg, const WgradArgs* w2, hipStream_t s) {
  if ((dg == nullptr) == (w2 == nullptr)) return hipErrorInvalidValue;
  if (!exp_wide_pair_wgrad_ok(w1.K, w1.M, w1.N) || !w1.db) return hipErrorInvalidValue;
  GemmParams p1, p2;
  SlabReduce r1, r2;
  gemm_host::make_wgrad(w1, p1, r1);
  set_extents<XMAJ, XMAJ>(p1);
  const int gx1 = (w1.N + 255) / 256, gy1 = (w1.M + 255) / 256;
  int gx2, gy2;
  if (w2) {
    if (!exp_wide_pair_wgrad_ok(w2->K, w2->M, w2->N) || !w2->db) return hipErrorInvalidValue;
    gemm_host::make_wgrad(*w2, p2, r2);
    set_extents<XMAJ, XMAJ>(p2);
    gx2 = (w2->N + 255) / 256; gy2 = (w2->M + 255) / 256;
  } else {
    // dZ[M rows][K out] x W[K out][N in] -> dX[M][N], times act'(Aprev)
    if (!exp_wide_pair_dgrad_ok(dg->M, dg->K, dg->N)) return hipErrorInvalidValue;
    p2 = GemmParams{};
    p2.A = dg->dZ; p2.lda = dg->lddz; p2.B = dg->W; p2.ldb = dg->ldw;
    p2.M = dg->M; p2.N = dg->N; p2.K = dg->K;
    p2.k_per_split = ((dg->K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
    p2.C = dg->dX; p2.ldc = dg->lddx; p2.aux = dg->Aprev; p2.ldaux = dg->lda_prev;
    set_extents<KMAJ, XMAJ>(p2);
    gx2 = (dg->N + 255) / 256; gy2 = (dg->M + 255) / 256;
  }
  const dim3 grid(gx1 * gy1 + gx2 * gy2), blk(PP_THREADS);
#define NNMPI_PAIR_LAUNCH(...)                                                                     \
  {                                                                                                \
    auto kfn = gemm_bf16_pp256_pair_kernel<XMAJ, XMAJ, EPI_F32, ACT_NONE, true, 1, __VA_ARGS__>;   \
    pp_attr_once(kfn);                                                                             \
    hipLaunchKernelGGL(kfn, grid, blk, PP_SMEM, s, p1, p2, gx1, gy1, gx2, gy2);                   \
    return hipGetLastError();                                                                      \
  }
  if (w2) NNMPI_PAIR_LAUNCH(XMAJ, XMAJ, EPI_F32, ACT_NONE, true, 1)
  switch (dg->act) {
    case ACT_RELU: NNMPI_PAIR_LAUNCH(KMAJ, XMAJ, EPI_DACT, ACT_RELU, false, 4)
    case ACT_TANH: NNMPI_PAIR_LAUNCH(KMAJ, XMAJ, EPI_DACT, ACT_TANH, false, 4)
    default: NNMPI_PAIR_LAUNCH(KMAJ, XMAJ, EPI_DACT, ACT_NONE, false, 4)
  }
#undef NNMPI_PAIR_LAUNCH
}

}  // namespace nnmpi
