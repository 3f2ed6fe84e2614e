// 256 x 256 forward GEMM tile with FOUR waves of 128 x 128 (the ISA
// tabulation in profiles/r4_isa_tab_wide8192_vs_hipblaslt.json): the shape hipBLASLt runs for
// the 8192-wide layers.  Each wave owns 8 x 8 MFMA tiles (256 fp32 accumulators per lane: one
// wave per SIMD, accumulators in AGPRs) and hides its OWN LDS reads behind its MFMAs -- the
// 8-wave ping-pong kernel (pp256_tile) instead hides memory work across waves and pays 8
// barriers + 21 lgkmcnt waits per K tile for it.
//
// LDS: five 32-deep stages (160 KiB), four in flight beside the one being read -- 128 KiB of
// L2 -> LDS traffic in flight per CU, the depth a 256 x 256 tile needs at the MFMA rate (it
// consumes 64 KiB per 0.98 us; a 2-stage 64-deep ring kept one stage in flight: 455 us).  Per
// stage t: the MFMAs of its first 16-deep k-step run beside the reads of its second; then wait
// for stage t+1, ONE barrier, the DMA of stage t+4 into the slot stage t-1 used, and the second
// k-step's MFMAs run beside the reads of stage t+1's first k-step.
// v_mfma_f32_32x32x16_bf16 (4 x 4 tiles per wave): a 16-deep k-step needs 8 fragments (32
// VGPRs), so double-buffering per k-step costs 64 VGPRs beside the 256 accumulators (16x16x32
// tiles needed 128 and hipcc shuffled accumulators through VGPRs: 240 v_accvgpr moves per K
// tile).  sched_group_barrier pins 1 ds_read per 2 MFMAs.  Not bitwise equal to pp256_tile (a
// different MFMA shape sums k in 16-deep pieces).
#include "kernels/gemm_tiles.h"

namespace nnmpi {

constexpr int W4_THREADS = 256;
constexpr int W4_BK = 32;                          // k per LDS stage
constexpr int W4_NS = 5;                           // stages: 4 in flight beside the one read
constexpr int W4_OP = 256 * W4_BK * 2;             // one operand's stage image: 16 KiB
constexpr int W4_STAGE = 2 * W4_OP;
constexpr int W4_SMEM = W4_NS * W4_STAGE;          // 160 KiB: the whole LDS

// KMAJ stage image of 256 rows x 32 k: rows of 64 B (4 chunks of 8 k), chunk c of row r at
// c ^ ((r >> 2) & 3) -- the 16 rows a ds_read_b128 phase reads hit 16 distinct 16-byte slots
__device__ __forceinline__ int w4_off(int r, int k8) { return r * 64 + ((k8 ^ ((r >> 2) & 3)) << 4); }

// LDS-DMA of one operand stage (full tiles only: M, N % 256, K % 32): 16 x 1 KiB, 4 per wave.
// Instruction q of wave w covers rows 16 (4w + q) + (lane >> 2), image chunk lane & 3, source
// chunk (lane & 3) ^ ((row >> 2) & 3) -- the same for every q (16-row steps keep (row >> 2) & 3),
// so one per-lane offset and a row stride describe all four.
struct W4Dma {
  unsigned off, step;
  __device__ __forceinline__ void init(int w, int lane, int x0, int ld) {
    const int r = 64 * w + (lane >> 2), cp = lane & 3;
    off = (unsigned)(((long long)(x0 + r) * ld + ((cp ^ ((r >> 2) & 3)) << 3)) * 2);
    step = (unsigned)(16 * ld * 2);
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* stage, int w, int k0) const {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(stage + (4 * w + q) * 1024), 16,
          off + (unsigned)q * step + (unsigned)k0 * 2u, 0, 0, 0);
  }
};

// 32-row operand fragment of v_mfma_f32_32x32x16_bf16 (lane l: row xb + (l & 31), k = 16 ks +
// 8 (l >> 5) + j) -- one 16-byte chunk of the stage image
__device__ __forceinline__ bf16x8 w4_frag(const char* img, int xb, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + w4_off(xb + (lane & 31), ks * 2 + (lane >> 5)));
}

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int ACT>
__global__ void __launch_bounds__(W4_THREADS, 1) gemm_w4_fwd_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int gx = gridDim.x, gy = gridDim.y;
  int tx, ty;
  grouped_tile(xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy), gx, gy, 4, tx, ty);
  const int m0 = ty * 256, n0 = tx * 256;
  const int nt = p.K / W4_BK;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)p.b_bytes, 0x00020000);
  W4Dma da, db;
  da.init(w, lane, m0, p.lda);
  db.init(w, lane, n0, p.ldb);
  auto SA = [&](int i) { return smem + i * W4_STAGE; };
  auto SB = [&](int i) { return smem + i * W4_STAGE + W4_OP; };
  auto issue = [&](int t) {
    const int i = t % W4_NS;
    da.issue(rsA, SA(i), w, t * W4_BK);
    db.issue(rsB, SB(i), w, t * W4_BK);
  };

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // prologue: stages 0..3 in flight (8 DMA instructions per wave each), stage 0 landed
  for (int t = 0; t < W4_NS - 1; ++t)
    if (t < nt) issue(t);
  if (nt >= 4) wait_vm<24>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  bf16x8 fa[2][4], fb[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[0][i] = w4_frag(SA(0), wm * 128 + i * 32, 0, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = w4_frag(SB(0), wn * 128 + j * 32, 0, lane);

  for (int t = 0; t < nt; ++t) {
    const int cur = t % W4_NS, nxt = (t + 1) % W4_NS;
    // ---- k-step 0 of stage t: MFMAs beside the reads of k-step 1 ----
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[1][i] = w4_frag(SA(cur), wm * 128 + i * 32, 1, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[1][j] = w4_frag(SB(cur), wn * 128 + j * 32, 1, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[0][j], fa[0][i], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // 2 MFMA
    }
    // ---- stage t+1 landed (stages t+2, t+3 may stay in flight); every wave's reads of stage
    // t-1 returned in the previous step: refill its slot with stage t+4 ----
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int newer = min(2, nt - 2 - t);   // issued stages younger than t+1
    if (newer >= 2) wait_vm<16>();
    else if (newer == 1) wait_vm<8>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (t + W4_NS - 1 < nt) issue(t + W4_NS - 1);
    // ---- k-step 1: MFMAs beside the reads of stage t+1's k-step 0 (a stale slot on the last
    // stage, unused: unconditional so reads and MFMAs form one scheduling region) ----
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[0][i] = w4_frag(SA(nxt), wm * 128 + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[0][j] = w4_frag(SB(nxt), wn * 128 + j * 32, 0, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[1][j], fa[1][i], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
  }
  // ---- epilogue: act(acc + bias) -> bf16.  Operands swapped (B first): lane holds row
  // m = .. + (lane & 31) of C and, per register group cg, 4 consecutive n = 8 cg + 4 (lane >> 5) ----
  bf16* C = reinterpret_cast<bf16*>(p.C);
  const int m_l = lane & 31, n_l = 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int cg = 0; cg < 4; ++cg) {
      const int n = n0 + wn * 128 + j * 32 + 8 * cg + n_l;
      const f32x4 bias = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * 128 + i * 32 + m_l;
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)act_fwd_t<ACT>(acc[i][j][4 * cg + e] + bias[e]);
        *reinterpret_cast<bf16x4*>(C + (long long)m * p.ldc + n) = o;
      }
    }
}

// Forward Y = act(X W^T + b) on the 4-wave tile (experiment: scripts/r4_w4_ab.py).  M, N
// multiples of 256, K of 64, N of 4 for the bias vector loads.
hipError_t gemm_w4_fwd(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias, bf16* Y,
                       int ldy, int M, int N, int K, int act, hipStream_t s) {
  if (M % 256 || N % 256 || K % W4_BK || K < W4_BK) return hipErrorInvalidValue;
  GemmParams p{};
  p.A = X; p.lda = ldx; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = K;
  p.C = Y; p.ldc = ldy; p.bias = bias;
  set_extents<KMAJ, KMAJ>(p);
  using Fn = void (*)(GemmParams);
  static const Fn fns[3] = {gemm_w4_fwd_kernel<ACT_NONE>, gemm_w4_fwd_kernel<ACT_RELU>, gemm_w4_fwd_kernel<ACT_TANH>};
  static bool attr = false;
  if (!attr) {
    for (Fn f : fns) (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, W4_SMEM);
    attr = true;
  }
  const Fn f = fns[act == ACT_RELU ? 1 : act == ACT_TANH ? 2 : 0];
  hipLaunchKernelGGL(f, dim3(N / 256, M / 256), dim3(W4_THREADS), W4_SMEM, s, p);
  return hipGetLastError();
}

}  // namespace nnmpi
