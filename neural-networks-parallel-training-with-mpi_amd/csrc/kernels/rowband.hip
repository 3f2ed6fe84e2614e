// Row-band step for narrow MLPs (equal hidden widths H = 256..1024, input width % 64, a
// regression head out == 1 with MSE): the reference's whole forward, loss and activation-gradient
// chain (ref.py:42-44,170-176: Linear+ReLU x L-1, Linear, MSELoss, and autograd's mm /
// threshold_backward down to dZ_0) in ONE launch, then every weight gradient in ONE grouped
// launch and every combine (+ the fused SGD-momentum update on one rank) in ONE more.
//
// Why: everything up to the weight gradients is ROW-LOCAL -- row r of a_l depends only on row r
// of a_{l-1}, the head's dlogit of row r only on row r of a_{L-2}, and row r of dZ_{l-1} only on
// row r of dZ_l.  A block that owns a band of 32 rows can therefore run all of it with the
// activations resident in LDS, and only the weights stream in: 512 x 512 bf16 = 512 KiB per
// layer, resident in every XCD's L2 after the first touch (1.5 MiB for three layers), read
// with 16-byte loads straight into MFMA B fragments.  The 128x128-tile launches it replaces pay
// a launch boundary, a first-fetch / epilogue fixed cost and an activation re-read from the
// Infinity Cache per GEMM (docs/PERF.md "Where a launch's time goes"): 8 launches per step
// become 3.
//
// Block = 8 waves (512 threads) x 32 rows; wave w owns H/8 output columns of every layer
// (2 x H/128 v_mfma_f32_16x16x32_bf16 tiles).  The weights stream from fragment-major images
// (one 16-byte load per lane fills one MFMA operand) straight into registers; the LDS holds only
// the band's activation images (see "v2" below).  After each pass the image is copied out
// row-contiguously (activations and dZ are needed by the weight gradients).  (The first form of
// this kernel staged every weight k-step through LDS: 52 vs 40 us per step, round 4.)
#include "gemm_tiles.h"
#include "knobs.h"

namespace nnmpi {

constexpr int RB_ROWS = 32;
constexpr int RB_WAVES = 8;
constexpr int RB_THREADS = 64 * RB_WAVES;
// byte offset of element (row r, column k) in an activation image
__device__ __forceinline__ int rb_off(int r, int k) {
  return (k >> 6) * (RB_ROWS * 128) + kmaj_off(r, (k >> 3) & 7) + ((k & 7) << 1);
}

// Row-contiguous copy between an LDS image and a [rows][ld] bf16 matrix (rows row0 .. row0 +
// nvalid - 1): each wave moves whole 128-byte row pieces (8 lanes per row).
template <int H>
__device__ __forceinline__ void rb_copy_out(const char* img, bf16* dst, int ld, int nvalid, int tid,
                                            int pol) {
  constexpr int CH = RB_ROWS * H / 8;
#pragma unroll
  for (int it = 0; it < CH / RB_THREADS; ++it) {
    const int id = tid + it * RB_THREADS;
    const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8));
    if (r < nvalid) store16(reinterpret_cast<bf16x8*>(dst + (long long)r * ld + kb * 64 + k8 * 8), v, pol);
  }
}

// =============================================================================================
// v2: packed weights streamed straight into MFMA fragments.
//
// The v1 passes above move every weight byte global -> VGPR -> ds_write -> ds_read -> MFMA: per
// CU and 64-deep k-step 64 KiB of LDS writes plus 64 KiB of LDS reads on top of the 64 KiB the
// L2 delivers, and ~2.7 non-MFMA VALU per MFMA (profiles/r3s2_rowband_pmc.txt).  Here the weights
// are kept (besides the arena's row-major bf16 shadow) in a FRAGMENT-MAJOR image: 1 KiB per
// 16 x 32 operand fragment, lane l's 16 bytes at l * 16, so ONE global_load_dwordx4 fills one
// v_mfma_f32_16x16x32_bf16 operand with a whole contiguous KiB (8 full cache lines).  Two images
// per hidden layer: W (forward B operand, [out][in]) and W^T (dgrad B operand, [in][out]).  The
// weights never touch the LDS; the LDS holds only the band's activation images.
//
// Each wave's weight loads form ONE stream across all matrices of the step (forward layers,
// then the dgrad layers): a D-deep register ring of k-steps whose refills run past the end of a
// matrix into the next one, so the epilogue, barrier, copy-out and head of a layer overlap the
// next layer's first weight fetches.
//
// LDS: max(nh, 2) activation slots of RB_ROWS x max(H, in) bf16 (KMAJ image per 64-deep block),
// no ping-pong barrier: forward layer l reads slot S_{l-1} (slot 0 = the input rows) and writes
// slot S_l, so every saved activation the dgrads need stays resident; the head works in place
// on a_{nh-1}; dgrad l writes dZ_{l-1} in place over its own act'(a_{l-1}) operand (each lane
// reads then writes the same elements).  One barrier per layer.
// =============================================================================================
// k-steps of the register ring (1 being consumed, D-1 in flight).  The ring is what hides the
// L2 latency: at D = 2 (8 KiB in flight per wave) the proxy's band streamed ~60 GB/s per CU,
// latency-bound (profiles/r4_rowband_v2_*).  Deeper where the registers allow it (every matrix
// of the stream must have a multiple of D k-steps: its ring phase is compile-time).
template <int H>
constexpr int rb2_depth() { return (H == 256 || H == 512) ? 4 : 2; }
static int rb2_depth_rt(int H) { return (H == 256 || H == 512) ? 4 : 2; }

template <int H>
struct Rb2Geom {
  static_assert(H % 128 == 0 && H >= 256 && H <= 1024, "row-band v2: H = 256 .. 1024, H % 128 == 0");
  static constexpr int NJ = H / 128;          // 16-column MFMA tiles per wave (8 waves x NJ x 16 = H)
  static constexpr int NF = 2 * NJ;           // 1 KiB operand fragments per 64-deep k-step per wave
  static constexpr int WCOLS = H / RB_WAVES;  // output columns per wave
  static constexpr int KB_BYTES = RB_ROWS * 128;
};

// One k-step (NF fragments) of the weight stream into ring slot `dst`: matrix base `b` (already
// offset to this wave's first tile), `ts` bytes between the wave's tiles, k-step `s`.  The loads
// are inline asm, counted by hand (rb2_wait): hipcc's own vmcnt bookkeeping merges the ring's
// loop-carried slots conservatively at the loop headers and waited for nearly the whole ring in
// the first sub-step (vmcnt(3) where 24 loads may stay in flight), so the ring bought nothing.
// kk-major issue order: the first k-half's fragments land first.  SGPR base + one lane-offset
// VGPR per load (global_load_dwordx4 v, v_off, s[base]).
template <int NJ>
__device__ __forceinline__ void rb2_issue(bf16x8 (&dst)[2 * NJ], const char* b, int ts, int s, int voff) {
  const char* base = b + s * 2048;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const char* bj = base + j * ts;
      if (kk == 0)
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst[2 * j]) : "v"(voff), "s"(bj));
      else
        asm volatile("global_load_dwordx4 %0, %1, %2 offset:1024" : "=v"(dst[2 * j + 1]) : "v"(voff), "s"(bj));
    }
}

// Wait until at most N of this wave's vector-memory operations are outstanding, then pin the
// k-half `kk` fragments of `f` behind the wait (their consumers cannot be hoisted above it; the
// asm loads' destinations count as written at issue for the compiler -- cdna_hip_programming.md
// §5.7 item 1, form (ii)).
template <int N, int NJ>
__device__ __forceinline__ void rb2_wait(bf16x8 (&f)[2 * NJ], int kk) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N));
#pragma unroll
  for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(f[2 * j + kk]));
}

// The stream's matrix q: forward layers 0 .. nh-1, then the dgrad images of layers nh-1 .. 1;
// past the end, the last matrix again with a zero tile stride (L1-resident dummy refills).
struct Rb2Mat {
  const char* b;   // this wave's first tile
  int ts;          // bytes between the wave's tiles
  int ks;          // 64-deep k-steps
};
template <int H>
__device__ __forceinline__ Rb2Mat rb2_mat(const RowbandArgs& p, int q, int t0) {   // t0: first 16-col tile
  const int nh = p.nh;
  const bool past = q >= 2 * nh - 1;
  if (past) q = 2 * nh - 2;
  const char* base;
  int K;
  if (q < nh) {
    base = reinterpret_cast<const char*>(p.Pf[q]);
    K = q == 0 ? p.in : H;
  } else {
    base = reinterpret_cast<const char*>(p.Pd[2 * nh - 1 - q]);
    K = H;
  }
  const int ts = (K >> 5) * 1024;
  Rb2Mat m;
  m.b = base + (long long)t0 * ts;
  m.ts = past ? 0 : ts;
  m.ks = K >> 6;
  return m;
}

// Main loop of one matrix: acc[i][j] += band rows 16i.. x fragments of this wave's tile j, the
// B operand from the ring.  Slot d holds k-step s0 + d on entry to sub-step d; after its MFMAs
// it is refilled with k-step s0 + d + D of this matrix or, past its end, of the next one.  (A
// do-while: every matrix has >= D k-steps, and a loop the compiler must assume can be skipped
// makes it wait for the refills at the loop exit -- rule: no global load between the ring
// refills and their use, or vmcnt drains the ring.)
template <int NJ, int D>
__device__ __forceinline__ void rb2_mainloop(bf16x8 (&ring)[D][2 * NJ], f32x4 (&acc)[2][NJ],
                                             const char* img, const Rb2Mat& cur, const Rb2Mat& nxt,
                                             int lane) {
  constexpr int NF = 2 * NJ, KB_BYTES = RB_ROWS * 128;
  const int voff = lane * 16;
  int s0 = 0;
  do {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = s0 + d;
      const char* kb = img + s * KB_BYTES;
      bf16x8 af[2][2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i][kk] = read_frag<64, KMAJ>(kb, 16 * i, kk, lane);
      // slot d: every later slot (D - 1 k-steps) may stay in flight, and the second k-half
      rb2_wait<(D - 1) * NF + NJ, NJ>(ring[d], 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[d][2 * j], af[i][0], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);   // (the first half's MFMAs stay ahead of the second wait)
      rb2_wait<(D - 1) * NF, NJ>(ring[d], 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[d][2 * j + 1], af[i][1], acc[i][j], 0, 0, 0);
      // (sched_barrier: the refill stays behind this sub-step's MFMAs, which read the slot)
      __builtin_amdgcn_sched_barrier(0);
      const int sn = s + D;
      const bool inc = sn < cur.ks;
      rb2_issue<NJ>(ring[d], inc ? cur.b : nxt.b, inc ? cur.ts : nxt.ts, inc ? sn : sn - cur.ks, voff);
      __builtin_amdgcn_sched_barrier(0);
    }
    s0 += D;
  } while (s0 < cur.ks);
}

// LDS parameter block after the activation slots (floats): every bias, the head weight, the
// band's targets, the head bias and the head's per-row scratch.  Loaded once at kernel start:
// a global load issued after the ring's refills would make its wait drain the whole ring.
struct Rb2Par {
  float* bias;   // [nh][H]
  float* wh;     // [H]
  float* y;      // [RB_ROWS]
  float* bh;     // [4]
  float* dls;    // [RB_ROWS]
  float* lss;    // [RB_ROWS]
};
__host__ __device__ __forceinline__ int rb2_par_bytes(int H, int nh) {
  return ((nh + 1) * H + 3 * RB_ROWS + 4) * 4;
}
__device__ __forceinline__ Rb2Par rb2_par(char* base, int H, int nh) {
  Rb2Par q;
  q.bias = reinterpret_cast<float*>(base);
  q.wh = q.bias + nh * H;
  q.y = q.wh + H;
  q.bh = q.y + RB_ROWS;
  q.dls = q.bh + 4;
  q.lss = q.dls + RB_ROWS;
  return q;
}

// The band's head weight/bias-gradient and loss partials (deterministic): column pair
// (2c, 2c+1) by lanes l and l + 32 of one wave -- rows 0..15 and 16..31, 4-byte LDS reads -- then
// one shuffle adds the two halves; the bias and loss partials by one 32-lane shuffle tree.  (One
// thread per column over all 32 rows with 2-byte reads, plus one thread summing the 32 bias and
// loss terms serially, took ~2.5 us of the head: profiles/r5_rowband_stamps.txt.)
template <int H>
__device__ __forceinline__ void rb2_head_partials(const RowbandArgs& p, const char* act,
                                                  const float* dls, const float* lss, int tid,
                                                  int band) {
  const int lane = tid & 63, h = lane >> 5;
  float dl[16];
#pragma unroll
  for (int i = 0; i < 16; i += 4) {
    const f32x4 d4 = *reinterpret_cast<const f32x4*>(dls + 16 * h + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) dl[i + e] = d4[e];
  }
#pragma unroll
  for (int it = 0; it < (H / 2 + RB_THREADS / 2 - 1) / (RB_THREADS / 2); ++it) {
    const int c = (tid >> 6) * 32 + (lane & 31) + it * (RB_THREADS / 2);   // column pair
    if (c < H / 2) {
      const int k = 2 * c;
      const char* base = act + (k >> 6) * (RB_ROWS * 128) + ((k & 7) << 1);
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = 16 * h + i;
        const bf16x2 v = *reinterpret_cast<const bf16x2*>(base + kmaj_off(r, (k >> 3) & 7));
        s0 = fmaf(dl[i], (float)v[0], s0);
        s1 = fmaf(dl[i], (float)v[1], s1);
      }
      s0 += __shfl_xor(s0, 32, 64);
      s1 += __shfl_xor(s1, 32, 64);
      if (h == 0) {
        float2 o;
        o.x = s0;
        o.y = s1;
        *reinterpret_cast<float2*>(p.wslab + (long long)band * H + k) = o;
      }
    }
  }
  if (tid < 64) {
    float b = tid < RB_ROWS ? dls[tid] : 0.f, l = tid < RB_ROWS ? lss[tid] : 0.f;
#pragma unroll
    for (int sh = 16; sh >= 1; sh >>= 1) {
      b += __shfl_xor(b, sh, 64);
      l += __shfl_xor(l, sh, 64);
    }
    if (tid == 0) {
      p.bslab[band] = b;
      p.loss_part[band] = l;
    }
  }
}

// Regression head of the band (out == 1, MSE) in place on `z` = a_{nh-1}: logit, loss, dlogit,
// the band's head-gradient partials, then dZ_{nh-1} = dl * w * act'(a) over a.
// LDS bytes of the v2 kernel: the activation slots and the parameter block (8-byte aligned)
__host__ __device__ __forceinline__ int rb2_smem_core(int H, int in, int nh) {
  return (((nh > 2 ? nh : 2) * RB_ROWS * (H > in ? H : in) * 2 + rb2_par_bytes(H, nh)) + 7) & ~7;
}

template <int H, int ACT, typename Stamp, typename Flush>
__device__ __forceinline__ void rb2_head(const RowbandArgs& p, char* z, const Rb2Par& q, int nvalid, int tid,
                                         int band, Stamp&& stamp, Flush&& flush) {
  constexpr int CPT = H / 8 / 16;   // 8-column chunks per thread (16 threads per row)
  const int r = tid >> 4, g = tid & 15;
  // (a and w are re-read from the LDS for the dZ pass instead of held: the weight ring is live
  // across the head, and holding them costs 16 * CPT registers)
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int k = 8 * (g + 16 * c);
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(z + rb_off(r, k));
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(q.wh + k);
    const f32x4 w1 = *reinterpret_cast<const f32x4*>(q.wh + k + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) dot += (float)v[e] * w0[e];
#pragma unroll
    for (int e = 0; e < 4; ++e) dot += (float)v[4 + e] * w1[e];
  }
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) dot += __shfl_xor(dot, sh, 64);
  const bool valid = r < nvalid;
  const float d = dot + q.bh[0] - q.y[r];
  const float dl = valid ? 2.f * d * p.inv_count : 0.f;
  if (g == 0) {
    q.dls[r] = dl;
    q.lss[r] = valid ? d * d : 0.f;
  }
  flush();   // the last forward layer's copy-out, before dZ replaces a (behind the next barrier)
  stamp();
  __syncthreads();
  stamp();
  rb2_head_partials<H>(p, z, q.dls, q.lss, tid, band);
  stamp();
  __syncthreads();   // every partial has read a before dZ replaces it
  stamp();
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int k = 8 * (g + 16 * c);
    bf16x8* pz = reinterpret_cast<bf16x8*>(z + rb_off(r, k));
    const bf16x8 v = *pz;
    const f32x4 w0 = *reinterpret_cast<const f32x4*>(q.wh + k);
    const f32x4 w1 = *reinterpret_cast<const f32x4*>(q.wh + k + 4);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = (bf16)(dl * w0[e] * act_bwd_t<ACT>((float)v[e]));
      o[4 + e] = (bf16)(dl * w1[e] * act_bwd_t<ACT>((float)v[4 + e]));
    }
    *pz = o;
  }
}

// Diagnostic phase stamps (ST, rowband_stamps != null; scripts/r5_rb_stamps.py): lane 0 of every
// wave records the shader-clock counter (s_memtime) at each phase boundary into an LDS table after
// the parameter block, copied to stamps[band][wave][RB_NST] at exit (slot RB_NST - 2 / - 1: the
// 100 MHz real-time counter at entry / exit, wave 0).  Never instantiated on the training path.
constexpr int RB_NST = 48;

template <int H, int ACT, int D, bool ST = false>
__global__ void __launch_bounds__(RB_THREADS) rowband2_kernel(RowbandArgs p) {
  using G = Rb2Geom<H>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  unsigned long long* stl = nullptr;
  int si = 0;
  if constexpr (ST) {
    stl = reinterpret_cast<unsigned long long*>(smem + rb2_smem_core(H, p.in, p.nh)) + w * RB_NST;
    if (lane == 0 && w == 0) {
      stl[RB_NST - 2] = __builtin_amdgcn_s_memrealtime();
      stl[RB_NST - 4] = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC id
      stl[RB_NST - 3] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW id
    }
  }
  auto stamp = [&]() {
    if constexpr (ST) {
      if (lane == 0 && si < RB_NST - 4) stl[si] = __builtin_amdgcn_s_memtime();
      ++si;
    }
  };
  stamp();
  const int blk = blockIdx.x;
  // band_map 1: the 32 blocks an XCD runs hold contiguous rows, so the row-split weight
  // gradients that read them next (wgrad_multi: split s's blocks sit on the XCDs that wrote its
  // rows) can find them in that XCD's L2.  Per-band partials stay indexed by band: the combine
  // order, and so every result bit, does not depend on the map.
  const int band = p.band_map ? xcd_remap(blk, gridDim.x) : blk;
  const int row0 = band * RB_ROWS;
  const int nvalid = min(RB_ROWS, p.rows - row0);
  const int nh = p.nh, IN = p.in;
  // column group of this wave, rotated per block so the 32 blocks of an XCD do not all fetch
  // the same weight lines at the same moment
  const int cg = (w + blk) & (RB_WAVES - 1);
  const int n0 = cg * G::WCOLS;
  const int SL = RB_ROWS * max(H, IN) * 2;
  const int nslot = max(nh, 2);
  auto slot = [&](int i) { return smem + i * SL; };
  const Rb2Par q = rb2_par(smem + nslot * SL, H, nh);
  // the next weight-gradient launch's fixup counters (wgrad_multi_fix) start from zero
  if (blk == 0 && p.zero_words)
    for (int i = tid; i < p.n_zero; i += RB_THREADS) p.zero_words[i] = 0;

  // Startup: the small operands (every bias, the head weight, the band's targets, the head
  // bias) and the band's input rows, THEN the ring's first D k-steps -- all counted asm loads,
  // so ONE vmcnt(D * NF) retires the operands while the whole ring stays in flight across the
  // barrier.  (With compiler-issued operand loads behind the ring, hipcc's own vmcnt(0) before
  // their use drained the ring: half of layer 0's weights fetched before the first MFMA, a
  // 4.7 us startup -- profiles/r5_rowband_stamps.txt.)
  bf16x8 ring[D][G::NF];
  Rb2Mat cur = rb2_mat<H>(p, 0, cg * G::NJ);
  {
    constexpr int MAXIT = 1024 * RB_ROWS / 8 / RB_THREADS;   // 8: input width <= 1024
    // (thread t < H / 4 loads float4 t of every layer's bias and of the head weight; the
    // layer index is unrolled so each bias pointer is a kernel argument)
    f32x4 bq[RB_MAXL], wq;
    float yq, bhq;
    bf16x8 xv[MAXIT];
    // (only the lanes that own an operand load it: every lane's 16 bytes pass the CU's address
    // unit, which also feeds the weight stream -- 64 B/clk)
    if (tid < H / 4) {
#pragma unroll
      for (int l = 0; l < RB_MAXL; ++l)
        if (l < nh)
          asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(bq[l]) : "v"(tid * 16), "s"(p.b[l]));
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(wq) : "v"(tid * 16), "s"(p.wh));
    }
    if (tid < RB_ROWS)
      asm volatile("global_load_dword %0, %1, %2" : "=v"(yq) : "v"(min(tid, nvalid - 1) * 4), "s"(p.y + row0));
    if (tid == 0) asm volatile("global_load_dword %0, %1, %2" : "=v"(bhq) : "v"(0), "s"(p.bh));
    // the band's rows (past the last valid row that row again -- padding rows are zeroed below)
    const int nit = IN * RB_ROWS / 8 / RB_THREADS;
    const bf16* xb = p.X + (long long)row0 * p.ldx;
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      if (it < nit) {
        const int id = tid + it * RB_THREADS;
        const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(xv[it])
                     : "v"((min(r, nvalid - 1) * p.ldx + kb * 64 + k8 * 8) * 2), "s"(xb));
      }
    }
    stamp();
#pragma unroll
    for (int d = 0; d < D; ++d) rb2_issue<G::NJ>(ring[d], cur.b, cur.ts, d, lane * 16);
    stamp();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * G::NF));
    stamp();
#pragma unroll
    for (int l = 0; l < RB_MAXL; ++l) asm volatile("" : "+v"(bq[l]));
    asm volatile("" : "+v"(wq), "+v"(yq), "+v"(bhq));
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) asm volatile("" : "+v"(xv[it]));
    char* img = slot(0);
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      if (it < nit) {
        const int id = tid + it * RB_THREADS;
        const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
        bf16x8 x = xv[it];
        if (r >= nvalid) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = (bf16)0.f;
        }
        *reinterpret_cast<bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8)) = x;
      }
    }
    if (tid < H / 4) {
#pragma unroll
      for (int l = 0; l < RB_MAXL; ++l)
        if (l < nh) reinterpret_cast<f32x4*>(q.bias)[l * (H / 4) + tid] = bq[l];
      reinterpret_cast<f32x4*>(q.wh)[tid] = wq;
    }
    if (tid < RB_ROWS) q.y[tid] = yq;
    if (tid == 0) q.bh[0] = bhq;
    stamp();
  }
  __syncthreads();
  stamp();

  // Copy-outs run one phase late: a phase's output image is complete at its closing barrier,
  // and the NEXT phase's waves copy it out between their epilogue and their own barrier -- the
  // time a wave that finished its main loop early would otherwise wait there (the waves of a
  // block end a main loop up to ~1.7 us apart: profiles/r5_rowband_stamps.txt).  No phase
  // overwrites an image before its copy-out: dZ_{l-1} replaces a_{l-1} one phase after a_{l-1}
  // was copied, and the head's dZ replaces a_{nh-1} behind the head's own flush.
  const char* pend_src = nullptr;
  bf16* pend_dst = nullptr;
  auto flush = [&]() {
    if (pend_src) rb_copy_out<H>(pend_src, pend_dst, H, nvalid, tid, p.out_pol);
    pend_src = nullptr;
  };

  f32x4 acc[2][G::NJ];
  // ---- forward: a_l = act(a_{l-1} W_l^T + b_l) ----
  for (int l = 0; l < nh; ++l) {
    const Rb2Mat nxt = rb2_mat<H>(p, l + 1, cg * G::NJ);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* in = slot(l == 0 ? 0 : l);
    char* out = l < nh - 1 ? slot(l + 1) : slot(nh >= 2 ? 0 : 1);
    rb2_mainloop<G::NJ, D>(ring, acc, in, cur, nxt, lane);
    stamp();
    // lane holds out[16i + (lane & 15)][n0 + 16j + 4(lane >> 4) .. +3]
    const float* bl = q.bias + l * H + n0 + 4 * (lane >> 4);
    f32x4 bv[G::NJ];   // (all bias reads issued together: one LDS round trip, not NJ)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) bv[j] = *reinterpret_cast<const f32x4*>(bl + 16 * j);
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = acc[i][j] + bv[j];
        f32x4 a;
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = act_fwd_t<ACT>(v[r]);
        *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) =
            __builtin_convertvector(a, bf16x4);
      }
    }
    stamp();
    flush();
    stamp();
    __syncthreads();
    stamp();
    // (a null p.a[l] -- the last hidden layer's activations, which no weight gradient reads --
    // skips the copy-out)
    pend_src = p.a[l] ? out : nullptr;
    pend_dst = p.a[l] ? p.a[l] + (long long)row0 * H : nullptr;
    cur = nxt;
  }
  // ---- head (in place on a_{nh-1}) ----
  char* z = slot(nh >= 2 ? 0 : 1);
  rb2_head<H, ACT>(p, z, q, nvalid, tid, band, stamp, flush);
  stamp();
  __syncthreads();
  stamp();
  pend_src = z;
  pend_dst = p.dz[nh - 1] + (long long)row0 * H;
  // ---- activation gradients: dZ_{l-1} = (dZ_l W_l) * act'(a_{l-1}), in place over a_{l-1} ----
  for (int l = nh - 1; l >= 1; --l) {
    const Rb2Mat nxt = rb2_mat<H>(p, 2 * nh - l, cg * G::NJ);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    char* out = slot(l);   // holds a_{l-1}
    rb2_mainloop<G::NJ, D>(ring, acc, z, cur, nxt, lane);
    stamp();
    // (every a_{l-1} read issued before the first dZ store: one LDS round trip, not 2 x NJ
    // read-after-write-ordered ones)
    bf16x4 ax[2][G::NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j)
        ax[i][j] = *reinterpret_cast<const bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4)));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) {
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] * act_bwd_t<ACT>((float)ax[i][j][r]);
        *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) =
            __builtin_convertvector(o, bf16x4);
      }
    stamp();
    flush();
    stamp();
    __syncthreads();
    stamp();
    pend_src = out;
    pend_dst = p.dz[l - 1] + (long long)row0 * H;
    z = out;
    cur = nxt;
  }
  flush();
  stamp();
  if constexpr (ST) {
    if (lane == 0 && w == 0) stl[RB_NST - 1] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    const unsigned long long* all = stl - w * RB_NST;
    for (int i = tid; i < RB_WAVES * RB_NST; i += RB_THREADS)
      p.stamps[(long long)band * RB_WAVES * RB_NST + i] = all[i];
  }
}

static int rb2_smem(int H, int in, int nh, bool st = false) {
  return rb2_smem_core(H, in, nh) + (st ? RB_WAVES * RB_NST * 8 : 0);
}

static bool rowband2_shape_ok(int H, int in, int nh) {
  // (the instantiated widths: rowband_fwd_bwd)
  if (H != 256 && H != 384 && H != 512 && H != 768 && H != 1024) return false;
  const int D = rb2_depth_rt(H);
  if (in % 64 || in < 64 || (in / 64) % D || (H / 64) % D) return false;
  return rb2_smem(H, in, nh) <= 160 * 1024;
}

static int rb_env(const char* name, int dflt) {
  const char* e = knob_env(name);
  return (e && e[0] >= '0' && e[0] <= '9') ? std::atoi(e) : dflt;
}

template <int H>
static hipError_t rowband2_launch(const RowbandArgs& p, hipStream_t s) {
  using Fn = void (*)(RowbandArgs);
  constexpr int D = rb2_depth<H>();
  static const Fn fns[3] = {rowband2_kernel<H, ACT_NONE, D>, rowband2_kernel<H, ACT_RELU, D>,
                            rowband2_kernel<H, ACT_TANH, D>};
  static bool attr = false;
  if (!attr) {
    for (Fn f : fns)
      (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const Fn f = fns[p.act == ACT_RELU ? 1 : p.act == ACT_TANH ? 2 : 0];
  if (p.stamps) {
    // diagnostic phase stamps: H = 512, relu only (experiments library)
    if constexpr (H == 512 && NNMPI_EXPERIMENTS_BUILD) {
      if (p.act != ACT_RELU || rb2_smem(H, p.in, p.nh, true) > 160 * 1024) return hipErrorInvalidValue;
      static bool sattr = false;
      if (!sattr) {
        (void)hipFuncSetAttribute((const void*)rowband2_kernel<H, ACT_RELU, D, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        sattr = true;
      }
      hipLaunchKernelGGL((rowband2_kernel<H, ACT_RELU, D, true>), dim3(rowband_blocks(p.rows)),
                         dim3(RB_THREADS), rb2_smem(H, p.in, p.nh, true), s, p);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(f, dim3(rowband_blocks(p.rows)), dim3(RB_THREADS), rb2_smem(H, p.in, p.nh), s, p);
  return hipGetLastError();
}

// =============================================================================================
// Column-split row-band kernel: small batches (strong-scaling shards, 64 .. 4,096 rows of the
// 512-wide proxy).  The band kernel above streams every weight byte through every band's CU --
// 2.5 MiB per step and CU, ~4 us per matrix at the address unit's 64 B/clk -- whatever the
// number of bands, so at 1,024 rows (32 bands on 32 CUs) it costs what it costs at 8,192.  Here
// the C blocks of a band (C = 8 / 4 / 2 at <= 32 / 64 / 128 bands: <= 256 blocks, one per CU)
// each own H / C output columns of every layer and stream only those weights (C x fewer bytes
// per CU), and the band's activations are exchanged between them once per layer:
//  * forward layer l < nh-1: the block's 32 x H/C slice of a_l goes to p.a[l] (row-major, the
//    buffer the weight gradients read anyway) with write-through (sc1) stores; every block of the
//    band counts in; each block then loads the whole band of a_l back (sc1 loads) into its LDS
//    image -- the next layer's A operand;
//  * the head: each block's partial logit dot over its own columns is exchanged (C x 32 floats)
//    and summed in block order by every block (the same bits everywhere); dZ_{nh-1}, the head's
//    weight-gradient partials and the bias / loss partials need only the block's own columns;
//  * activation gradient l: the block's slice of dZ_{l-1} = (dZ_l W_l)[:, own] * act'(a_{l-1})
//    goes to p.dz[l-1] and is exchanged like a_l (dZ_0 is not exchanged).
// 2 nh - 1 hand-offs per step.  Each hand-off follows MI355X_MICROARCH.md "Valid forms" row 1:
// the handed-off bytes stored write-through (sc1) -- or plain where every block of the band
// reported the same XCC id in the first hand-off's counter (the consumers' sc1 loads then read
// that XCD's L2) -- every storing wave drains vmcnt before the workgroup barrier, one lane's
// agent-scope atomic add on the band's phase counter; one lane polls it with sc1 loads (bounded:
// past RBS_TIMEOUT it records the timeout in the sticky error word xsync[0] and goes on -- no
// block ever waits without bound), the block joins it at a barrier, every load of the handed-off
// bytes is an sc1 load.  The last block of a band to finish resets the band's counters
// (graph-replayable).  Grid <= 256 blocks of 256 / 512 threads (host: <= blocks per CU x CUs at
// the kernel's occupancy); the C blocks of a band share blockIdx.x % 8 (one XCD under round-robin
// dispatch).  (Computing the whole head in every block from a gathered a_{nh-1} -- one hand-off
// fewer -- measured no faster: profiles/r6_split_head_handoff_ab.txt.)  The weight stream and its
// D-deep register ring are the band kernel's (rb2_mainloop), for NJ 16-column tiles per wave.
// (Reference: dataParallelTraining_NN_MPI.py:99-146 -- the fixed dataset split over P ranks, so
// a rank's step shrinks as P grows.)
// =============================================================================================
constexpr int RBS_SYNC = 32;                // ints per band: phase counters [0, 2nh-1), done [31]
constexpr int RBS_NST = 48;                 // diagnostic stamps per block
constexpr int RBS_MAXB = 128;               // bands (4,096 rows)
constexpr int RBS_XS = 32 + RBS_MAXB * RBS_SYNC;   // sync words at the start of the workspace
constexpr long long RBS_TIMEOUT = 200000;   // 100 MHz ticks (2 ms) before a wait gives up

static int g_rbs_groups = -1;   // NNMPI_RB_SPLIT: 0 off, 2 / 4 / 8 force C, else automatic
static int rbs_groups(int rows) {
  if (g_rbs_groups < 0) {
    const char* e = knob_env("NNMPI_RB_SPLIT");
    g_rbs_groups = (e && e[0] >= '0' && e[0] <= '9') ? std::atoi(e) : 1;
  }
  const int nb = (rows + RB_ROWS - 1) / RB_ROWS;
  if (g_rbs_groups == 0 || nb > RBS_MAXB) return 0;
  if (g_rbs_groups == 2 || g_rbs_groups == 4 || g_rbs_groups == 8)
    return nb * g_rbs_groups <= 256 ? g_rbs_groups : 0;
  for (int c = 8; c >= 2; c >>= 1)
    if (nb * c <= 256) return c;
  return 0;
}
void set_rb_split(int v) { g_rbs_groups = v; }

__host__ __device__ __forceinline__ int rbs_smem(int in, int nh) {
  // the band kernel's activation slots + parameter block, then the head's column-partial scratch
  return rb2_smem_core(512, in, nh) + 512 * 4 + RBS_NST * 8;
}

template <int NJ, int NW, int ACT, bool ST = false>
__global__ void __launch_bounds__(64 * NW) rowband_split_kernel(RowbandArgs p) {
  // (ring depth: 4 k-steps, 2 at NJ = 4 -- the 4-deep ring, the accumulators and tanh's
  // temporaries overflow the 256 VGPRs there and the compiler parks values in AGPRs, including
  // asm-loaded ring registers before their loads land)
  // (an 8-deep ring at one tile per wave -- a block's whole slice of the next matrix in flight
  // during a hand-off -- measured no faster: the ~1 us main loop is the MFMA / LDS dependency
  // chain of 4 MFMAs per k-step, not the weight fetch; profiles/r5_split_stamps.txt)
  constexpr int H = 512, D = NJ >= 4 ? 2 : 4, NF = 2 * NJ, NT = 64 * NW;
  constexpr int NC = 16 * NJ * NW;  // this block's output columns (NW waves x NJ tiles of 16)
  constexpr int C = H / NC;         // blocks per band
  constexpr int TPC = NT / NC;      // head partials: threads per column
  constexpr int TPR = NT / RB_ROWS; // head logits / dZ: threads per row
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Block -> (band, column group).  XCD-grouped map (p.rbs_map): blocks are dealt round-robin
  // over the 8 XCDs (b and b + 8 share one -- observed placement, speed only), so the C blocks of
  // a band are C consecutive ids among those with the same b % 8 and its hand-offs can stay in
  // one L2; the grid is padded to a multiple of 8 bands (padding bands exit at once).  Else the
  // C blocks of a band are consecutive ids (one per XCD at C = 8).
  int band, c;
  if (p.rbs_map) {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
    band = (j / C) * 8 + x;
    c = j % C;
  } else {
    band = blockIdx.x / C;
    c = blockIdx.x % C;
  }
  const int row0 = band * RB_ROWS, nvalid = max(0, min(RB_ROWS, p.rows - row0));
  const int nh = p.nh, IN = p.in;
  const int c0 = c * NC;                  // the block's first column
  const int n0 = c0 + w * 16 * NJ;        // the wave's first column
  constexpr int SL = RB_ROWS * H * 2;     // (IN <= H)
  auto slot = [&](int i) { return smem + i * SL; };
  const int nslot = max(nh, 2);
  const Rb2Par q = rb2_par(smem + nslot * SL, H, nh);
  float* red = reinterpret_cast<float*>(smem + rb2_smem_core(H, IN, nh));   // [TPC][NC]
  // diagnostic phase stamps (ST: wave 0's shader clock at every phase boundary, LDS table after
  // the head scratch, copied to p.stamps[block][RBS_NST] at exit; scripts/r5_split_stamps.py)
  unsigned long long* stl = reinterpret_cast<unsigned long long*>(smem + rb2_smem_core(H, IN, nh) + 512 * 4);
  int si = 0;
  auto stamp = [&]() {
    if constexpr (ST) {
      if (tid == 0 && si < RBS_NST) stl[si] = __builtin_amdgcn_s_memtime();
      ++si;
    }
  };
  stamp();
  int* err = p.xsync;
  int* sy = p.xsync + 32 + band * RBS_SYNC;
  if (blockIdx.x == 0 && p.zero_words)
    for (int i = tid; i < p.n_zero; i += NT) p.zero_words[i] = 0;
  if (band >= p.rbs_bands) return;   // a padding band of the XCD-grouped map: no block of it works
  // The first hand-off's counter (phase 0) also says where the band runs: each block adds
  // 1 << 4 * (its XCC id), so the word holds per-XCC arrival counts (C <= 8 < 16 per nibble).
  // When every block of the band sits on one XCC, the later hand-offs store PLAIN (the bytes stay
  // in that XCD's L2, which the consumers' sc1 loads read) instead of write-through -- decided
  // from the hardware's XCC ids, not from the dispatch order the band map hopes for; a band that
  // spans XCCs keeps the write-through form.
  const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 7;   // HW_REG_XCC_ID
  bool local = false;   // (uniform in the block: set after phase 0 from the counter's final value)

  // ---- hand-off primitives ----
  auto arrive = [&](int ph) {   // after this block's stores of phase ph
    stamp();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_add(sy + ph, ph == 0 ? 1 << (4 * xcc) : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp();
  };
  int* lflag = reinterpret_cast<int*>(red);   // (LDS word: phase 0's placement verdict)
  auto arrivals = [&](int ph, int v) {
    if (ph != 0) return v;
    int n = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) n += (v >> (4 * x)) & 15;
    return n;
  };
  auto wait = [&](int ph) {
    if (tid == 0) {
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      int v;
      while (arrivals(ph, v = ld_sc1_i(sy + ph)) < C) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > RBS_TIMEOUT) {
          __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = 0;   // (a timed-out band keeps the write-through form)
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // every block of the band counted on ONE XCC: exactly one nonzero nibble
      if (ph == 0) {
        int nz = 0;
#pragma unroll
        for (int x = 0; x < 8; ++x) nz += ((v >> (4 * x)) & 15) != 0;
        lflag[0] = p.rbs_local && nz == 1;
      }
    }
    __syncthreads();
    if (ph == 0) {
      local = lflag[0] != 0;
      __syncthreads();   // (the word is the head scratch later)
    }
    stamp();
  };
  // a 16-byte piece of a handed-off matrix: plain when the band is on one XCC, else write-through
  auto st16 = [&](bf16* dst, bf16x8 v) {
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    const u32x4 d = __builtin_bit_cast(u32x4, v);
    if (local)
      asm volatile("global_store_dwordx4 %0, %1, off\n s_nop 1" ::"v"(dst), "v"(d) : "memory");
    else
      asm volatile("global_store_dwordx4 %0, %1, off sc1\n s_nop 1" ::"v"(dst), "v"(d) : "memory");
  };
  // K-major operand fragments for the small-batch weight gradients (p.kbands, wgrad_small's
  // image path): fragment (g, band) of a [rows][*] matrix from its LDS image -- lane i holds rows
  // 8 (i >> 4) .. + 7 of column 16 g + (i & 15), zero past the batch -- one 16-byte store
  auto kfrag = [&](const char* img, bf16* dst, int g) {
    const int k = 16 * g + (lane & 15), r0 = 8 * (lane >> 4);
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      v[e] = r0 + e < nvalid ? *reinterpret_cast<const bf16*>(img + rb_off(r0 + e, k)) : (bf16)0.f;
    *reinterpret_cast<bf16x8*>(dst + ((long long)g * p.kbands + band) * 512 + lane * 8) = v;
  };
  // ... of the wave's own column groups of an H-wide matrix (NJ stores)
  auto kown = [&](const char* img, bf16* dst) {
    if (!dst) return;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < NJ; ++j) kfrag(img, dst, n0 / 16 + j);
  };
  // the whole band of a handed-off [rows][H] matrix into an LDS image (padding rows zero).  With
  // kdst, the own fragments of the matrix the image holds now (the band's own columns are the same
  // bits in both) are written while the loads fly: their NJ stores, the youngest, stay out of the
  // loads' wait -- issued before the loads, the wait would hold for their write acknowledgements
  auto gather = [&](const bf16* src, char* img, bf16* kdst) {
    constexpr int IT = RB_ROWS * H / 8 / NT;
    bf16x8 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int id = tid + it * NT;
      const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
      v[it] = ld_sc1_b16(src + (long long)(row0 + min(r, nvalid - 1)) * H + kb * 64 + k8 * 8);
    }
    if (kdst) {
      kown(img, kdst);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NJ) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      asm volatile("" : "+v"(v[it]));
      const int id = tid + it * NT;
      const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
      bf16x8 x = v[it];
      if (r >= nvalid) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = (bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8)) = x;
    }
    __syncthreads();
    stamp();
  };
  // the wave's own 32 x 16NJ tile of an LDS image -> dst rows (sc1, 16-byte pieces; the wave
  // reads back its own LDS writes: no barrier)
  auto put = [&](const char* img, bf16* dst) {
    // (a compiler fence: the bf16x8 reads below alias the epilogue's bf16x4 LDS writes)
    asm volatile("" ::: "memory");
    const int r = lane >> 1;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) {
      const int k = n0 + 8 * ((lane & 1) + 2 * jj);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + rb_off(r, k));
      if (r < nvalid) st16(dst + (long long)(row0 + r) * H + k, v);
    }
  };

  // ---- startup: operands, the band's input rows, the ring's first D k-steps (band kernel) ----
  bf16x8 ring[D][NF];
  Rb2Mat cur = rb2_mat<H>(p, 0, n0 / 16);
  {
    constexpr int MAXIT = H * RB_ROWS / 8 / NT;
    f32x4 bq[RB_MAXL], wq;
    float yq, bhq;
    bf16x8 xv[MAXIT];
    if (tid < H / 4) {
#pragma unroll
      for (int l = 0; l < RB_MAXL; ++l)
        if (l < nh)
          asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(bq[l]) : "v"(tid * 16), "s"(p.b[l]));
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(wq) : "v"(tid * 16), "s"(p.wh));
    }
    if (tid < RB_ROWS)
      asm volatile("global_load_dword %0, %1, %2" : "=v"(yq) : "v"(min(tid, nvalid - 1) * 4), "s"(p.y + row0));
    if (tid == 0) asm volatile("global_load_dword %0, %1, %2" : "=v"(bhq) : "v"(0), "s"(p.bh));
    const int nit = IN * RB_ROWS / 8 / NT;
    const bf16* xb = p.X + (long long)row0 * p.ldx;
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      if (it < nit) {
        const int id = tid + it * NT;
        const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(xv[it])
                     : "v"((min(r, nvalid - 1) * p.ldx + kb * 64 + k8 * 8) * 2), "s"(xb));
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) rb2_issue<NJ>(ring[d], cur.b, cur.ts, d, lane * 16);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * NF));
#pragma unroll
    for (int l = 0; l < RB_MAXL; ++l) asm volatile("" : "+v"(bq[l]));
    asm volatile("" : "+v"(wq), "+v"(yq), "+v"(bhq));
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) asm volatile("" : "+v"(xv[it]));
    char* img = slot(0);
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      if (it < nit) {
        const int id = tid + it * NT;
        const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
        bf16x8 x = xv[it];
        if (r >= nvalid) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = (bf16)0.f;
        }
        *reinterpret_cast<bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8)) = x;
      }
    }
    if (tid < H / 4) {
#pragma unroll
      for (int l = 0; l < RB_MAXL; ++l)
        if (l < nh) reinterpret_cast<f32x4*>(q.bias)[l * (H / 4) + tid] = bq[l];
      reinterpret_cast<f32x4*>(q.wh)[tid] = wq;
    }
    if (tid < RB_ROWS) q.y[tid] = yq;
    if (tid == 0) q.bh[0] = bhq;
  }
  __syncthreads();
  stamp();
  // the input's fragments (the block's share of its column groups), from slot 0: at the first
  // hand-off (stores issued here would hold up the first main loop's counted ring waits), or
  // after the forward pass when there is none (nh == 1: slot 0 keeps the input)
  auto kinput = [&]() {
    if (!p.ka[0]) return;
    const int gpb = IN / 16 / C;
    for (int gi = w; gi < gpb; gi += NW) kfrag(slot(0), p.ka[0], c * gpb + gi);
  };

  f32x4 acc[2][NJ];
  // ---- forward: slot(l + 1) receives the whole band of a_l; the last layer's own columns go
  // to slot 0 (the input rows' slot: free by then) ----
  for (int l = 0; l < nh; ++l) {
    const Rb2Mat nxt = rb2_mat<H>(p, l + 1, n0 / 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool last = l == nh - 1;
    char* out = !last ? slot(l + 1) : slot(nh >= 2 ? 0 : 1);
    rb2_mainloop<NJ, D>(ring, acc, slot(l), cur, nxt, lane);
    stamp();
    const float* bl = q.bias + l * H + n0 + 4 * (lane >> 4);
    f32x4 bv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bv[j] = *reinterpret_cast<const f32x4*>(bl + 16 * j);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = acc[i][j] + bv[j];
        f32x4 a;
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = act_fwd_t<ACT>(v[r]);
        *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) =
            __builtin_convertvector(a, bf16x4);
      }
    if (p.a[l]) put(out, p.a[l]);
    cur = nxt;
    if (!last) {
      arrive(l);
      if (l == 0) kinput();
      wait(l);
      gather(p.a[l], out, p.ka[l + 1]);
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (nh == 1) kinput();
    }
  }
  // ---- head: partial logits over the own columns, exchanged and summed in block order ----
  char* z = slot(nh >= 2 ? 0 : 1);
  {
    const int r = tid / TPR, g = tid % TPR;
    float dot = 0.f;
#pragma unroll
    for (int cc = 0; cc < NC / (8 * TPR); ++cc) {
      const int k = c0 + 8 * (g + TPR * cc);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(z + rb_off(r, k));
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(q.wh + k);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(q.wh + k + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) dot += (float)v[e] * w0[e];
#pragma unroll
      for (int e = 0; e < 4; ++e) dot += (float)v[4 + e] * w1[e];
    }
#pragma unroll
    for (int sh = TPR / 2; sh >= 1; sh >>= 1) dot += __shfl_xor(dot, sh, 64);
    if (g == 0) {
      float* hp = p.hx + ((long long)band * C + c) * RB_ROWS + r;
      if (local) *hp = dot;
      else st_sc1_f(hp, dot);
    }
  }
  arrive(nh - 1);
  wait(nh - 1);
  if (tid < RB_ROWS) {
    float part[C];
#pragma unroll
    for (int cb = 0; cb < C; ++cb) part[cb] = ld_sc1_f(p.hx + ((long long)band * C + cb) * RB_ROWS + tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float dot = 0.f;
#pragma unroll
    for (int cb = 0; cb < C; ++cb) {
      asm volatile("" : "+v"(part[cb]));
      dot += part[cb];
    }
    const bool valid = tid < nvalid;
    const float d = dot + q.bh[0] - q.y[tid];
    q.dls[tid] = valid ? 2.f * d * p.inv_count : 0.f;
    q.lss[tid] = valid ? d * d : 0.f;
  }
  __syncthreads();
  // the band's head-gradient partials of the own columns (rows split over TPC threads, summed
  // in order), the bias / loss partials by block 0 of the band
  {
    const int col = tid % NC, part = tid / NC, k = c0 + col;
    constexpr int RPT = RB_ROWS / TPC;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = part * RPT + i;
      s = fmaf(q.dls[r], (float)*reinterpret_cast<const bf16*>(z + rb_off(r, k)), s);
    }
    red[part * NC + col] = s;
    __syncthreads();
    if (tid < NC) {
      float t = red[tid];
#pragma unroll
      for (int pp = 1; pp < TPC; ++pp) t += red[pp * NC + tid];
      p.wslab[(long long)band * H + c0 + tid] = t;
    }
    if (c == 0 && tid >= 64 && tid < 128) {
      const int lt = tid - 64;
      float b = lt < RB_ROWS ? q.dls[lt] : 0.f, ls = lt < RB_ROWS ? q.lss[lt] : 0.f;
#pragma unroll
      for (int sh = 16; sh >= 1; sh >>= 1) {
        b += __shfl_xor(b, sh, 64);
        ls += __shfl_xor(ls, sh, 64);
      }
      if (lt == 0) {
        p.bslab[band] = b;
        p.loss_part[band] = ls;
      }
    }
  }
  // dZ_{nh-1} of the own columns = dl * w * act'(a), in place (the image fragments) and to
  // p.dz[nh-1]
  {
    const int r = tid / TPR, g = tid % TPR;
    const float dl = q.dls[r];
#pragma unroll
    for (int cc = 0; cc < NC / (8 * TPR); ++cc) {
      const int k = c0 + 8 * (g + TPR * cc);
      bf16x8* pz = reinterpret_cast<bf16x8*>(z + rb_off(r, k));
      const bf16x8 v = *pz;
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(q.wh + k);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(q.wh + k + 4);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = (bf16)(dl * w0[e] * act_bwd_t<ACT>((float)v[e]));
        o[4 + e] = (bf16)(dl * w1[e] * act_bwd_t<ACT>((float)v[4 + e]));
      }
      if (r < nvalid) st16(p.dz[nh - 1] + (long long)(row0 + r) * H + k, o);
      if (p.kz[nh - 1]) *pz = o;
    }
  }
  if (nh >= 2) {
    arrive(nh);
    wait(nh);
    gather(p.dz[nh - 1], z, p.kz[nh - 1]);
  } else if (p.kz[0]) {
    __syncthreads();
    kown(z, p.kz[0]);
  }
  // ---- activation gradients: the own columns of dZ_{l-1}, over a_{l-1} in slot(l) ----
  for (int l = nh - 1; l >= 1; --l) {
    const Rb2Mat nxt = rb2_mat<H>(p, 2 * nh - l, n0 / 16);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    char* out = slot(l);
    rb2_mainloop<NJ, D>(ring, acc, z, cur, nxt, lane);
    stamp();
    bf16x4 ax[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        ax[i][j] = *reinterpret_cast<const bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4)));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        f32x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] * act_bwd_t<ACT>((float)ax[i][j][r]);
        *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) =
            __builtin_convertvector(o, bf16x4);
      }
    put(out, p.dz[l - 1]);
    cur = nxt;
    if (l >= 2) {
      const int ph = 2 * nh - l;
      arrive(ph);
      wait(ph);
      gather(p.dz[l - 1], out, p.kz[l - 1]);
    } else {
      kown(out, p.kz[0]);
    }
    z = out;
  }
  // ---- the last block of the band to get here resets the band's counters ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0 &&
      __hip_atomic_fetch_add(sy + RBS_SYNC - 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == C - 1) {
    for (int i = 0; i < 2 * nh - 1; ++i) __hip_atomic_store(sy + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sy + RBS_SYNC - 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (ST) {
    stamp();
    __syncthreads();
    for (int i = tid; i < RBS_NST; i += NT) p.stamps[(long long)blockIdx.x * RBS_NST + i] = stl[i];
  }
}

template <int NJ, int NW>
static hipError_t rbs_launch(const RowbandArgs& p, hipStream_t s);
template <int NJ, int NW>
static int rbs_occupancy(int smem);
static int rbs_waves();
static int rbs_map();

// The split kernel's blocks of a band wait for each other, so the grid must fit the chip at the
// kernel's occupancy (all blocks resident at once when nothing else holds CUs; with CUs held by
// another stream a band still completes once resident bands exit -- the bounded wait covers the
// rest).  The occupancy query is made once per (form, LDS size).
static bool rbs_fits(int rows, int in, int nh) {
  const int C = rbs_groups(rows);
  if (C <= 0) return false;
  const int smem = rbs_smem(in, nh);
  int per_cu = 0;
  switch (C) {
    case 8: per_cu = rbs_occupancy<1, 4>(smem); break;
    case 4: per_cu = rbs_waves() == 8 ? rbs_occupancy<1, 8>(smem) : rbs_occupancy<2, 4>(smem); break;
    case 2: per_cu = rbs_waves() == 8 ? rbs_occupancy<2, 8>(smem) : rbs_occupancy<4, 4>(smem); break;
    default: return false;
  }
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = -1;
  }
  if (cus < 0) return true;   // no device (a CPU process): the shape predicate alone
  const int nb = rowband_blocks(rows);
  const long long grid = (long long)(rbs_map() ? (nb + 7) / 8 * 8 : nb) * C;
  return per_cu > 0 && grid <= (long long)per_cu * cus;
}

bool rowband_split_ok(int rows, int H, int in, int nh, int act) {
  const int c = rbs_groups(rows);
  (void)act;   // every activation (relu / tanh / none) has a form
  return rows > 0 && H == 512 && in >= 256 && in <= H && in % 256 == 0 && nh >= 1 && nh <= RB_MAXL &&
         c > 0 && rbs_smem(in, nh) <= 160 * 1024 && rbs_fits(rows, in, nh);
}

// (NJ x NW: 1 x 4 -> 8 blocks per band, 2 x 4 -> 4, 4 x 4 -> 2)
// waves per block at 4 / 2 blocks per band: 8 (1 / 2 tiles per wave) or 4 (2 / 4 tiles per wave;
// NNMPI_RB_SPLIT_WAVES=4, A/B).  Measured 24.6 vs 25.9 us at 2,048 rows and 32.4 vs 33.9 us at
// 4,096 (profiles/r5_split_waves_ab.txt).
// The XCD-grouped band map (NNMPI_RB_SPLIT_MAP, default 1) and, under it, plain stores for the
// hand-offs of a band found on one XCC (NNMPI_RB_SPLIT_LOCAL, default 1); A/B knobs.
static int rbs_map() {
  static const int v = rb_env("NNMPI_RB_SPLIT_MAP", 1) ? 1 : 0;
  return v;
}
static int rbs_local() {
  static const int v = rb_env("NNMPI_RB_SPLIT_LOCAL", 1) ? 1 : 0;
  return v;
}
static int g_rbs_waves = -1;
static int rbs_waves() {
  if (g_rbs_waves < 0) g_rbs_waves = rb_env("NNMPI_RB_SPLIT_WAVES", 8) == 4 ? 4 : 8;
  return g_rbs_waves;
}
template <int NJ, int NW>
static int rbs_occupancy(int smem) {
  static int cached_smem = -1, cached = 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return 0;
  if (cached_smem != smem) {
    int n = 0;
    // (the attribute must allow the dynamic LDS size before the query can answer for it)
    (void)hipFuncSetAttribute((const void*)rowband_split_kernel<NJ, NW, ACT_RELU>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rowband_split_kernel<NJ, NW, ACT_RELU>, 64 * NW,
                                                     smem) != hipSuccess)
      n = 0;
    cached_smem = smem;
    cached = n;
  }
  return cached;
}
template <int NJ, int NW>
static hipError_t rbs_launch(const RowbandArgs& p, hipStream_t s) {
  using Fn = void (*)(RowbandArgs);
  static const Fn fns[3] = {rowband_split_kernel<NJ, NW, ACT_NONE>, rowband_split_kernel<NJ, NW, ACT_RELU>,
                            rowband_split_kernel<NJ, NW, ACT_TANH>};
  static bool attr = false;
  if (!attr) {
    for (Fn f : fns)
      (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  Fn f = fns[p.act == ACT_RELU ? 1 : p.act == ACT_TANH ? 2 : 0];
  if (p.stamps) {   // diagnostic stamps: relu only (experiments library)
#if NNMPI_EXPERIMENTS_BUILD
    if (p.act != ACT_RELU) return hipErrorInvalidValue;
    f = rowband_split_kernel<NJ, NW, ACT_RELU, true>;
    static bool sattr = false;
    if (!sattr) {
      (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      sattr = true;
    }
#else
    return hipErrorNotSupported;
#endif
  }
  const int C = 512 / (16 * NJ * NW);
  RowbandArgs q = p;
  q.rbs_bands = rowband_blocks(p.rows);
  q.rbs_map = rbs_map();
  q.rbs_local = q.rbs_map && rbs_local();
  const int nbp = q.rbs_map ? (q.rbs_bands + 7) / 8 * 8 : q.rbs_bands;
  hipLaunchKernelGGL(f, dim3(nbp * C), dim3(64 * NW), rbs_smem(p.in, p.nh), s, q);
  return hipGetLastError();
}

// ---- fragment-major weight images (rb_pk_off) of every hidden layer: Pf[l] = W_l ([H][in_l]),
// Pd[l] = W_l^T ([in_l][H], l >= 1), one thread per 16-byte fragment piece ----
struct RbPackJob {
  const bf16* W;     // source [rows][ld] row-major
  bf16* dst;         // fragment-major image of M = W (trans 0) or W^T (trans 1), M is [NR][KC]
  int ld, KC, trans;
  long long start;   // first 16-byte piece of this job in the launch
};
struct RbPackParams {
  RbPackJob job[2 * RB_MAXL];
  int nj;
  long long total;
};

__global__ void __launch_bounds__(256) rb_pack_kernel(RbPackParams g) {
  const long long id = (long long)blockIdx.x * 256 + threadIdx.x;
  if (id >= g.total) return;
  int j = 0;
#pragma unroll 1
  while (j + 1 < g.nj && id >= g.job[j + 1].start) ++j;
  const RbPackJob& jb = g.job[j];
  const long long c = id - jb.start;
  const int lane = (int)(c & 63);
  const long long frag = c >> 6;
  const int KH = jb.KC >> 5;
  const int n = (int)(frag / KH) * 16 + (lane & 15);
  const int k0 = (int)(frag % KH) * 32 + 8 * (lane >> 4);
  bf16x8 v;
  if (!jb.trans) {
    v = *reinterpret_cast<const bf16x8*>(jb.W + (long long)n * jb.ld + k0);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = jb.W[(long long)(k0 + e) * jb.ld + n];
  }
  *reinterpret_cast<bf16x8*>(jb.dst + c * 8) = v;
}

hipError_t rowband_pack(const RowbandArgs& p, hipStream_t s) {
  RbPackParams g{};
  long long n = 0;
  auto add = [&](const bf16* W, const bf16* dst, int ld, int NR, int KC, int trans) {
    if (!dst) return;
    g.job[g.nj] = RbPackJob{W, const_cast<bf16*>(dst), ld, KC, trans, n};
    n += (long long)NR * KC / 8;
    ++g.nj;
  };
  for (int l = 0; l < p.nh; ++l) {
    const int K = l == 0 ? p.in : p.H;
    add(p.W[l], p.Pf[l], K, p.H, K, 0);        // forward: W_l [H][K]
    if (l >= 1) add(p.W[l], p.Pd[l], K, K, p.H, 1);   // dgrad: W_l^T [K][H]
  }
  g.total = n;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(rb_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
  return hipGetLastError();
}

int rowband_blocks(int rows) { return (rows + RB_ROWS - 1) / RB_ROWS; }

bool rowband2_ok(int rows, int H, int in, int nh, int out, int loss, int act) {
  return rows > 0 && nh >= 1 && nh <= RB_MAXL && out == 1 && loss == LOSS_MSE &&
         (act == ACT_RELU || act == ACT_TANH || act == ACT_NONE) && rowband2_shape_ok(H, in, nh);
}

size_t rowband_packed_elems(int H, int in, int nh) {
  // forward images of every layer + dgrad images of layers 1 .. nh-1
  return (size_t)H * in + (size_t)(nh - 1) * H * H * 2;
}


// XCD-contiguous band order of the v2 kernel (RowbandArgs::band_map): NNMPI_RB_BANDMAP=0/1
// (experiments); results are bitwise the same either way.
static int g_rb_band_map = -1;
constexpr int RB_BAND_MAP_DEFAULT = 0;
void set_rb_band_map(int v) { g_rb_band_map = v; }
static int rb_band_map() {
  if (g_rb_band_map < 0) g_rb_band_map = rb_env("NNMPI_RB_BANDMAP", RB_BAND_MAP_DEFAULT) ? 1 : 0;
  return g_rb_band_map;
}

// diagnostic: phase stamps of the v2 kernel into this buffer (rowband_blocks x 8 x RB_NST uint64;
// the stamped kernel twins exist in the experiments library only)
static unsigned long long* g_rb_stamps = nullptr;
#if NNMPI_EXPERIMENTS_BUILD
void set_rowband_stamps(unsigned long long* buf) { g_rb_stamps = buf; }
int rowband_stamp_slots() { return RB_WAVES * RB_NST; }
int rowband_split_stamp_slots() { return RBS_NST; }
#endif

// copy-out store policy (RowbandArgs::out_pol): NNMPI_RB_STORE=0/1/2 (experiments)
static int g_rb_store = -1;
constexpr int RB_STORE_DEFAULT = 0;
void set_rb_store_policy(int pol) { g_rb_store = pol; }
static int rb_store_policy() {
  if (g_rb_store < 0) g_rb_store = rb_env("NNMPI_RB_STORE", RB_STORE_DEFAULT);
  return (g_rb_store >= 0 && g_rb_store <= 2) ? g_rb_store : RB_STORE_DEFAULT;
}

hipError_t rowband_fwd_bwd(const RowbandArgs& p0, hipStream_t s) {
  RowbandArgs p = p0;
  p.band_map = rb_band_map();
  p.out_pol = rb_store_policy();
  p.stamps = g_rb_stamps;
  if (!p.Pf[0] || !rowband2_ok(p.rows, p.H, p.in, p.nh, 1, LOSS_MSE, p.act)) return hipErrorInvalidValue;
  for (int l = 0; l < p.nh; ++l)
    if (!p.Pf[l] || (l >= 1 && !p.Pd[l])) return hipErrorInvalidValue;
  if (p.xsync && p.hx && rowband_split_ok(p.rows, p.H, p.in, p.nh, p.act)) {
    // small batch: the column-split form (its hand-offs go through p.a[l], l < nh - 1)
    for (int l = 0; l + 1 < p.nh; ++l)
      if (!p.a[l]) return hipErrorInvalidValue;
    switch (rbs_groups(p.rows)) {
      case 8: return rbs_launch<1, 4>(p, s);
      case 4: return rbs_waves() == 8 ? rbs_launch<1, 8>(p, s) : rbs_launch<2, 4>(p, s);
      case 2: return rbs_waves() == 8 ? rbs_launch<2, 8>(p, s) : rbs_launch<4, 4>(p, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (p.H) {
    case 256: return rowband2_launch<256>(p, s);
    case 384: return rowband2_launch<384>(p, s);
    case 512: return rowband2_launch<512>(p, s);
    case 768: return rowband2_launch<768>(p, s);
    case 1024: return rowband2_launch<1024>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// ---- the whole step: row-band launch, grouped weight gradients, grouped combines ----------
static size_t rb_pad4(size_t n) { return (n + 3) & ~(size_t)3; }

// weight-gradient slabs per layer: explicit, else NNMPI_RB_SPLITS (A/B), else fill the chip
static int rb_splits(int splits, int nh, int H, int rows) {
  if (splits > 0) return splits;
  static const int env = rb_env("NNMPI_RB_SPLITS", 0);
  return env > 0 ? env : wgrad_multi_splits(nh, H, H, rows);
}

// Split-K slabs of layer l's weight gradient under plan 0 / 1 (RowbandStep::plan).  A layer's
// gradient sums its slabs in a fixed order, so the phases of one plan are bitwise equal to its
// single launch.
static int rb_layer_splits(int plan, int splits, int nh, int H, int rows, int l) {
  if (plan == 0) return rb_splits(splits, nh, H, rows);
  return rb_splits(0, l == nh - 1 ? 1 : std::max(1, nh - 1), H, rows);
}

// slab capacity per layer: the largest count of either plan
static int rb_max_splits(int splits, int nh, int H, int rows) {
  return std::max(rb_splits(splits, nh, H, rows), rb_splits(0, 1, H, rows));
}

// per-tile arrival counters of the in-launch fixup (wgrad_multi_fix), one set per layer, after
// the slabs: zero in a fresh workspace, reset by each tile's last arrival
#if NNMPI_EXPERIMENTS_BUILD
static size_t rb_counters(int H, int in) { return rb_pad4((size_t)wgrad_fix_counters(H, std::max(H, in))); }
#else
static size_t rb_counters(int, int) { return 0; }
#endif

// K-major operand images of the small-batch weight gradients (RowbandArgs::ka / kz): 2 nh of
// them, each up to 128 bands (4,096 rows) x 32 rows x max(H, in) bf16 (floats)
static size_t rb_kimg_floats(int H, int in) { return (size_t)128 * RB_ROWS * std::max(H, in) / 2; }

// Workspace (floats): the column-split kernel's sync words (RBS_XS ints at a fixed place: they
// must read zero between launches whatever the batch size), the head partials, the weight-
// gradient slabs, the fixup counters, the split kernel's head exchange (G x 8 x 32), the K-major
// operand images.
size_t rowband_workspace_bytes(int rows, int H, int in, int nh, int splits) {
  const size_t G = (size_t)rowband_blocks(rows);
  const int S = rb_max_splits(splits, nh, H, rows);
  const size_t head = G * H + rb_pad4(G) + rb_pad4(G);
  return (RBS_XS + head + (size_t)nh * S * ((size_t)H * std::max(H, in) + H) +
          (size_t)nh * rb_counters(H, in) + G * 8 * RB_ROWS + 2 * (size_t)nh * rb_kimg_floats(H, in)) *
         sizeof(float);
}
int rowband_error_word() { return 0; }   // int index into the workspace: a split-kernel wait timed out

// The split-K combine of the row-band weight gradients: as its own launch (slab_multi, default)
// or inside the weight-gradient launch (wgrad_multi_fix, NNMPI_RB_FIXUP=1: the tile's splits
// combine cooperatively once all have arrived).  Bitwise the same results.  Measured on the proxy
// step: 37.4 us for the fused launch vs 25.4 + 9.1 us for the two (profiles/r5_wgrad_fixup_ab.txt)
// -- the combine moves the same slab and optimizer bytes at the same per-CU rate either way, and
// the fused form adds the wait for a tile's last split -- so it stays off.
// (experiments library only)
#if NNMPI_EXPERIMENTS_BUILD
static int g_rb_fixup = -1;
constexpr int RB_FIXUP_DEFAULT = 0;
void set_rb_fixup(int on) { g_rb_fixup = on; }
static bool rb_fixup() {
  if (g_rb_fixup < 0) g_rb_fixup = rb_env("NNMPI_RB_FIXUP", RB_FIXUP_DEFAULT) ? 1 : 0;
  return g_rb_fixup == 1;
}
#else
static constexpr bool rb_fixup() { return false; }
#endif

// Small batches (the column-split kernel's): the weight gradients as 64 x 64 tiles over the whole
// K with the update in their epilogue and the head's combine in the same launch (wgrad_small) --
// NNMPI_RB_WGSMALL=0 keeps the split-K slabs + combine launch (A/B).
static int g_rb_wgsmall = -1;
void set_rb_wgsmall(int v) { g_rb_wgsmall = v; }
static bool rb_wgsmall() {
  if (g_rb_wgsmall < 0) g_rb_wgsmall = rb_env("NNMPI_RB_WGSMALL", 1) ? 1 : 0;
  return g_rb_wgsmall == 1;
}

hipError_t rowband_step(const RowbandStep& st0, hipStream_t s) {
  RowbandStep st = st0;
  RowbandArgs& p = st.fb;
  const bool ok = p.Pf[0] && rowband2_ok(p.rows, p.H, p.in, p.nh, 1, LOSS_MSE, p.act);
  if (!ok || !st.ws || st.phase < 0 || st.phase > 2) return hipErrorInvalidValue;
  const int H = p.H, nh = p.nh;
  const size_t G = (size_t)rowband_blocks(p.rows);
  p.xsync = st.split != 0 ? reinterpret_cast<int*>(st.ws) : nullptr;
  float* ws = st.ws + RBS_XS;
  p.wslab = ws;
  p.bslab = ws + G * H;
  p.loss_part = p.bslab + rb_pad4(G);
  float* slabs = p.loss_part + rb_pad4(G);
  const size_t per = (size_t)rb_max_splits(st.splits, nh, H, p.rows) * ((size_t)H * std::max(H, p.in) + H);
  int* cnt = reinterpret_cast<int*>(slabs + (size_t)nh * per);
  p.hx = reinterpret_cast<float*>(cnt + (size_t)nh * rb_counters(H, p.in));
  if (rb_fixup()) {
    p.zero_words = cnt;
    p.n_zero = nh * (int)rb_counters(H, p.in);
  }
  // the small-batch weight gradients' image path: the split kernel writes the operand images
  // (<= 2,048 rows the LDS-DMA tiles, up to 4,096 the image path: above 2,048 rows the tiles' un-split
  // k loop loses to the split-K slabs + combine, the image path does not: profiles/r6_wgrad_small_kimg.txt)
  const bool split_ok = p.xsync && rb_wgsmall() && rowband_split_ok(p.rows, H, p.in, nh, p.act);
  const bool kimg = split_ok && p.rows <= 4096 && wgrad_kimg_ok(p.rows);
  const bool wgs = kimg || (split_ok && p.rows <= 2048);
  for (int l = 0; l < RB_MAXL; ++l) p.ka[l] = p.kz[l] = nullptr;
  p.kbands = 0;
  if (kimg) {
    bf16* kb = reinterpret_cast<bf16*>(p.hx + G * 8 * RB_ROWS);
    const size_t per_img = 2 * rb_kimg_floats(H, p.in);   // (bf16 elements)
    for (int l = 0; l < nh; ++l) {
      p.ka[l] = kb + (size_t)(2 * l) * per_img;
      p.kz[l] = kb + (size_t)(2 * l + 1) * per_img;
    }
    p.kbands = (int)G;
  }
  hipError_t e = hipSuccess;
  if (st.phase <= 1) {
    e = rowband_fwd_bwd(p, s);
    if (e != hipSuccess) return e;
  }
  if (st.plan < 0 || st.plan > 1) return hipErrorInvalidValue;
  // the layers of this phase: [l0, l1); phase 1 also combines the head
  const int l0 = st.phase == 1 ? nh - 1 : 0;
  const int l1 = st.phase == 2 ? nh - 1 : nh;
  const bool head = st.phase != 2;
  WgradArgs jobs[RB_MAXL];
  SlabReduce red[RB_MAXL + 1];
  int sp[RB_MAXL];
  const int nj = l1 - l0;
  for (int l = l0; l < l1; ++l) {
    jobs[l - l0] = WgradArgs{p.dz[l], H, l == 0 ? p.X : p.a[l - 1], l == 0 ? p.ldx : H, st.gW[l],
                             st.gb[l], H, l == 0 ? p.in : H, p.rows, slabs + (size_t)l * per, st.sg};
    sp[l - l0] = rb_layer_splits(st.plan, st.splits, nh, H, p.rows, l);
  }
  const SlabReduce head_red{p.wslab, (int)G, H, 1, H, st.gWh, H, p.bslab, 1, st.gbh, p.loss_part,
                            (int)G, st.loss_scale, st.loss_out, st.sg};
  // (<= 2,048 rows: above, the un-split k loop -- ~0.35 us per 64 rows -- loses to the split-K
  // slabs + combine: 4,096 rows 31.3 vs 16.8 + 9.1 us, 3,000 rows 25.5 vs 14.7 + 9.1;
  // profiles/r5_wgrad_small_ab.txt)
  if (nj > 0 && wgs) {
    WgOut im[RB_MAXL];
    const bool img = st.sg.g_base && p.Pf[0];
    for (int l = l0; l < l1; ++l)
      im[l - l0] = WgOut{img ? const_cast<bf16*>(p.Pf[l]) : nullptr,
                         img && l >= 1 ? const_cast<bf16*>(p.Pd[l]) : nullptr, nullptr, p.kz[l], p.ka[l]};
    return wgrad_small(jobs, nj, im, head ? &head_red : nullptr, s, p.kbands);
  }
#if NNMPI_EXPERIMENTS_BUILD
  if (nj > 0 && rb_fixup()) {
    // one launch: every layer's weight gradient, its split-K combine + update in the tile's last
    // split, and the head's combine in extra blocks
    WgOut fx[RB_MAXL];
    for (int l = l0; l < l1; ++l) {
      const bool img = st.sg.g_base && p.Pf[0];
      fx[l - l0] = WgOut{img ? const_cast<bf16*>(p.Pf[l]) : nullptr,
                              img && l >= 1 ? const_cast<bf16*>(p.Pd[l]) : nullptr,
                              cnt + (size_t)l * rb_counters(H, p.in)};
    }
    const hipError_t ef = wgrad_multi_fix(jobs, nj, sp, fx, head ? &head_red : nullptr, s);
    if (ef != hipErrorNotSupported) return ef;   // (more splits than the fixup takes: below)
  }
#endif
  if (nj > 0) {
    e = wgrad_multi(jobs, nj, sp, red, s);
    if (e != hipSuccess) return e;
    if (st.sg.g_base && p.Pf[0]) {
      // one rank: the combines apply the update, and write the v2 weight images of the NEW
      // weights for the next step's row-band launch
      for (int l = l0; l < l1; ++l) {
        red[l - l0].pkf = const_cast<bf16*>(p.Pf[l]);
        red[l - l0].pkd = l >= 1 ? const_cast<bf16*>(p.Pd[l]) : nullptr;
      }
    }
  }
  int nr = nj;
  if (head) red[nr++] = head_red;
  if (nr == 0) return hipSuccess;
  return slab_reduce_multi(red, nr, s);
}

}  // namespace nnmpi
