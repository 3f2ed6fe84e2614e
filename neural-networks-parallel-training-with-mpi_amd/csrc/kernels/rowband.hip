// Row-band step for narrow square MLPs (every hidden width and the input width = H = 512, a
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
// Block = 8 waves (512 threads) x 32 rows; wave w owns output columns [64w, 64w+64) of every
// layer (2 x 4 v_mfma_f32_16x16x32_bf16 tiles).  LDS (the whole 160 KiB): ONE activation image
// of the band (the KMAJ image of gemm_tiles.h per 64-deep k-block: conflict-free row-fragment
// reads), updated in place by every pass -- a barrier separates a pass's main loop from its
// epilogue -- and two 8 KiB weight stages per wave: KMAJ [64 n][64 k] for the forward's B
// operand, XMAJ [64 k][64 x] for the dgrad's transposed operand (ds_read_b64_tr_b16, the GEMMs'
// XMAJ image).  The weights stream global -> registers (whole 128-byte lines per load
// instruction, a 1-deep ring of k-steps pinned with sched_barrier) -> the stage buffer the
// fragment reads of the current k-step are not using.  After each pass the image is copied out
// row-contiguously (activations and dZ are needed by the weight gradients).
#include "gemm_tiles.h"
#include "knobs.h"

namespace nnmpi {

constexpr int RB_ROWS = 32;
constexpr int RB_WAVES = 8;
constexpr int RB_THREADS = 64 * RB_WAVES;
// k-steps of weight loads in flight per lane beyond the staged one: 1 measured fastest with the
// double-buffered stage (0.0772-0.0775 ms/step vs 0.0783-0.0784 at 2 and 0.0802-0.0805 at 3,
// profiles/r3s2_rowband_ring_depth_ab.txt) -- deeper rings only add VGPRs and queued requests
constexpr int RB_RING = 1;

template <int H>
struct RbGeom {
  static_assert(H == 512, "row-band step: H = 512");
  static constexpr int KSTEPS = H / 64;
  static constexpr int WCOLS = H / RB_WAVES;       // output columns per wave
  static constexpr int NJ = WCOLS / 16;            // 16-column MFMA tiles per wave
  static constexpr int KB_BYTES = RB_ROWS * 128;   // one 64-deep k-block of an image
  static constexpr int BUF = RB_ROWS * H * 2;      // one activation image
  static constexpr int STAGE = 64 * WCOLS * 2;     // wave-private dgrad weight stage
  static constexpr int SMEM = BUF + RB_WAVES * 2 * STAGE;   // 160 KiB: the whole LDS
  static constexpr int FLD = 2 * NJ;               // forward: weight loads per lane per k-step
  static constexpr int DLD = WCOLS / 8;            // dgrad: 16-B stage chunks per lane per k-step
};

// byte offset of element (row r, column k) in an activation image
__device__ __forceinline__ int rb_off(int r, int k) {
  return (k >> 6) * (RB_ROWS * 128) + kmaj_off(r, (k >> 3) & 7) + ((k & 7) << 1);
}

// Row-contiguous copy between an LDS image and a [rows][ld] bf16 matrix (rows row0 .. row0 +
// nvalid - 1): each wave moves whole 128-byte row pieces (8 lanes per row).
template <int H>
__device__ __forceinline__ void rb_copy_out(const char* img, bf16* dst, int ld, int nvalid, int tid) {
  constexpr int CH = RB_ROWS * H / 8;
#pragma unroll
  for (int it = 0; it < CH / RB_THREADS; ++it) {
    const int id = tid + it * RB_THREADS;
    const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8));
    if (r < nvalid) *reinterpret_cast<bf16x8*>(dst + (long long)r * ld + kb * 64 + k8 * 8) = v;
  }
}

template <int H>
__device__ __forceinline__ void rb_load_in(char* img, const bf16* src, int ld, int nvalid, int tid) {
  constexpr int CH = RB_ROWS * H / 8;
  bf16x8 v[CH / RB_THREADS];
#pragma unroll
  for (int it = 0; it < CH / RB_THREADS; ++it) {
    const int id = tid + it * RB_THREADS;
    const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
    const int rr = min(r, nvalid - 1);   // clamped: every load issues; padding rows zeroed below
    v[it] = *reinterpret_cast<const bf16x8*>(src + (long long)rr * ld + kb * 64 + k8 * 8);
    if (r >= nvalid) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[it][e] = (bf16)0.f;
    }
  }
#pragma unroll
  for (int it = 0; it < CH / RB_THREADS; ++it) {
    const int id = tid + it * RB_THREADS;
    const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
    *reinterpret_cast<bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8)) = v[it];
  }
}

// One forward layer of the band: out = act(in . W^T + b) into the other image.  The wave's
// weight rows stream through its private stage as a KMAJ image ([64 n][64 k] per k-step,
// 8 lanes per 128-byte row piece: whole cache lines per load instruction).  Loading the B
// fragments straight from global memory (16 rows x 32-64 B per load instruction, two k
// permutations tried) ran the three forward passes in 51 us vs 29 us staged
// (profiles/r3s2_rowband_ab.txt, r3s2_rowband_fwd_direct_and_wgrad_ns_ab.txt).
template <int H, int ACT, int RING = RB_RING>
__device__ __forceinline__ void rb_forward(const bf16* __restrict__ W, const float* __restrict__ bias,
                                           const char* in, char* out, char* stage, int w, int lane) {
  using G = RbGeom<H>;
  const int n0 = w * G::WCOLS;
  f32x4 acc[2][G::NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // stage chunk q of k-step t: W[n0 + (lane >> 3) + 8q][64t + 8(lane & 7) .. +7]
  const bf16* wp = W + (long long)(n0 + (lane >> 3)) * H + 8 * (lane & 7);
  int soff[G::DLD];
#pragma unroll
  for (int q = 0; q < G::DLD; ++q) soff[q] = kmaj_off((lane >> 3) + 8 * q, lane & 7);
  bf16x8 ring[RING][G::DLD];
  auto issue = [&](int t, bf16x8 (&dst)[G::DLD]) {
#pragma unroll
    for (int q = 0; q < G::DLD; ++q)
      dst[q] = *reinterpret_cast<const bf16x8*>(wp + (long long)8 * q * H + 64 * t);
  };
  f32x4 bv[G::NJ];
#pragma unroll
  for (int j = 0; j < G::NJ; ++j) bv[j] = *reinterpret_cast<const f32x4*>(bias + n0 + 16 * j + 4 * (lane >> 4));
#pragma unroll
  for (int s = 0; s < RING; ++s) issue(s, ring[s]);
  // (sched_barrier: keep each ring refill where it is issued -- left alone, the scheduler sinks
  // the loads next to their first use and the ring degenerates to a few loads in flight)
  __builtin_amdgcn_sched_barrier(0);
  {
    // two stage buffers: the stage write of k-step t+1 is issued behind the fragment reads of
    // k-step t, so the MFMAs of t wait for their reads only, not for the next write
#pragma unroll
    for (int q = 0; q < G::DLD; ++q) *reinterpret_cast<bf16x8*>(stage + soff[q]) = ring[0][q];
    __builtin_amdgcn_sched_barrier(0);
    if (RING < G::KSTEPS) issue(RING, ring[0]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int t = 0; t < G::KSTEPS; ++t) {
    const char* st = stage + (t & 1) * G::STAGE;
    const char* kb = in + t * G::KB_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], bfr[G::NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = read_frag<64, KMAJ>(kb, 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) bfr[j] = read_frag<64, KMAJ>(st, 16 * j, kk, lane);
      {
        if (kk == 1) {
          // the next k-step's stage write goes out behind this half's reads: the MFMAs below
          // wait for the reads only
          __builtin_amdgcn_sched_barrier(0);
          if (t + 1 < G::KSTEPS) {
            char* nx = stage + ((t + 1) & 1) * G::STAGE;
#pragma unroll
            for (int q = 0; q < G::DLD; ++q) *reinterpret_cast<bf16x8*>(nx + soff[q]) = ring[(t + 1) % RING][q];
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 + RING < G::KSTEPS) issue(t + 1 + RING, ring[(t + 1) % RING]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();   // in place: every wave has read the whole input image
  // lane holds out[16i + (lane & 15)][n0 + 16j + 4(lane >> 4) .. +3]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) {
      const f32x4 v = acc[i][j] + bv[j];
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)act_fwd_t<ACT>(v[r]);
      *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) = o;
    }
}

// One activation-gradient layer: out = (in . W) * act'(aux), in = dZ_l (image), aux = a_{l-1}
// rows of this band in global memory (written by this block's earlier copy-out).
template <int H, int ACT, int RING = RB_RING>
__device__ __forceinline__ void rb_dgrad(const bf16* __restrict__ W, const char* in, char* out,
                                         char* stage, const bf16* aux, int nvalid, int w, int lane) {
  using G = RbGeom<H>;
  const int n0 = w * G::WCOLS;
  f32x4 acc[2][G::NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // stage chunk q of k-step t: W[64t + (lane >> 3) + 8q][n0 + 8(lane & 7) .. +7] -> XMAJ image
  const bf16* wp = W + (long long)(lane >> 3) * H + n0 + 8 * (lane & 7);
  int soff[G::DLD];
#pragma unroll
  for (int q = 0; q < G::DLD; ++q) {
    const int k = (lane >> 3) + 8 * q, ch = lane & 7;
    soff[q] = k * (G::WCOLS * 2) + ((ch ^ swz_x<G::WCOLS>(k)) << 4);
  }
  bf16x8 ring[RING][G::DLD];
  auto issue = [&](int t, bf16x8 (&dst)[G::DLD]) {
#pragma unroll
    for (int q = 0; q < G::DLD; ++q)
      dst[q] = *reinterpret_cast<const bf16x8*>(wp + (long long)(64 * t + 8 * q) * H);
  };
  // the epilogue's saved activations, loaded up front (their latency hides under the main loop)
  bf16x4 ax[2][G::NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) {
      const int m = min(16 * i + (lane & 15), nvalid - 1);
      ax[i][j] = *reinterpret_cast<const bf16x4*>(aux + (long long)m * H + n0 + 16 * j + 4 * (lane >> 4));
    }
#pragma unroll
  for (int s = 0; s < RING; ++s) issue(s, ring[s]);
  __builtin_amdgcn_sched_barrier(0);
  {
#pragma unroll
    for (int q = 0; q < G::DLD; ++q) *reinterpret_cast<bf16x8*>(stage + soff[q]) = ring[0][q];
    __builtin_amdgcn_sched_barrier(0);
    if (RING < G::KSTEPS) issue(RING, ring[0]);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int t = 0; t < G::KSTEPS; ++t) {
    const char* st = stage + (t & 1) * G::STAGE;
    const char* kb = in + t * G::KB_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], bfr[G::NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = read_frag<64, KMAJ>(kb, 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) bfr[j] = read_frag<G::WCOLS, XMAJ>(st, 16 * j, kk, lane);
      {
        if (kk == 1) {
          // the next k-step's stage write goes out behind this half's reads: the MFMAs below
          // wait for the reads only
          __builtin_amdgcn_sched_barrier(0);
          if (t + 1 < G::KSTEPS) {
            char* nx = stage + ((t + 1) & 1) * G::STAGE;
#pragma unroll
            for (int q = 0; q < G::DLD; ++q) *reinterpret_cast<bf16x8*>(nx + soff[q]) = ring[(t + 1) % RING][q];
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 + RING < G::KSTEPS) issue(t + 1 + RING, ring[(t + 1) % RING]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();   // in place: every wave has read the whole input image
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] * act_bwd_t<ACT>((float)ax[i][j][r]));
      *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) = o;
    }
}

// The band's head weight/bias-gradient and loss partials: column k of wslab by thread k, rows in
// order (deterministic), from the per-row dlogits / squared errors in LDS.
template <int H>
__device__ __forceinline__ void rb_head_partials(const RowbandArgs& p, const char* act,
                                                 const float* dls, const float* lss, int tid,
                                                 int blk) {
  for (int k = tid; k < H; k += RB_THREADS) {
    float s = 0.f;
#pragma unroll 8
    for (int r = 0; r < RB_ROWS; ++r) s += dls[r] * (float)*reinterpret_cast<const bf16*>(act + rb_off(r, k));
    p.wslab[(long long)blk * H + k] = s;
  }
  if (tid == 0) {
    float b = 0.f, l = 0.f;
    for (int r = 0; r < RB_ROWS; ++r) {
      b += dls[r];
      l += lss[r];
    }
    p.bslab[blk] = b;
    p.loss_part[blk] = l;
  }
}

// Regression head (out == 1, MSE) on the band's last activations `in`: logit, loss, dlogit, the
// head's weight/bias-gradient partials of this band, and dZ_{L-2} = dl * w * act'(a) into `out`.
template <int H, int ACT>
__device__ __forceinline__ void rb_head(const RowbandArgs& p, const char* in, char* out, float* dls,
                                        float* lss, int row0, int nvalid, int tid) {
  constexpr int CPT = H / 8 / 16;   // 8-column chunks per thread (16 threads per row)
  const int r = tid >> 4, g = tid & 15;
  float a[CPT][8], wv[CPT][8];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int k = 8 * (g + 16 * c);
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + rb_off(r, k));
    const float4 w0 = *reinterpret_cast<const float4*>(p.wh + k);
    const float4 w1 = *reinterpret_cast<const float4*>(p.wh + k + 4);
    wv[c][0] = w0.x; wv[c][1] = w0.y; wv[c][2] = w0.z; wv[c][3] = w0.w;
    wv[c][4] = w1.x; wv[c][5] = w1.y; wv[c][6] = w1.z; wv[c][7] = w1.w;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[c][e] = (float)v[e];
      dot += a[c][e] * wv[c][e];
    }
  }
#pragma unroll
  for (int sh = 8; sh >= 1; sh >>= 1) dot += __shfl_xor(dot, sh, 64);
  const bool valid = r < nvalid;
  const float yv = p.y[row0 + min(r, nvalid - 1)];
  const float d = dot + p.bh[0] - yv;
  const float dl = valid ? 2.f * d * p.inv_count : 0.f;
  if (g == 0) {
    dls[r] = dl;
    lss[r] = valid ? d * d : 0.f;
  }
  {
    // in place: the band's weight-gradient partial reads the activations before dZ replaces them
    __syncthreads();
    rb_head_partials<H>(p, in, dls, lss, tid, blockIdx.x);
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int k = 8 * (g + 16 * c);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)(dl * wv[c][e] * act_bwd_t<ACT>(a[c][e]));
    *reinterpret_cast<bf16x8*>(out + rb_off(r, k)) = o;
  }
}

// The band's whole chain.  ONE activation image, updated in place by every pass (a barrier
// between a pass's main loop and its epilogue), and two 8 KiB stage buffers per wave: the whole
// 160 KiB LDS.  (Two ping-pong images + one stage buffer per wave: 0.0815-0.0819 vs 0.0804-0.0808
// ms/step, profiles/r3s2_rowband_inplace_db_ab.txt.)
template <int H, int ACT, int RING = RB_RING>
__global__ void __launch_bounds__(RB_THREADS) rowband_kernel(RowbandArgs p) {
  using G = RbGeom<H>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  char* img = smem;
  char* stage = smem + G::BUF + w * 2 * G::STAGE;
  // head scratch: wave 0's stage, idle between the last forward pass and the first dgrad
  float* dls = reinterpret_cast<float*>(smem + G::BUF);
  float* lss = dls + RB_ROWS;
  const int blk = blockIdx.x;
  const int row0 = blk * RB_ROWS;
  const int nvalid = min(RB_ROWS, p.rows - row0);
  const int nh = p.nh;
  const int cg = (w + blk) & (RB_WAVES - 1);

  rb_load_in<H>(img, p.X + (long long)row0 * p.ldx, p.ldx, nvalid, tid);
  __syncthreads();
  for (int l = 0; l < nh; ++l) {
    rb_forward<H, ACT, RING>(p.W[l], p.b[l], img, img, stage, cg, lane);
    __syncthreads();
    rb_copy_out<H>(img, p.a[l] + (long long)row0 * H, H, nvalid, tid);
  }
  // (the partials' reads and the dZ writes are ordered by the head's own barriers; the stage
  // scratch is free: every wave has passed the last forward pass's barriers)
  rb_head<H, ACT>(p, img, img, dls, lss, row0, nvalid, tid);
  __syncthreads();
  rb_copy_out<H>(img, p.dz[nh - 1] + (long long)row0 * H, H, nvalid, tid);
  for (int l = nh - 1; l >= 1; --l) {
    rb_dgrad<H, ACT, RING>(p.W[l], img, img, stage, p.a[l - 1] + (long long)row0 * H, nvalid, cg, lane);
    __syncthreads();
    rb_copy_out<H>(img, p.dz[l - 1] + (long long)row0 * H, H, nvalid, tid);
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
__device__ __forceinline__ Rb2Mat rb2_mat(const RowbandArgs& p, int q, int cg) {
  using G = Rb2Geom<H>;
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
  m.b = base + (long long)cg * G::NJ * ts;
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
template <int H, int D>
__device__ __forceinline__ void rb2_mainloop(bf16x8 (&ring)[D][Rb2Geom<H>::NF],
                                             f32x4 (&acc)[2][Rb2Geom<H>::NJ], const char* img,
                                             const Rb2Mat& cur, const Rb2Mat& nxt, int lane) {
  using G = Rb2Geom<H>;
  const int voff = lane * 16;
  int s0 = 0;
  do {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = s0 + d;
      const char* kb = img + s * G::KB_BYTES;
      bf16x8 af[2][2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i][kk] = read_frag<64, KMAJ>(kb, 16 * i, kk, lane);
      // slot d: every later slot (D - 1 k-steps) may stay in flight, and the second k-half
      rb2_wait<(D - 1) * G::NF + G::NJ, G::NJ>(ring[d], 0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[d][2 * j], af[i][0], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);   // (the first half's MFMAs stay ahead of the second wait)
      rb2_wait<(D - 1) * G::NF, G::NJ>(ring[d], 1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < G::NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[d][2 * j + 1], af[i][1], acc[i][j], 0, 0, 0);
      // (sched_barrier: the refill stays behind this sub-step's MFMAs, which read the slot)
      __builtin_amdgcn_sched_barrier(0);
      const int sn = s + D;
      const bool inc = sn < cur.ks;
      rb2_issue<G::NJ>(ring[d], inc ? cur.b : nxt.b, inc ? cur.ts : nxt.ts, inc ? sn : sn - cur.ks, voff);
      __builtin_amdgcn_sched_barrier(0);
    }
    s0 += D;
  } while (s0 < cur.ks);
}

// The band's input rows into the image (runtime width, a multiple of 128 up to 1024): all of a
// thread's loads are issued before any LDS write, so they are in flight together.  Every load
// issues unconditionally (past the width: the chunk of iteration 0 again, an L1 hit) -- a load
// guarded by the runtime width made hipcc wait for each one separately.
__device__ __forceinline__ void rb2_load_in(char* img, const bf16* src, int ld, int width, int nvalid, int tid) {
  constexpr int MAXIT = 1024 * RB_ROWS / 8 / RB_THREADS;   // 8
  const int nit = width * RB_ROWS / 8 / RB_THREADS;
  bf16x8 v[MAXIT];
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    const int id = tid + min(it, nit - 1) * RB_THREADS;
    const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
    v[it] = *reinterpret_cast<const bf16x8*>(src + (long long)min(r, nvalid - 1) * ld + kb * 64 + k8 * 8);
  }
#pragma unroll
  for (int it = 0; it < MAXIT; ++it) {
    if (it < nit) {
      const int id = tid + it * RB_THREADS;
      const int kb = id / (RB_ROWS * 8), r = (id >> 3) & (RB_ROWS - 1), k8 = id & 7;
      bf16x8 x = v[it];
      if (r >= nvalid) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = (bf16)0.f;
      }
      *reinterpret_cast<bf16x8*>(img + kb * (RB_ROWS * 128) + kmaj_off(r, k8)) = x;
    }
  }
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

// Regression head of the band (out == 1, MSE) in place on `z` = a_{nh-1}: logit, loss, dlogit,
// the band's head-gradient partials, then dZ_{nh-1} = dl * w * act'(a) over a.
template <int H, int ACT>
__device__ __forceinline__ void rb2_head(const RowbandArgs& p, char* z, const Rb2Par& q, int nvalid, int tid,
                                         int band) {
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
  __syncthreads();
  rb_head_partials<H>(p, z, q.dls, q.lss, tid, band);
  __syncthreads();   // every partial has read a before dZ replaces it
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

template <int H, int ACT, int D>
__global__ void __launch_bounds__(RB_THREADS) rowband2_kernel(RowbandArgs p) {
  using G = Rb2Geom<H>;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
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

  // Startup: the ring's first D k-steps, the band's rows and the small operands are all issued
  // before the first wait, so the launch pays one memory round trip, not one per operand.
  bf16x8 ring[D][G::NF];
  Rb2Mat cur = rb2_mat<H>(p, 0, cg);
#pragma unroll
  for (int d = 0; d < D; ++d) rb2_issue<G::NJ>(ring[d], cur.b, cur.ts, d, lane * 16);
  {
    // (thread t < H / 4 loads float4 t of every layer's bias and of the head weight; the layer
    // index is unrolled so each bias pointer is a kernel-argument load, not a memory load of
    // the pointer array that hipcc would wait for)
    f32x4 bq[RB_MAXL], wq;
    const int tq = min(tid, H / 4 - 1);
#pragma unroll
    for (int l = 0; l < RB_MAXL; ++l) bq[l] = reinterpret_cast<const f32x4*>(p.b[l < nh ? l : 0])[tq];
    wq = reinterpret_cast<const f32x4*>(p.wh)[tq];
    const float yq = p.y[row0 + min(tid & (RB_ROWS - 1), nvalid - 1)];
    const float bhq = p.bh[0];
    rb2_load_in(slot(0), p.X + (long long)row0 * p.ldx, p.ldx, IN, nvalid, tid);
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

  f32x4 acc[2][G::NJ];
  // ---- forward: a_l = act(a_{l-1} W_l^T + b_l) ----
  for (int l = 0; l < nh; ++l) {
    const Rb2Mat nxt = rb2_mat<H>(p, l + 1, cg);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* in = slot(l == 0 ? 0 : l);
    char* out = l < nh - 1 ? slot(l + 1) : slot(nh >= 2 ? 0 : 1);
    rb2_mainloop<H, D>(ring, acc, in, cur, nxt, lane);
    // lane holds out[16i + (lane & 15)][n0 + 16j + 4(lane >> 4) .. +3]
    const float* bl = q.bias + l * H + n0 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < G::NJ; ++j) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(bl + 16 * j);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = acc[i][j] + bv;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)act_fwd_t<ACT>(v[r]);
        *reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4))) = o;
      }
    }
    __syncthreads();
    rb_copy_out<H>(out, p.a[l] + (long long)row0 * H, H, nvalid, tid);
    cur = nxt;
  }
  // ---- head (in place on a_{nh-1}) ----
  char* z = slot(nh >= 2 ? 0 : 1);
  rb2_head<H, ACT>(p, z, q, nvalid, tid, band);
  __syncthreads();
  rb_copy_out<H>(z, p.dz[nh - 1] + (long long)row0 * H, H, nvalid, tid);
  // ---- activation gradients: dZ_{l-1} = (dZ_l W_l) * act'(a_{l-1}), in place over a_{l-1} ----
  for (int l = nh - 1; l >= 1; --l) {
    const Rb2Mat nxt = rb2_mat<H>(p, 2 * nh - l, cg);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    char* out = slot(l);   // holds a_{l-1}
    rb2_mainloop<H, D>(ring, acc, z, cur, nxt, lane);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < G::NJ; ++j) {
        bf16x4* po = reinterpret_cast<bf16x4*>(out + rb_off(16 * i + (lane & 15), n0 + 16 * j + 4 * (lane >> 4)));
        const bf16x4 ax = *po;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] * act_bwd_t<ACT>((float)ax[r]));
        *po = o;
      }
    __syncthreads();
    rb_copy_out<H>(out, p.dz[l - 1] + (long long)row0 * H, H, nvalid, tid);
    z = out;
    cur = nxt;
  }
}

static int rb2_smem(int H, int in, int nh) {
  return std::max(nh, 2) * RB_ROWS * std::max(H, in) * 2 + rb2_par_bytes(H, nh);
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
  hipLaunchKernelGGL(f, dim3(rowband_blocks(p.rows)), dim3(RB_THREADS), rb2_smem(H, p.in, p.nh), s, p);
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

bool rowband_ok(int rows, int H, int in, int nh, int out, int loss, int act) {
  return rows > 0 && H == 512 && in == H && nh >= 1 && nh <= RB_MAXL && out == 1 &&
         loss == LOSS_MSE && (act == ACT_RELU || act == ACT_TANH || act == ACT_NONE);
}

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

hipError_t rowband_fwd_bwd(const RowbandArgs& p0, hipStream_t s) {
  RowbandArgs p = p0;
  p.band_map = rb_band_map();
  if (p.Pf[0]) {   // v2: packed weight images
    if (!rowband2_ok(p.rows, p.H, p.in, p.nh, 1, LOSS_MSE, p.act)) return hipErrorInvalidValue;
    for (int l = 0; l < p.nh; ++l)
      if (!p.Pf[l] || (l >= 1 && !p.Pd[l])) return hipErrorInvalidValue;
    switch (p.H) {
      case 256: return rowband2_launch<256>(p, s);
      case 384: return rowband2_launch<384>(p, s);
      case 512: return rowband2_launch<512>(p, s);
      case 768: return rowband2_launch<768>(p, s);
      case 1024: return rowband2_launch<1024>(p, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (!rowband_ok(p.rows, p.H, p.H, p.nh, 1, LOSS_MSE, p.act)) return hipErrorInvalidValue;

  using G = RbGeom<512>;
  using Fn = void (*)(RowbandArgs);
  static const Fn fns[3] = {rowband_kernel<512, ACT_NONE>, rowband_kernel<512, ACT_RELU>,
                            rowband_kernel<512, ACT_TANH>};
  static bool attr = false;
  if (!attr) {
    for (Fn f : fns)
      (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, G::SMEM);
    attr = true;
  }
  const Fn f = fns[p.act == ACT_RELU ? 1 : p.act == ACT_TANH ? 2 : 0];
  hipLaunchKernelGGL(f, dim3(rowband_blocks(p.rows)), dim3(RB_THREADS), G::SMEM, s, p);
  return hipGetLastError();
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

size_t rowband_workspace_bytes(int rows, int H, int in, int nh, int splits) {
  const size_t G = (size_t)rowband_blocks(rows);
  const int S = rb_max_splits(splits, nh, H, rows);
  const size_t head = G * H + rb_pad4(G) + rb_pad4(G);
  return (head + (size_t)nh * S * ((size_t)H * std::max(H, in) + H)) * sizeof(float);
}

hipError_t rowband_step(const RowbandStep& st0, hipStream_t s) {
  RowbandStep st = st0;
  RowbandArgs& p = st.fb;
  if (!p.Pf[0]) p.in = p.H;
  const bool ok = p.Pf[0] ? rowband2_ok(p.rows, p.H, p.in, p.nh, 1, LOSS_MSE, p.act)
                          : rowband_ok(p.rows, p.H, p.H, p.nh, 1, LOSS_MSE, p.act);
  if (!ok || !st.ws || st.phase < 0 || st.phase > 2) return hipErrorInvalidValue;
  const int H = p.H, nh = p.nh;
  const size_t G = (size_t)rowband_blocks(p.rows);
  float* ws = st.ws;
  p.wslab = ws;
  p.bslab = ws + G * H;
  p.loss_part = p.bslab + rb_pad4(G);
  float* slabs = p.loss_part + rb_pad4(G);
  hipError_t e = hipSuccess;
  if (st.phase <= 1) {
    e = rowband_fwd_bwd(p, s);
    if (e != hipSuccess) return e;
  }
  const size_t per = (size_t)rb_max_splits(st.splits, nh, H, p.rows) * ((size_t)H * std::max(H, p.in) + H);
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
  if (head) {
    red[nr++] = SlabReduce{p.wslab, (int)G, H, 1, H, st.gWh, H, p.bslab, 1, st.gbh, p.loss_part,
                           (int)G, st.loss_scale, st.loss_out, st.sg};
  }
  if (nr == 0) return hipSuccess;
  return slab_reduce_multi(red, nr, s);
}

}  // namespace nnmpi
