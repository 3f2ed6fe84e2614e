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
                                                 const float* dls, const float* lss, int tid) {
  const int blk = blockIdx.x;
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
    rb_head_partials<H>(p, in, dls, lss, tid);
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

int rowband_blocks(int rows) { return (rows + RB_ROWS - 1) / RB_ROWS; }

bool rowband_ok(int rows, int H, int in, int nh, int out, int loss, int act) {
  return rows > 0 && H == 512 && in == H && nh >= 1 && nh <= RB_MAXL && out == 1 &&
         loss == LOSS_MSE && (act == ACT_RELU || act == ACT_TANH || act == ACT_NONE);
}

static int rb_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e && e[0] >= '0' && e[0] <= '9') ? std::atoi(e) : dflt;
}

hipError_t rowband_fwd_bwd(const RowbandArgs& p0, hipStream_t s) {
  RowbandArgs p = p0;
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

size_t rowband_workspace_bytes(int rows, int H, int nh, int splits) {
  const size_t G = (size_t)rowband_blocks(rows);
  const int S = rb_splits(splits, nh, H, rows);
  const size_t head = G * H + rb_pad4(G) + rb_pad4(G);
  return (head + (size_t)nh * S * ((size_t)H * H + H)) * sizeof(float);
}

hipError_t rowband_step(const RowbandStep& st0, hipStream_t s) {
  RowbandStep st = st0;
  RowbandArgs& p = st.fb;
  if (!rowband_ok(p.rows, p.H, p.H, p.nh, 1, LOSS_MSE, p.act) || !st.ws) return hipErrorInvalidValue;
  const int H = p.H, nh = p.nh;
  const size_t G = (size_t)rowband_blocks(p.rows);
  float* ws = st.ws;
  p.wslab = ws;
  p.bslab = ws + G * H;
  p.loss_part = p.bslab + rb_pad4(G);
  float* slabs = p.loss_part + rb_pad4(G);
  hipError_t e = rowband_fwd_bwd(p, s);
  if (e != hipSuccess) return e;
  const int S = rb_splits(st.splits, nh, H, p.rows);
  WgradArgs jobs[RB_MAXL];
  SlabReduce red[RB_MAXL + 1];
  for (int l = 0; l < nh; ++l) {
    jobs[l] = WgradArgs{p.dz[l], H, l == 0 ? p.X : p.a[l - 1], l == 0 ? p.ldx : H, st.gW[l],
                        st.gb[l], H, H, p.rows, slabs + (size_t)l * S * ((size_t)H * H + H), st.sg};
  }
  e = wgrad_multi(jobs, nh, S, red, s);
  if (e != hipSuccess) return e;
  red[nh] = SlabReduce{p.wslab, (int)G, H, 1, H, st.gWh, H, p.bslab, 1, st.gbh, p.loss_part, (int)G,
                       st.loss_scale, st.loss_out, st.sg};
  return slab_reduce_multi(red, nh + 1, s);
}

}  // namespace nnmpi
