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
#include "common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>

namespace nnmpi {

enum Layout : int { KMAJ = 0, XMAJ = 1 };

constexpr int GEMM_BK = 64;
constexpr int GEMM_THREADS = 256;

struct GemmParams {
  const bf16* A;
  const bf16* B;
  int lda, ldb;
  int M, N, K;
  int k_per_split;
  void* C;
  int ldc;
  long long c_split_stride;
  const float* bias;
  const bf16* aux;
  int ldaux;
  float* bias_grad;
  long long bg_split_stride;
  unsigned a_bytes, b_bytes;  // extents of A / B storage (buffer-resource range, DMA path)
};

// XOR swizzle of the 16-byte chunk index for XMAJ images (rows of BX bf16).
template <int BX>
__device__ __forceinline__ int swz_x(int k) {
  if constexpr (BX == 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1;  // BX == 64
}

// KMAJ image: rows of 64 k = 128 B, 8 chunks.
__device__ __forceinline__ int kmaj_off(int r, int k8) { return r * 128 + ((k8 ^ ((r >> 1) & 7)) << 4); }

template <int BX, int LAYOUT>
__device__ __forceinline__ int xmaj_off(int k, int x) {
  return k * (BX * 2) + ((((x >> 3) ^ swz_x<BX>(k))) << 4) + ((x & 7) << 1);
}

template <int BX, int LAYOUT>
struct TileLoader {
  static constexpr int CHUNKS = BX * GEMM_BK / 8;
  static constexpr int PER_THREAD = CHUNKS / GEMM_THREADS;
  static_assert(PER_THREAD >= 1, "tile too small");
  uint4 regs[PER_THREAD];

  __device__ __forceinline__ void load(const bf16* __restrict__ base, int ld, int x0, int X,
                                       int k0, int kend, int tid) {
#pragma unroll
    for (int it = 0; it < PER_THREAD; ++it) {
      const int c = tid + it * GEMM_THREADS;
      int x, k;
      if constexpr (LAYOUT == KMAJ) {
        x = x0 + (c >> 3);
        k = k0 + ((c & 7) << 3);
      } else {
        constexpr int CPR = BX / 8;
        k = k0 + c / CPR;
        x = x0 + (c % CPR) * 8;
      }
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (x < X && k < kend) {
        const bf16* ptr = (LAYOUT == KMAJ) ? base + (long long)x * ld + k : base + (long long)k * ld + x;
        v = *reinterpret_cast<const uint4*>(ptr);
      }
      regs[it] = v;
    }
  }

  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int it = 0; it < PER_THREAD; ++it) {
      const int c = tid + it * GEMM_THREADS;
      int off;
      if constexpr (LAYOUT == KMAJ) {
        off = kmaj_off(c >> 3, c & 7);
      } else {
        constexpr int CPR = BX / 8;
        const int k = c / CPR, ch = c % CPR;
        off = k * (BX * 2) + ((ch ^ swz_x<BX>(k)) << 4);
      }
      *reinterpret_cast<uint4*>(lds + off) = regs[it];
    }
  }
};

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds operand (x = xb + (l&15), k = kk*32 +
// 8*(l>>4) + j), j = 0..7.  Same lane map for the A and the B operand.
template <int BX, int LAYOUT>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int xb, int kk, int lane) {
  if constexpr (LAYOUT == KMAJ) {
    const int r = xb + (lane & 15);
    const int k8 = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off(r, k8));
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int k = kk * 32 + 8 * (lane >> 4) + q;
    const int x = xb + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(lds + xmaj_off<BX, LAYOUT>(k, x)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s16x4*)(lds + xmaj_off<BX, LAYOUT>(k + 4, x)));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Epilogue shared by both main loops: lane holds C[m][n..n+3] for each (i, j) fragment.
// All epilogue operands (bias, activation aux) are loaded up front, then every fragment is
// finished and stored: no load waits behind the stores (stores count in vmcnt on gfx950).
template <int BM, int BN, int WGM, int WGN, int EPI, int ACT, bool BIASGRAD>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p,
                                              f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16],
                                              f32x4 (&accb)[BM / WGM / 16], bool do_bg, int m0, int n0,
                                              int wm, int wn, int lane, int split) {
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  int mrow[MI];
  int ncol[NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) mrow[i] = m0 + wm * WM + i * 16 + (lane & 15);
#pragma unroll
  for (int j = 0; j < NJ; ++j) ncol[j] = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
  if constexpr (EPI == EPI_BIAS_ACT) {
    f32x4 bias[NJ];
    // unconditional (clamped) loads: no per-element branch -> no vmcnt(0) per element
    if (p.bias) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bias[j] = *reinterpret_cast<const f32x4*>(p.bias + min(ncol[j], p.N - 4));
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bias[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if (mrow[i] >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (ncol[j] >= p.N) continue;
        const f32x4 v = acc[i][j] + bias[j];
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)act_fwd_t<ACT>(v[r]);
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p.C) + (long long)mrow[i] * p.ldc + ncol[j]) = o;
      }
    }
  } else if constexpr (EPI == EPI_DACT) {
    bf16x4 aux[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        aux[i][j] = *reinterpret_cast<const bf16x4*>(p.aux + (long long)min(mrow[i], p.M - 1) * p.ldaux +
                                                     min(ncol[j], p.N - 4));
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if (mrow[i] >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (ncol[j] >= p.N) continue;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[i][j][r] * act_bwd_t<ACT>((float)aux[i][j][r]));
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p.C) + (long long)mrow[i] * p.ldc + ncol[j]) = o;
      }
    }
  } else {
    float* cbase = reinterpret_cast<float*>(p.C) + split * p.c_split_stride;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      if (mrow[i] >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (ncol[j] >= p.N) continue;
        *reinterpret_cast<f32x4*>(cbase + (long long)mrow[i] * p.ldc + ncol[j]) = acc[i][j];
      }
    }
  }
  if constexpr (BIASGRAD) {
    if (do_bg && (lane >> 4) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + wm * WM + i * 16 + lane;
        if (m < p.M) p.bias_grad[split * p.bg_split_stride + m] = accb[i][0];
      }
    }
  }
}

template <int BM, int BN, int LA, int LB, int EPI, int ACT, bool BIASGRAD>
__global__ void __launch_bounds__(GEMM_THREADS) gemm_bf16_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BK = GEMM_BK;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NJ = WN / 16;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int gx = gridDim.x, gy = gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
  const int tx = bid % gx, ty = bid / gx;
  const int m0 = ty * BM, n0 = tx * BN;
  const int split = blockIdx.z;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  TileLoader<BM, LA> la;
  TileLoader<BN, LB> lb;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bg = BIASGRAD && tx == 0 && wn == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;

  if (nt > 0) {
    la.load(p.A, p.lda, m0, p.M, kbeg, kend, tid);
    lb.load(p.B, p.ldb, n0, p.N, kbeg, kend, tid);
    la.store(smem, tid);
    lb.store(smem + A_BYTES, tid);
    __syncthreads();
  }
  for (int t = 0; t < nt; ++t) {
    const char* cur = smem + (t & 1) * STAGE;
    const bool more = t + 1 < nt;
    if (more) {
      la.load(p.A, p.lda, m0, p.M, kbeg + (t + 1) * BK, kend, tid);
      lb.load(p.B, p.ldb, n0, p.N, kbeg + (t + 1) * BK, kend, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = read_frag<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = read_frag<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      if constexpr (BIASGRAD) {
        if (do_bg) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[i], accb[i], 0, 0, 0);
        }
      }
    }
    if (more) {
      char* nxt = smem + ((t + 1) & 1) * STAGE;
      la.store(nxt, tid);
      lb.store(nxt + A_BYTES, tid);
    }
    __syncthreads();
  }

  gemm_epilogue<BM, BN, 2, 2, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, m0, n0, wm, wn, lane, split);
}


// ------------------------------------------------------------------------------------------
// v2 main loop: LDS-DMA (buffer_load ... lds) into an NS-deep ring, counted vmcnt, raw barrier.
//
// The MLP GEMMs are short-K (K = 512..8192 per block) and, at one 256-thread block per CU, a
// register-staged loop exposes one full memory round trip per 64-deep k-step.  Here every wave
// DMAs its share of each stage straight into LDS (16 B per lane, no VGPR round trip) and keeps
// NS-1 stages in flight; one counted `s_waitcnt vmcnt` + one `s_barrier` per k-step
// (cdna_hip_programming.md §5 "Pipelining across barriers", rules 21/4(a)).  The LDS images are
// the same XOR-swizzled images as v1; since a DMA writes lane-linearly, the swizzle is applied to
// each lane's SOURCE address (rule 21).  Out-of-range chunks (M/N/K tails, split-K ends) get a
// source offset past the buffer-resource range, so the hardware returns zeros.
// ------------------------------------------------------------------------------------------
constexpr unsigned DMA_OOB = 0x7FFFFFF0u;

__device__ __forceinline__ constexpr int waitcnt_vm(int n) {
  return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8);
}

template <int N>
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(waitcnt_vm(N)); }

template <int BX, int LAYOUT, int NW>
struct DmaPlan {
  static constexpr int IMG = BX * GEMM_BK * 2;          // bytes per stage for this operand
  static constexpr int NI = IMG / 1024 / NW;            // DMA instructions per wave per stage
  static_assert(NI >= 1 && NI * NW * 1024 == IMG, "operand stage must split evenly over the waves");
  unsigned off[NI];   // byte offset of this lane's source chunk for k0 = 0
  int kq[NI];         // k offset of the chunk within the tile
  bool xv[NI];        // x in range
  unsigned kstride;   // bytes per unit of k0

  __device__ __forceinline__ void init(int w, int lane, int x0, int X, int ld) {
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int o = (w * NI + q) * 1024 + lane * 16;
      if constexpr (LAYOUT == KMAJ) {
        const int r = o >> 7, cp = (o >> 4) & 7, c = cp ^ ((r >> 1) & 7);
        off[q] = (unsigned)(((long long)(x0 + r) * ld + c * 8) * 2);
        kq[q] = c * 8;
        xv[q] = (x0 + r) < X;
      } else {
        constexpr int RB = BX * 2;
        const int r = o / RB, cp = (o % RB) >> 4, c = cp ^ swz_x<BX>(r);
        off[q] = (unsigned)(((long long)r * ld + x0 + c * 8) * 2);
        kq[q] = r;
        xv[q] = (x0 + c * 8) < X;
      }
    }
    kstride = (LAYOUT == KMAJ) ? 2u : (unsigned)ld * 2u;
  }

  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* lds_stage, int w, int k0,
                                        int kend) const {
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const unsigned v = (xv[q] && (k0 + kq[q]) < kend) ? off[q] + (unsigned)k0 * kstride : DMA_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(lds_stage + (w * NI + q) * 1024), 16, v, 0, 0, 0);
    }
  }
};

template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int ACT, bool BIASGRAD, int NS>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_bf16_dma_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr int NW = WGM * WGN;
  constexpr int BK = GEMM_BK;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  constexpr int PER_TILE = DmaPlan<BM, LA, NW>::NI + DmaPlan<BN, LB, NW>::NI;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int gx = gridDim.x, gy = gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
  const int tx = bid % gx, ty = bid / gx;
  const int m0 = ty * BM, n0 = tx * BN;
  const int split = blockIdx.z;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, (short)0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, (short)0, (int)p.b_bytes, 0x00020000);
  DmaPlan<BM, LA, NW> da;
  DmaPlan<BN, LB, NW> db;
  da.init(w, lane, m0, p.M, p.lda);
  db.init(w, lane, n0, p.N, p.ldb);

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bg = BIASGRAD && tx == 0 && wn == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;

  // prologue: NS-1 stages in flight
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) {
    if (t < nt) {
      char* st = smem + t * STAGE;
      da.issue(rsA, st, w, kbeg + t * BK, kend);
      db.issue(rsB, st + A_BYTES, w, kbeg + t * BK, kend);
    }
  }
  for (int t = 0; t < nt; ++t) {
    // retire stage t: allow the (newer) stages t+1 .. min(t+NS-2, nt-1) to stay in flight
    const int newer = min(NS - 2, nt - 1 - t);
    if constexpr (NS >= 4) {
      if (newer >= 2) wait_vm<2 * PER_TILE>();
      else if (newer == 1) wait_vm<PER_TILE>();
      else wait_vm<0>();
    } else if constexpr (NS == 3) {
      if (newer >= 1) wait_vm<PER_TILE>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    // refill the stage consumed in iteration t-1 (all waves are past its reads)
    if (t + NS - 1 < nt) {
      char* st = smem + ((t + NS - 1) % NS) * STAGE;
      da.issue(rsA, st, w, kbeg + (t + NS - 1) * BK, kend);
      db.issue(rsB, st + A_BYTES, w, kbeg + (t + NS - 1) * BK, kend);
    }
    const char* cur = smem + (t % NS) * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[MI], bfr[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = read_frag<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bfr[j] = read_frag<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      if constexpr (BIASGRAD) {
        if (do_bg) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[i], accb[i], 0, 0, 0);
        }
      }
    }
    // all of this wave's LDS reads of stage t are consumed before the next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  gemm_epilogue<BM, BN, WGM, WGN, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, m0, n0, wm, wn, lane, split);
}

// Deterministic split-K / partial-slab combine, one launch for the three jobs a backward needs:
//   blocks [0, nb_main)         out[m][n] = sum_z ws[z][m][n]     (64 float4 columns per block)
//   blocks [nb_main, +nb_bias)  bout[m]   = sum_z bws[z][m]       (64 scalars per block)
//   one more block (optional)   *loss_out = loss_scale * sum_i loss_part[i]
// WS waves per block split the S partials (wave w sums z = w, w+WS, ... in order) and the wave
// partials are combined in wave order through LDS: bitwise reproducible for a given (S, WS).
template <int WS>
__global__ void __launch_bounds__(64 * WS) slab_reduce_kernel(
    const float* __restrict__ ws, int S, long long stride, int M, int N, float* __restrict__ out,
    int ldo, int nb_main, const float* __restrict__ bws, long long bstride, float* __restrict__ bout,
    int nb_bias, const float* __restrict__ loss_part, int n_loss_part, float loss_scale,
    float* __restrict__ loss_out, SgdFuse sg) {
  __shared__ f32x4 part[WS][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x;
  if (b < nb_main) {
    const int nv = N >> 2;
    const long long nvec = (long long)M * nv;
    const long long v = (long long)b * 64 + lane;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    long long m = 0, n = 0;
    if (v < nvec) {
      m = v / nv;
      n = (v % nv) * 4;
      const float* p = ws + m * N + n;
#pragma unroll 4
      for (int z = w; z < S; z += WS) acc += *reinterpret_cast<const f32x4*>(p + z * stride);
    }
    part[w][lane] = acc;
    __syncthreads();
    if (w == 0 && v < nvec) {
      f32x4 t = part[0][lane];
#pragma unroll
      for (int k = 1; k < WS; ++k) t += part[k][lane];
      if (sg.g_base) sgd_fused_store4(sg, out + m * ldo + n, t);
      else *reinterpret_cast<f32x4*>(out + m * ldo + n) = t;
    }
    return;
  }
  if (b < nb_main + nb_bias) {
    const long long m = (long long)(b - nb_main) * 64 + lane;
    float acc = 0.f;
    if (m < M) {
#pragma unroll 4
      for (int z = w; z < S; z += WS) acc += bws[z * bstride + m];
    }
    part[w][lane][0] = acc;
    __syncthreads();
    if (w == 0 && m < M) {
      float t = part[0][lane][0];
#pragma unroll
      for (int k = 1; k < WS; ++k) t += part[k][lane][0];
      if (sg.g_base) sgd_fused_store(sg, bout + m, t);
      else bout[m] = t;
    }
    return;
  }
  // loss partials: strided per-thread sums, then a fixed-order combine
  float acc = 0.f;
  for (int i = threadIdx.x; i < n_loss_part; i += 64 * WS) acc += loss_part[i];
  acc = wave_sum(acc);
  if (lane == 0) part[w][0][0] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < WS; ++k) t += part[k][0][0];
    *loss_out = t * loss_scale;
  }
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static int g_gemm_impl = -1;

static int gemm_impl() {
  if (g_gemm_impl < 0) {
    const char* e = getenv("NNMPI_GEMM");
    g_gemm_impl = (e && e[0] == '1') ? 1 : 2;   // 2 = LDS-DMA ring (default), 1 = register-staged
  }
  return g_gemm_impl;
}

void set_gemm_impl(int impl) { g_gemm_impl = impl; }
int get_gemm_impl() { return gemm_impl(); }

template <int LA, int LB>
static void set_extents(GemmParams& p) {
  // storage extents (bytes) of the operands, for the buffer-resource range checks
  const long long a = (LA == KMAJ) ? ((long long)(p.M - 1) * p.lda + p.K) : ((long long)(p.K - 1) * p.lda + p.M);
  const long long b = (LB == KMAJ) ? ((long long)(p.N - 1) * p.ldb + p.K) : ((long long)(p.K - 1) * p.ldb + p.N);
  p.a_bytes = (unsigned)std::min<long long>(a * 2, DMA_OOB - 16);
  p.b_bytes = (unsigned)std::min<long long>(b * 2, DMA_OOB - 16);
}

template <int BM, int BN, int WGM, int WGN, int NS, int LA, int LB, int EPI, int ACT, bool BG>
static hipError_t launch_dma(GemmParams p, int splits, hipStream_t s) {
  dim3 grid((p.N + BN - 1) / BN, (p.M + BM - 1) / BM, splits);
  constexpr int smem = NS * (BM + BN) * GEMM_BK * 2;
  set_extents<LA, LB>(p);
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

template <int BM, int BN, int LA, int LB, int EPI, int ACT, bool BG>
static hipError_t launch_t(GemmParams p, int splits, hipStream_t s) {
  if (gemm_impl() == 2) {
    if constexpr (BM == 128 && BN == 128) {
      switch (g_variant) {
        case 1: return launch_dma<128, 128, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 2: return launch_dma<128, 128, 2, 4, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 3: return launch_dma<128, 128, 4, 2, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 4: return launch_dma<128, 128, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 5: return launch_dma<64, 128, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);  // 2 blocks/CU
        case 6: return launch_dma<128, 64, 2, 2, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 7: return launch_dma<64, 128, 2, 4, 3, LA, LB, EPI, ACT, BG>(p, splits, s);
        case 8: return launch_dma<128, 128, 2, 2, 4, LA, LB, EPI, ACT, BG>(p, splits, s);
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

template <int BM, int BN, int LA, int LB, int EPI, bool BG>
static hipError_t launch_act(const GemmParams& p, int act, int splits, hipStream_t s) {
  switch (act) {
    case ACT_RELU: return launch_t<BM, BN, LA, LB, EPI, ACT_RELU, BG>(p, splits, s);
    case ACT_TANH: return launch_t<BM, BN, LA, LB, EPI, ACT_TANH, BG>(p, splits, s);
    default: return launch_t<BM, BN, LA, LB, EPI, ACT_NONE, BG>(p, splits, s);
  }
}

static int g_force_tile = 0;  // 0 = heuristic; 64 / 128 force a tile edge (experiments)
void set_gemm_tile(int t) { g_force_tile = t; }

static int pick_tile(int M, int N) {
  if (g_force_tile) return g_force_tile;
  // 128x128 when that already yields ~a full wave of blocks, else 64x64.
  const long long t128 = (long long)((M + 127) / 128) * ((N + 127) / 128);
  return t128 >= 192 ? 128 : 64;
}

hipError_t linear_fwd_bf16(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                           bf16* Y, int ldy, int M, int N, int K, int act, hipStream_t s) {
  GemmParams p{};
  p.A = X; p.lda = ldx; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = Y; p.ldc = ldy; p.bias = bias;
  if (pick_tile(M, N) == 128) return launch_act<128, 128, KMAJ, KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s);
  return launch_act<64, 64, KMAJ, KMAJ, EPI_BIAS_ACT, false>(p, act, 1, s);
}

hipError_t linear_dgrad_bf16(const bf16* dZ, int lddz, const bf16* W, int ldw, const bf16* Aprev,
                             int lda_prev, bf16* dX, int lddx, int M, int N, int K, int act,
                             hipStream_t s) {
  GemmParams p{};
  p.A = dZ; p.lda = lddz; p.B = W; p.ldb = ldw; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((K + GEMM_BK - 1) / GEMM_BK) * GEMM_BK;
  p.C = dX; p.ldc = lddx; p.aux = Aprev; p.ldaux = lda_prev;
  if (pick_tile(M, N) == 128) return launch_act<128, 128, KMAJ, XMAJ, EPI_DACT, false>(p, act, 1, s);
  return launch_act<64, 64, KMAJ, XMAJ, EPI_DACT, false>(p, act, 1, s);
}

static int wgrad_tile(int M, int N) {
  if (g_force_tile) return g_force_tile;
  return (M >= 128 && N >= 128) ? 128 : 64;
}

int wgrad_splits(int M, int N, int K) {
  // split the (long) batch reduction until ~one block per CU; keep >= 4 k-steps per split
  const int t = wgrad_tile(M, N);
  const int tiles = ((M + t - 1) / t) * ((N + t - 1) / t);
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  int s = 1;
  while (tiles * s < 256 && ksteps / (s * 2) >= 4 && s < 64) s *= 2;
  return s;
}

size_t wgrad_workspace_bytes(int M, int N, int K) {
  const int s = wgrad_splits(M, N, K);
  if (s == 1) return 0;
  return (size_t)s * ((size_t)M * N + M) * sizeof(float);
}

hipError_t linear_wgrad_bf16(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                             float* db, int M, int N, int K, float* ws, hipStream_t s,
                             const SgdFuse* sgd) {
  // dW[M=out][N=in] = sum_k dZ[k][m] X[k][n]; db[m] = sum_k dZ[k][m].
  const int splits = wgrad_splits(M, N, K);
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  const bool big = wgrad_tile(M, N) == 128;
  GemmParams p{};
  p.A = dZ; p.lda = lddz; p.B = X; p.ldb = ldx; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((ksteps + splits - 1) / splits) * GEMM_BK;
  float* bws = nullptr;
  if (splits == 1) {
    p.C = dW; p.ldc = N; p.c_split_stride = 0;
    p.bias_grad = db; p.bg_split_stride = 0;
  } else {
    if (ws == nullptr) return hipErrorInvalidValue;
    p.C = ws; p.ldc = N; p.c_split_stride = (long long)M * N;
    bws = ws + (size_t)splits * M * N;
    p.bias_grad = bws; p.bg_split_stride = M;
  }
  hipError_t e;
  if (big) e = db ? launch_t<128, 128, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, splits, s)
                  : launch_t<128, 128, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, splits, s);
  else e = db ? launch_t<64, 64, XMAJ, XMAJ, EPI_F32, ACT_NONE, true>(p, splits, s)
              : launch_t<64, 64, XMAJ, XMAJ, EPI_F32, ACT_NONE, false>(p, splits, s);
  if (e != hipSuccess || splits == 1) return e;
  return splitk_reduce(ws, splits, (long long)M * N, M, N, dW, N, db ? bws : nullptr, (long long)M, db,
                       nullptr, 0, 0.f, nullptr, s, sgd);
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

hipError_t splitk_reduce(const float* ws, int S, long long stride, int M, int N, float* out, int ldo,
                         const float* bws, long long bstride, float* bout, const float* loss_part,
                         int n_loss_part, float loss_scale, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd) {
  SgdFuse sg{};
  if (sgd) sg = *sgd;
  const long long nvec = (ws && out && S > 0) ? (long long)M * (N / 4) : 0;
  const int nb_main = (int)((nvec + 63) / 64);
  const int nb_bias = (bws && bout && S > 0) ? (M + 63) / 64 : 0;
  const int nb = nb_main + nb_bias + (loss_out ? 1 : 0);
  if (nb == 0) return hipSuccess;
#define SLAB_LAUNCH(WSV)                                                                          \
  hipLaunchKernelGGL(slab_reduce_kernel<WSV>, dim3(nb), dim3(64 * WSV), 0, s, ws, S, stride, M, N, \
                     out, ldo, nb_main, bws, bstride, bout, nb_bias, loss_part, n_loss_part,       \
                     loss_scale, loss_out, sg)
  if (S >= 64 || n_loss_part >= 4096) SLAB_LAUNCH(16);
  else if (S >= 8) SLAB_LAUNCH(8);
  else SLAB_LAUNCH(4);
#undef SLAB_LAUNCH
  return hipGetLastError();
}

}  // namespace nnmpi
