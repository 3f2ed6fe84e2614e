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
  SgdFuse sg;                 // EPI_F32 without split-K: apply the optimizer instead of storing
  int store_pol;              // epilogue output stores: 0 plain, 1 nt, 2 sc1 (write-through)
  bf16* c16;                  // EPI_F32 without split-K: store the gradient as bf16 here instead
  bf16* bg16;                 // (same ldc as C) and the bias gradient here -- the bf16 payload
  // Deferred update of ANOTHER arena region with the same [M][N] shape (several ranks, bf16
  // payload): this tile stores its own gradient as bf16 into c16 and applies SGD-momentum to the
  // other region's element (m, n) with the reduced bf16 gradient g16o[m * ldc + n]; sg2's bases
  // point at the other region's first element.  256x256 tiles, full tiles only.
  SgdFuse sg2;
  const bf16* g16o;
  int stage_epi;              // 256x256 forward: bias+act tile staged through LDS, row stores
  int sgd_serial;             // SGD epilogue form (A/B): 0 LDS-staged rows (256x256 tiles,
                              // default), 1 per fragment, 2 fragment rows batched
};
static int g_stage_epi = -1;   // NNMPI_STAGE_EPI=1: LDS-staged 256x256 forward epilogue (A/B)
void set_stage_epi(int on) { g_stage_epi = on; }   // -1: re-read the environment
static int stage_epi() {
  if (g_stage_epi < 0) {
    const char* e = std::getenv("NNMPI_STAGE_EPI");
    g_stage_epi = (e && e[0] == '1') ? 1 : 0;
  }
  return g_stage_epi;
}
static int g_sgd_serial = -1;   // NNMPI_SGD_SERIAL=<form> (experiments)
void set_sgd_epilogue(int form) { g_sgd_serial = form; }   // -1: re-read the environment
static int sgd_serial() {
  if (g_sgd_serial < 0) {
    const char* e = std::getenv("NNMPI_SGD_SERIAL");
    g_sgd_serial = (e && e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 0;
  }
  return g_sgd_serial;
}

// Epilogue output store of 16 bytes with a selectable cache policy (experiments: what the
// kernel leaves dirty in L2 is written back at the launch boundary, MI355X_MICROARCH.md
// "boundary" row; nt / sc1 stores move that traffic into the epilogue).  Vector stores only.
template <typename V>
__device__ __forceinline__ void store16(V* ptr, const V& v, int pol) {
  static_assert(sizeof(V) == 16, "16-byte store");
  if (pol == 1) {
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(ptr));
  } else if (pol == 2) {
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    const u32x4 d = __builtin_bit_cast(u32x4, v);
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ptr), "v"(d) : "memory");
  } else {
    *ptr = v;
  }
}
static int g_store_pol = 0;   // host: store16 policy the launches put in GemmParams (0 plain)

// s_waitcnt with only the vector-memory counter constrained (lgkm/exp counters left free).
__device__ __forceinline__ constexpr int waitcnt_vm(int n) {
  return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8);
}

template <int N>
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(waitcnt_vm(N)); }

// XOR swizzle of the 16-byte chunk index for XMAJ images (rows of BX bf16).
template <int BX>
__device__ __forceinline__ int swz_x(int k) {
  // rows of 256 B (BX 128) or 512 B (BX 256) both start at bank 0: same chunk XOR
  if constexpr (BX >= 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
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

// read_frag for kernels that retire their LDS reads themselves (explicit lgkmcnt(0) +
// sched_barrier before the consumers): the transposed reads are issued as inline asm, because
// for the ds_read_b64_tr_b16 builtin the compiler cannot prove independence from in-flight
// LDS-DMA writes and drains them with a vmcnt(0) in front of every such read, which would
// serialise the DMA pipeline.
template <int BX, int LAYOUT>
__device__ __forceinline__ bf16x8 read_frag_async(const char* lds, int xb, int kk, int lane) {
  if constexpr (LAYOUT == KMAJ) {
    return read_frag<BX, LAYOUT>(lds, xb, kk, lane);
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    const int k = kk * 32 + 8 * (lane >> 4) + q;
    const int x = xb + 4 * p;
    const unsigned a0 = (unsigned)(uintptr_t)(lds + xmaj_off<BX, LAYOUT>(k, x));
    const unsigned a1 = (unsigned)(uintptr_t)(lds + xmaj_off<BX, LAYOUT>(k + 4, x));
    typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
    u32x2 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(a1));
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    u32x4 v = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// SGD-momentum update of an accumulator tile in the epilogue (un-split weight gradient, single
// rank), batched: the master and momentum vectors of RB fragment rows (RB x NJ fragments) are
// loaded together BEFORE any of their results is stored, so a tile pays MI/RB memory round trips
// instead of MI x NJ (sgd_fused_store4 per fragment: the compiler cannot hoist the next
// fragment's loads above this one's stores -- the arena pointers may alias).  The
// hyper-parameters are read once.  Same arithmetic as sgd_fused_store4: bitwise identical.
template <int MI, int NJ, int RB = 1>
__device__ __forceinline__ void sgd_epilogue_batched(const SgdFuse& f, const f32x4 (&acc)[MI][NJ],
                                                     const int (&mrow)[MI], const int (&ncol)[NJ],
                                                     const float* cbase, int ldc, int M, int N) {
  const float lr = f.hp[0], mom = f.hp[1], damp = f.hp[2], wd = f.hp[3], gs = f.hp[4];
  const bool nest = f.nesterov != 0, first = f.first != 0;
  const long long base = cbase - f.g_base;
  auto offset = [&](int i, int j) {
    // clamped (always in range) so every load issues unconditionally; out-of-range fragments
    // are skipped at the store
    return base + (long long)min(mrow[i], M - 1) * ldc + min(ncol[j], N - 4);
  };
#pragma unroll
  for (int i0 = 0; i0 < MI; i0 += RB) {
    f32x4 pv[RB][NJ], bv[RB][NJ];
#pragma unroll
    for (int ii = 0; ii < RB; ++ii)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const long long o = offset(i0 + ii, j);
        pv[ii][j] = *reinterpret_cast<const f32x4*>(f.p_base + o);
        bv[ii][j] = *reinterpret_cast<const f32x4*>(f.m_base + o);
      }
#pragma unroll
    for (int ii = 0; ii < RB; ++ii) {
      if (mrow[i0 + ii] >= M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (ncol[j] >= N) continue;
        const long long o = offset(i0 + ii, j);
        f32x4 p = pv[ii][j], b = bv[ii][j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float bb = b[r];
          p[r] = sgd_elem(p[r], acc[i0 + ii][j][r], bb, lr, mom, damp, wd, gs, nest, first);
          b[r] = bb;
        }
        *reinterpret_cast<f32x4*>(f.p_base + o) = p;
        if (mom != 0.f) *reinterpret_cast<f32x4*>(f.m_base + o) = b;
        if (f.s_base) {
          bf16x4 sv;
#pragma unroll
          for (int r = 0; r < 4; ++r) sv[r] = (bf16)p[r];
          *reinterpret_cast<bf16x4*>(f.s_base + o) = sv;
        }
      }
    }
  }
}

// Epilogue shared by both main loops: lane holds C[m][n..n+3] for each (i, j) fragment.
// All epilogue operands (bias, activation aux) are loaded up front, then every fragment is
// finished and stored: no load waits behind the stores (stores count in vmcnt on gfx950).
// mrow[i]: this lane's output row of fragment row i; ncol[j]: first of its 4 output columns of
// fragment column j.
// bias_pre: the bias fragments already loaded at kernel start (EPI_BIAS_ACT; null: load here).
template <int MI, int NJ, int EPI, int ACT, bool BIASGRAD>
__device__ __forceinline__ void epilogue_store(const GemmParams& p, f32x4 (&acc)[MI][NJ],
                                               f32x4 (&accb)[MI], bool do_bg, const int (&mrow)[MI],
                                               const int (&ncol)[NJ], int lane, int split,
                                               const f32x4* bias_pre = nullptr,
                                               bool main_done = false) {
  if constexpr (EPI == EPI_BIAS_ACT) {
   if (!main_done) {
    f32x4 bias[NJ];
    // unconditional (clamped) loads: no per-element branch -> no vmcnt(0) per element
    if (bias_pre) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bias[j] = bias_pre[j];
    } else if (p.bias) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bias[j] = *reinterpret_cast<const f32x4*>(p.bias + min(ncol[j], p.N - 4));
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bias[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // Retire the operand loads explicitly BEFORE the first store: stores count in vmcnt too,
    // and behind the predicated (branchy) store sequence the compiler's own count goes
    // conservative -- it otherwise emits vmcnt(0/1) in front of every store, serialising
    // each store behind the previous one's completion.
    wait_vm<0>();
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
   }
  } else if constexpr (EPI == EPI_DACT) {
    bf16x4 aux[MI][NJ];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        aux[i][j] = *reinterpret_cast<const bf16x4*>(p.aux + (long long)min(mrow[i], p.M - 1) * p.ldaux +
                                                     min(ncol[j], p.N - 4));
    wait_vm<0>();   // see EPI_BIAS_ACT
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
    // a final (un-split) weight gradient on a single rank: the optimizer update is applied
    // here, in the epilogue -- no gradient store and no separate optimizer pass over it
    const bool fuse = p.sg.g_base != nullptr;
    bool batched = main_done;   // (the caller already applied the LDS-staged form)
    if (!batched) {
      if (fuse && !p.c16 && p.sgd_serial != 1) {
        sgd_epilogue_batched<MI, NJ>(p.sg, acc, mrow, ncol, cbase, p.ldc, p.M, p.N);
        batched = true;
      }
    }
    if (!batched) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (mrow[i] >= p.M) continue;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if (ncol[j] >= p.N) continue;
          if (p.c16) {   // the bf16 all-reduce payload, rounded as cast_f32_bf16 rounds
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (bf16)acc[i][j][r];
            *reinterpret_cast<bf16x4*>(p.c16 + (long long)mrow[i] * p.ldc + ncol[j]) = o;
            continue;
          }
          float* g = cbase + (long long)mrow[i] * p.ldc + ncol[j];
          if (fuse) sgd_fused_store4(p.sg, g, acc[i][j]);
          else *reinterpret_cast<f32x4*>(g) = acc[i][j];
        }
      }
    }
  }
  if constexpr (BIASGRAD) {
    // accb[i] = rowsum(A) of fragment row i; lane l < 16 holds the sum of row mrow[i] (= base + l)
    if (do_bg && (lane >> 4) == 0) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = mrow[i];
        if (m >= p.M) continue;
        if (p.bg16) { p.bg16[m] = (bf16)accb[i][0]; continue; }
        float* g = p.bias_grad + split * p.bg_split_stride + m;
        if (p.sg.g_base) sgd_fused_store(p.sg, g, accb[i][0]);
        else *g = accb[i][0];
      }
    }
  }
}

// Standard wave-grid epilogue: wave (wm, wn) owns the contiguous WM x WN sub-tile.
template <int BM, int BN, int WGM, int WGN, int EPI, int ACT, bool BIASGRAD>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p,
                                              f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16],
                                              f32x4 (&accb)[BM / WGM / 16], bool do_bg, int m0, int n0,
                                              int wm, int wn, int lane, int split,
                                              const f32x4* bias_pre = nullptr) {
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  int mrow[MI];
  int ncol[NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i) mrow[i] = m0 + wm * WM + i * 16 + (lane & 15);
#pragma unroll
  for (int j = 0; j < NJ; ++j) ncol[j] = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
  epilogue_store<MI, NJ, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, mrow, ncol, lane, split, bias_pre);
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
// Row-contiguous epilogue for 128x128 tiles (LDS transpose).
//
// In fragment order a lane owns 4 consecutive columns of one row per fragment, so every store
// instruction of a wave writes 16 separate 32-byte row pieces (and the dgrad epilogue READS its
// saved activation the same way): a store-issue-bound tail of several microseconds per launch
// (a 1-k-step 8192x512 forward still took 5.5 us).  Here the fp32 accumulators are parked in
// the idle LDS ring as a swizzled [128][128] image (16-byte chunk c of row r at c ^ (r & 31):
// conflict-free ds_write_b128 / ds_read_b128), read back 8 columns per lane, and every wave
// instruction then stores (and loads its epilogue operands for) 4 whole output rows.  The
// arithmetic is unchanged (same fp32 values, same bias / activation order): results are bitwise
// identical to the fragment-order epilogue.
// ------------------------------------------------------------------------------------------
constexpr int LEPI_ROWS = 4;   // rows per wave-iteration (16 lanes x 8 columns per row)

__device__ __forceinline__ int lepi_off(int r, int c4) { return r * 128 + ((c4 ^ (r & 31)) << 2); }

template <int EPI>
__device__ __forceinline__ bool lepi_ok(const GemmParams& p) {
  // whole 16-byte column chunks, 16-byte aligned rows (the fragment epilogue covers the rest)
  if (p.N % 8) return false;
  if constexpr (EPI == EPI_F32)
    return p.c16 == nullptr && (p.ldc % 4) == 0 && ((uintptr_t)p.C & 15) == 0;
  else if constexpr (EPI == EPI_DACT)
    return (p.ldc % 8) == 0 && ((uintptr_t)p.C & 15) == 0 && (p.ldaux % 8) == 0 &&
           ((uintptr_t)p.aux & 15) == 0;
  else return (p.ldc % 8) == 0 && ((uintptr_t)p.C & 15) == 0 && ((uintptr_t)p.bias & 15) == 0;
}

template <int WGM, int WGN, int EPI, int ACT>
__device__ __forceinline__ void lds_epilogue(const GemmParams& p,
                                             f32x4 (&acc)[128 / WGM / 16][128 / WGN / 16],
                                             char* smem, int m0, int n0, int wm, int wn, int w,
                                             int lane, int split) {
  constexpr int NW = WGM * WGN, WM = 128 / WGM, WN = 128 / WGN, MI = WM / 16, NJ = WN / 16;
  constexpr int ITER = 128 / (NW * LEPI_ROWS);
  float* img = reinterpret_cast<float*>(smem);
  const int q = lane & 15;                        // this lane's 8-column chunk of a row
  const int gn = n0 + q * 8;
  // epilogue operands first (their latency hides under the LDS staging below)
  f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = {0.f, 0.f, 0.f, 0.f};
  bf16x8 aux[EPI == EPI_DACT ? ITER : 1];
  if constexpr (EPI == EPI_BIAS_ACT) {
    if (p.bias && gn < p.N) {
      b0 = *reinterpret_cast<const f32x4*>(p.bias + gn);
      b1 = *reinterpret_cast<const f32x4*>(p.bias + gn + 4);
    }
  } else if constexpr (EPI == EPI_DACT) {
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int gm = min(m0 + (it * NW + w) * LEPI_ROWS + (lane >> 4), p.M - 1);
      aux[it] = *reinterpret_cast<const bf16x8*>(p.aux + (long long)gm * p.ldaux + min(gn, p.N - 8));
    }
  }
  // every wave is past its last read of the ring (and, with the final vmcnt(0), every DMA landed)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = wm * WM + i * 16 + (lane & 15);
      const int c4 = (wn * WN + j * 16) / 4 + (lane >> 4);
      *reinterpret_cast<f32x4*>(img + lepi_off(r, c4)) = acc[i][j];
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const bool fuse = (EPI == EPI_F32) && p.sg.g_base != nullptr;
  float* cbase = reinterpret_cast<float*>(p.C) + (EPI == EPI_F32 ? split * p.c_split_stride : 0);
#pragma unroll
  for (int it = 0; it < ITER; ++it) {
    const int r = (it * NW + w) * LEPI_ROWS + (lane >> 4);
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(img + lepi_off(r, 2 * q));
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(img + lepi_off(r, 2 * q + 1));
    const int gm = m0 + r;
    if (gm >= p.M || gn >= p.N) continue;
    if constexpr (EPI == EPI_F32) {
      float* g = cbase + (long long)gm * p.ldc + gn;
      if (fuse) {
        sgd_fused_store4(p.sg, g, v0);
        sgd_fused_store4(p.sg, g + 4, v1);
      } else {
        store16(reinterpret_cast<f32x4*>(g), v0, p.store_pol);
        store16(reinterpret_cast<f32x4*>(g + 4), v1, p.store_pol);
      }
    } else {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if constexpr (EPI == EPI_BIAS_ACT) {
          o[e] = (bf16)act_fwd_t<ACT>(v0[e] + b0[e]);
          o[e + 4] = (bf16)act_fwd_t<ACT>(v1[e] + b1[e]);
        } else {
          o[e] = (bf16)(v0[e] * act_bwd_t<ACT>((float)aux[it][e]));
          o[e + 4] = (bf16)(v1[e] * act_bwd_t<ACT>((float)aux[it][e + 4]));
        }
      }
      store16(reinterpret_cast<bf16x8*>(reinterpret_cast<bf16*>(p.C) + (long long)gm * p.ldc + gn), o,
              p.store_pol);
    }
  }
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

// One output tile (tx, ty) of K-split `split` — the body shared by the standalone GEMM launch
// and the grouped backward launch (bwd_group_kernel).
// ASYNC_TR (only matters when an operand is XMAJ, i.e. read with ds_read_b64_tr_b16):
//   0  compiler-scheduled reads -- hipcc cannot prove the tr-read builtin independent of the
//      in-flight LDS-DMA and drains vmcnt(0) in front of it, so the DMA ring degenerates to
//      load-then-compute inside the block;
//   1  the whole stage's fragments through asm reads + ONE explicit lgkmcnt per k-step (most
//      VGPRs: every fragment of the stage is live at once);
//   2  asm reads + explicit lgkmcnt per 32-deep k-half (half the fragment registers of 1, so
//      the 512-thread grouped launch keeps 2 blocks per CU).
template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int ACT, bool BIASGRAD, int NS,
          int ASYNC_TR = 1>
__device__ __forceinline__ void dma_gemm_tile(const GemmParams& p, char* smem, int tx, int ty,
                                              int split) {
  constexpr int NW = WGM * WGN;
  constexpr int BK = GEMM_BK;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NJ = WN / 16;
  constexpr int PER_TILE = DmaPlan<BM, LA, NW>::NI + DmaPlan<BN, LB, NW>::NI;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int m0 = ty * BM, n0 = tx * BN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.K, kbeg + p.k_per_split);
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // The epilogue's bias is fetched before the main loop (it is the oldest load, so the ring's
  // counted vmcnt waits retire it first): no dependent L2 round trip between the last MFMA and
  // the first output store.
  f32x4 bias_pre[EPI == EPI_BIAS_ACT ? NJ : 1];
  if constexpr (EPI == EPI_BIAS_ACT) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = min(n0 + wn * WN + j * 16 + (lane >> 4) * 4, p.N - 4);
      bias_pre[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
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
    constexpr bool TR = (LA == XMAJ || LB == XMAJ);
    if constexpr (ASYNC_TR == 2 && TR) {
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 af[MI], bfr[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = read_frag_async<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j] = read_frag_async<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
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
    } else if constexpr (ASYNC_TR == 1 && TR) {
      // transposed operands: all fragments of the stage through asm reads (read_frag_async),
      // one explicit lgkmcnt(0), then the MFMAs -- keeps the compiler from draining the
      // in-flight DMA ring (vmcnt(0)) in front of every ds_read_b64_tr_b16
      bf16x8 af[MI][BK / 32], bfr[NJ][BK / 32];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i][kk] = read_frag_async<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[j][kk] = read_frag_async<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
        if constexpr (BIASGRAD) {
          if (do_bg) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
              accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[i][kk], accb[i], 0, 0, 0);
          }
        }
      }
    } else {
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
    }
    // all of this wave's LDS reads of stage t are consumed before the next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (BM == 128 && BN == 128 && NS * STAGE >= 128 * 128 * 4) {
    if (lepi_ok<EPI>(p)) {
      lds_epilogue<WGM, WGN, EPI, ACT>(p, acc, smem, m0, n0, wm, wn, w, lane, split);
      if constexpr (BIASGRAD) {
        // bias gradient: lane l < 16 holds the row sum of row wm*WM + i*16 + l
        if (do_bg && (lane >> 4) == 0) {
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int m = m0 + wm * WM + i * 16 + (lane & 15);
            if (m >= p.M) continue;
            float* g = p.bias_grad + split * p.bg_split_stride + m;
            if (p.sg.g_base) sgd_fused_store(p.sg, g, accb[i][0]);
            else *g = accb[i][0];
          }
        }
      }
      return;
    }
  }
  gemm_epilogue<BM, BN, WGM, WGN, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, m0, n0, wm, wn, lane, split,
                                                      EPI == EPI_BIAS_ACT ? bias_pre : nullptr);
}

template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int ACT, bool BIASGRAD, int NS>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm_bf16_dma_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int gx = gridDim.x, gy = gridDim.y;
  const int bid = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy);
  dma_gemm_tile<BM, BN, WGM, WGN, LA, LB, EPI, ACT, BIASGRAD, NS>(p, smem, bid % gx, bid / gx, blockIdx.z);
}

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

hipError_t linear_fwd_bf16_stamped(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
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

// ------------------------------------------------------------------------------------------
// Large-shape kernel: 256x256 tile, 8 waves as 2 (M) x 4 (N), "ping-pong" phase schedule
// (cdna_hip_programming.md §5, 256² 8-phase template; structure re-derived here for our operand
// layouts).
//
// Each operand's K-tile is split into two HALVES of 128 contiguous x (A rows / B columns) x 64
// k: every half is an ordinary 128-wide swizzled image (16 KiB, full 128-B source lines for
// both operand layouts), filled by DmaPlan<128>.  Wave (wm, wn) owns rows
// {h*128 + wm*64 + [0, 64)} and columns {h*128 + wn*32 + [0, 32)} of both halves h, so its
// 128x64 output splits into four 64x32 QUADRANTS (A half, B half), computed in four PHASES
// per K-tile: P1 (A0, B0), P2 (A0, B1), P3 (A1, B1), P4 (A1, B0).  Every half is read into
// registers ONCE per K-tile -- P1 A0, P2 B1, P3 A1, P4 the NEXT K-tile's B0 (second register
// set) -- so the memory sections are balanced (8 | 4 | 8 | 4 fragment reads); then the phase
// issues its share of LDS-DMA for later K-tiles and runs its 16 MFMAs at raised priority.
// Wave row 1 runs one barrier behind wave row 0, so on every SIMD one wave's memory section
// overlaps the other's MFMA section.
//
// LDS: 2 K-tile buffers x {A0, A1, B0, B1} x 16 KiB = 128 KiB.  While computing K-tile t:
// P1 issues A1(t+1), P3 A0(t+2) + B0(t+2), P4 B1(t+2) -- each half restaged two phases after
// its single read (WAR) and issued ~six phases before it is read.  Before each barrier a
// counted `vmcnt` retires exactly the half the NEXT phase reads (RAW: "read a staged buffer one
// phase AFTER the wait that retires it").  Past the end of K the DMAs carry an out-of-range
// offset (zero fill, no traffic) so every wave's vmcnt arithmetic stays uniform.
// ------------------------------------------------------------------------------------------
constexpr int PP_HALF = 16384;             // bytes of one half image
constexpr int PP_BUF = 4 * PP_HALF;        // one K-tile: A0 A1 B0 B1
constexpr int PP_SMEM = 2 * PP_BUF;        // 128 KiB
constexpr int PP_THREADS = 512;

// LATE_LGKM: the phase's LDS reads are retired AFTER the pre-MFMA barrier (their latency
// overlaps the barrier wait; cdna_hip_programming.md 8-phase template order).  WAR margin: a
// half is re-staged >= 2 phases after its read, and with the one-barrier stagger the earliest
// overwriting DMA issue is 3 barriers after the read's phase barrier, so retiring the reads one
// barrier later stays inside it.
// GM: grouped tile order (grouped_tile) -- 32 blocks resident per XCD read 4 A + 8 B panels per
// K-tile instead of 1 A + 32 B at the 8192-wide shape.
// SGD epilogue of a full 256x256 weight-gradient tile, staged through the (then idle) 128 KiB LDS
// ring: each 128-row half of the fp32 tile is written to LDS ([128 rows][64 float4], float4 index
// XOR (row & 15): conflict-free for the fragment writes and the row reads), then every wave
// updates whole rows -- each memory instruction moves 1 KiB contiguous of master / momentum
// (512 B of the bf16 shadow) instead of 16 row pieces of 64 B, and each lane keeps 8 rows of
// master + momentum loads in flight (2 round trips per half instead of 4 fragment rows).  Same
// arithmetic as sgd_fused_store4: bitwise identical.
// OTHER: the tile's own gradient goes to the bf16 payload c16 (row stores from the same staged
// image) and the update applies to the region sg2 / g16o (see GemmParams).
template <bool OTHER = false>
__device__ __forceinline__ void sgd_epilogue_lds_256(const GemmParams& p, const f32x4 (&acc)[8][4],
                                                     char* smem, int m0, int n0, int wm, int wn,
                                                     int w, int lane, int split) {
  const SgdFuse& f = OTHER ? p.sg2 : p.sg;
  const float lr = f.hp[0], mom = f.hp[1], damp = f.hp[2], wd = f.hp[3], gs = f.hp[4];
  const bool nest = f.nesterov != 0, first = f.first != 0;
  const float* cbase = reinterpret_cast<const float*>(p.C) + split * p.c_split_stride;
  const long long base = OTHER ? 0 : cbase - f.g_base;
  f32x4* img = reinterpret_cast<f32x4*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();   // the ring (h 0) / the previous half's rows (h 1) are no longer read
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int r = wm * 64 + ii * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cv = ((j >> 1) * 128 + wn * 32 + (j & 1) * 16) / 4 + (lane >> 4);
        img[r * 64 + (cv ^ (r & 15))] = acc[h * 4 + ii][j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      f32x4 pv[8], bv[8];
      f32x4 gov[OTHER ? 8 : 1];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = w * 16 + sb * 8 + k;
        const long long o = base + (long long)(m0 + h * 128 + r) * p.ldc + n0 + lane * 4;
        pv[k] = *reinterpret_cast<const f32x4*>(f.p_base + o);
        bv[k] = *reinterpret_cast<const f32x4*>(f.m_base + o);
        if constexpr (OTHER) {
          const bf16x4 gq = *reinterpret_cast<const bf16x4*>(p.g16o + o);
          gov[k] = f32x4{(float)gq[0], (float)gq[1], (float)gq[2], (float)gq[3]};
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = w * 16 + sb * 8 + k;
        const long long o = base + (long long)(m0 + h * 128 + r) * p.ldc + n0 + lane * 4;
        const f32x4 a = img[r * 64 + (lane ^ (r & 15))];
        f32x4 g = a;
        if constexpr (OTHER) {
          g = gov[k];
          bf16x4 o16;   // own gradient -> bf16 payload, rounded as cast_f32_bf16 rounds
#pragma unroll
          for (int e = 0; e < 4; ++e) o16[e] = (bf16)a[e];
          *reinterpret_cast<bf16x4*>(p.c16 + (long long)(m0 + h * 128 + r) * p.ldc + n0 + lane * 4) = o16;
        }
        f32x4 q = pv[k], b = bv[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float bb = b[e];
          q[e] = sgd_elem(q[e], g[e], bb, lr, mom, damp, wd, gs, nest, first);
          b[e] = bb;
        }
        *reinterpret_cast<f32x4*>(f.p_base + o) = q;
        if (mom != 0.f) *reinterpret_cast<f32x4*>(f.m_base + o) = b;
        if (f.s_base) {
          bf16x4 sv;
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[e] = (bf16)q[e];
          *reinterpret_cast<bf16x4*>(f.s_base + o) = sv;
        }
      }
    }
  }
}

// Forward epilogue of a full 256x256 tile staged through the idle 128 KiB LDS ring (A/B,
// NNMPI_STAGE_EPI=1): act(acc + bias) as bf16 into a [256 rows][64 x 8 B] image (8-byte unit
// index XOR 2*(row & 15): conflict-free fragment writes and row reads), then every wave stores
// whole rows -- 512 B contiguous per instruction instead of 16 row pieces of 32 B.
template <int ACT>
__device__ __forceinline__ void bias_act_lds_256(const GemmParams& p, const f32x4 (&acc)[8][4],
                                                 char* smem, int m0, int n0, int wm, int wn, int w,
                                                 int lane) {
  bf16x4* img = reinterpret_cast<bf16x4*>(smem);
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = n0 + (j >> 1) * 128 + wn * 32 + (j & 1) * 16 + (lane >> 4) * 4;
    bias[j] = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();   // the ring is no longer read
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int r = (i >> 2) * 128 + wm * 64 + (i & 3) * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int u = ((j >> 1) * 128 + wn * 32 + (j & 1) * 16) / 4 + (lane >> 4);
      const f32x4 v = acc[i][j] + bias[j];
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (bf16)act_fwd_t<ACT>(v[e]);
      img[r * 64 + (u ^ ((r & 15) << 1))] = o;
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int k = 0; k < 32; ++k) {
    const int r = w * 32 + k;
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(p.C) + (long long)(m0 + r) * p.ldc + n0 + lane * 4) =
        img[r * 64 + (lane ^ ((r & 15) << 1))];
  }
}

// One 256x256 output tile: `bid` is the tile's XCD-remapped id in a gx x gy grid (the standalone
// launch below, or one job of gemm_bf16_pp256_pair_kernel).
template <int LA, int LB, int EPI, int ACT, bool BIASGRAD, bool LATE_LGKM = true, int GM = 4>
__device__ __forceinline__ void pp256_tile(const GemmParams& p, char* smem, int bid, int gx, int gy,
                                           int split) {
  constexpr int BK = GEMM_BK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  int tx, ty;
  grouped_tile(bid, gx, gy, GM, tx, ty);
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
  auto A0 = [&](int b) { return smem + b * PP_BUF; };
  auto A1 = [&](int b) { return smem + b * PP_BUF + PP_HALF; };
  auto B0 = [&](int b) { return smem + b * PP_BUF + 2 * PP_HALF; };
  auto B1 = [&](int b) { return smem + b * PP_BUF + 3 * PP_HALF; };
  auto kof = [&](int t) { return kbeg + t * BK; };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rsum[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) rsum[i] = 0.f;
  const bool do_bg = BIASGRAD && tx == 0 && wn == 0;

  // prologue: K-tile 0 whole, K-tile 1's A0, B0, B1 (the steady-state issue order); retire
  // K-tile 0's A0 + B0 (five newer halves may stay in flight)
  pa0.issue(rsA, A0(0), w, kof(0), kend);
  pb0.issue(rsB, B0(0), w, kof(0), kend);
  pb1.issue(rsB, B1(0), w, kof(0), kend);
  pa1.issue(rsA, A1(0), w, kof(0), kend);
  pa0.issue(rsA, A0(1), w, kof(1), kend);
  pb0.issue(rsB, B0(1), w, kof(1), kend);
  pb1.issue(rsB, B1(1), w, kof(1), kend);
  wait_vm<10>();
  __builtin_amdgcn_s_barrier();

  bf16x8 af[4][2], b0f[2][2], b0n[2][2], b1f[2][2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) b0n[jj][kk] = read_frag_async<128, LB>(B0(0), wn * 32 + jj * 16, kk, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (wm == 1) __builtin_amdgcn_s_barrier();   // wave row 1 runs one barrier behind

  for (int t = 0; t < nt; ++t) {
    const int b = t & 1, nb = b ^ 1;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      // ---- memory section: new fragments, DMA, retire the half the next phase reads ----
      // Every half is read ONCE per K-tile: P1 A0, P2 B1, P3 A1, P4 B0 of the NEXT K-tile
      // (into a second register set; this K-tile's B0 is still needed by P4's MFMAs).
      if (ph == 0 || ph == 2) {
        const char* ai = ph ? A1(b) : A0(b);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) af[i][kk] = read_frag_async<128, LA>(ai, wm * 64 + i * 16, kk, lane);
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
          for (int kk = 0; kk < 2; ++kk) b1f[jj][kk] = read_frag_async<128, LB>(B1(b), wn * 32 + jj * 16, kk, lane);
      } else if (ph == 3) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) b0n[jj][kk] = read_frag_async<128, LB>(B0(nb), wn * 32 + jj * 16, kk, lane);
      }
      // issue: P1 A1(t+1) | P3 A0(t+2), B0(t+2) | P4 B1(t+2); retire: P1 -> B1(t) [vmcnt 10],
      // P2 -> A1(t) [8], P3 -> A0 + B0 (t+1) [8] (read in P4 and in the next P1)
      if (ph == 0) {
        pa1.issue(rsA, A1(nb), w, kof(t + 1), kend);
        wait_vm<10>();
      } else if (ph == 1) {
        wait_vm<8>();
      } else if (ph == 2) {
        pa0.issue(rsA, A0(b), w, kof(t + 2), kend);
        pb0.issue(rsB, B0(b), w, kof(t + 2), kend);
        wait_vm<8>();
      } else {
        pb1.issue(rsB, B1(b), w, kof(t + 2), kend);
      }
      if constexpr (LATE_LGKM) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
      }
      // ---- MFMA section: quadrant (hA, hB) ----
      const int hA = ph >> 1;                        // P1,P2 -> A0; P3,P4 -> A1
      const int hB = (ph == 1 || ph == 2) ? 1 : 0;   // P1,P4 -> B0; P2,P3 -> B1
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
        // bias gradient = row sums of A: VALU partial sums of the A fragments this lane holds
        // (rows lane&15, 16 of the 64 k), combined across the 4 lane groups at the end
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
  bool main_done = false;
  if constexpr (EPI == EPI_BIAS_ACT) {
    if (p.stage_epi && m0 + 256 <= p.M && n0 + 256 <= p.N) {
      bias_act_lds_256<ACT>(p, acc, smem, m0, n0, wm, wn, w, lane);
      main_done = true;
    }
  }
  if constexpr (EPI == EPI_F32) {
    // block-uniform condition (full tile, fused SGD): the LDS-staged row form
    if (p.sg.g_base && !p.c16 && p.sgd_serial == 0 && m0 + 256 <= p.M && n0 + 256 <= p.N) {
      sgd_epilogue_lds_256(p, acc, smem, m0, n0, wm, wn, w, lane, split);
      main_done = true;
    } else if (p.g16o && p.c16) {   // (the host admits full tiles only)
      sgd_epilogue_lds_256<true>(p, acc, smem, m0, n0, wm, wn, w, lane, split);
      main_done = true;
    }
  }
  epilogue_store<8, 4, EPI, ACT, BIASGRAD>(p, acc, accb, do_bg, mrow, ncol, lane, split, nullptr,
                                           main_done);
}

template <int LA, int LB, int EPI, int ACT, bool BIASGRAD, bool LATE_LGKM = true, int GM = 4>
__global__ void __launch_bounds__(PP_THREADS) gemm_bf16_pp256_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int gx = gridDim.x, gy = gridDim.y;
  pp256_tile<LA, LB, EPI, ACT, BIASGRAD, LATE_LGKM, GM>(
      p, smem, xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy), gx, gy, blockIdx.z);
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
    if (combiner && v < nvec) {
      f32x4 t = part[cg * WS * 64 + lane];
#pragma unroll
      for (int k = 1; k < WS; ++k) t += part[(cg * WS + k) * 64 + lane];
      if (upd) sgd_apply4(r.sg, pre, t);
      else if (r.sg.g_base) sgd_fused_store4(r.sg, o, t);
      else *reinterpret_cast<f32x4*>(o) = t;
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

constexpr int SLAB_PART_BYTES = 16 * 64 * 16;   // max(WS, NW) x 64 lanes x f32x4

template <int WS>
__global__ void __launch_bounds__(SLAB_THREADS) slab_reduce_kernel(SlabReduce r, int nb_main, int nb_bias) {
  __shared__ f32x4 part[SLAB_PART_BYTES / 16];
  slab_reduce_block<WS>(r, blockIdx.x, nb_main, nb_bias, part);
}

__device__ __forceinline__ void slab_reduce_any(int ws, const SlabReduce& r, int b, int nb_main,
                                                int nb_bias, f32x4* part) {
  switch (ws) {
    case 1: slab_reduce_block<1>(r, b, nb_main, nb_bias, part); break;
    case 2: slab_reduce_block<2>(r, b, nb_main, nb_bias, part); break;
    case 4: slab_reduce_block<4>(r, b, nb_main, nb_bias, part); break;
    case 8: slab_reduce_block<8>(r, b, nb_main, nb_bias, part); break;
    default: slab_reduce_block<16>(r, b, nb_main, nb_bias, part); break;
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
// 256x256 ping-pong kernel tile order per epilogue (index into its kernel table: 0 GM 4,
// 1 early reads GM 1, 2 GM 1, 3 GM 8): forward, dgrad, weight gradient
static int g_pp_order[3] = {0, 0, 2};
void set_pp256_order(int epi, int idx) {
  if (epi >= 0 && epi < 3 && idx >= 0 && idx < 4) g_pp_order[epi] = idx;
}

// Kernel-selection knobs of the training step (scripts/step_ab.py A/Bs them; -1 / 0 = default).
static int g_fwd_variant = -1;    // forward GEMM main-loop variant (launch_t's switch)
static int g_group_async = -1;    // grouped-backward LDS read mode (dma_gemm_tile ASYNC_TR)
static int g_wgrad_splits = 0;    // > 0: upper bound on the weight-gradient split-K factor
constexpr int FWD_VARIANT_DEFAULT = 0;
constexpr int GROUP_ASYNC_DEFAULT = 2;   // measured: 102.3 -> 97.9 us/step (proxy512, step_ab)
void set_fwd_variant(int v) { g_fwd_variant = v; }
void set_group_async(int m) { g_group_async = m; }
void set_wgrad_splits(int s) { g_wgrad_splits = s; }
void set_store_policy(int p) { g_store_pol = p; }

template <int BM, int BN, int LA, int LB, int EPI, int ACT, bool BG>
static hipError_t launch_t(GemmParams p, int splits, hipStream_t s, int variant = -1) {
  if (variant < 0) variant = g_variant;
  if constexpr (BM == 256 && BN == 256) {
    // large shapes: 256x256 tile, 8 waves (each 128x64), 128 KiB LDS, 1 block/CU
    if (variant == 9) return launch_dma<256, 256, 2, 4, 2, LA, LB, EPI, ACT, BG>(p, splits, s);
    dim3 grid((p.N + 255) / 256, (p.M + 255) / 256, splits);
    set_extents<LA, LB>(p);
    // default: reads retired after the barrier + grouped tile order (GM 4); A/B variants:
    // 15 = GM 4 (the non-fp32 default), 16 = both off (previous default), 17 = late reads +
    // row-major order (the fp32 default), 18 = GM 8
    using K = void (*)(GemmParams);
    static const K kfns[4] = {gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 4>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, false, 1>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 1>,
                              gemm_bf16_pp256_kernel<LA, LB, EPI, ACT, BG, true, 8>};
    // (the weight gradient -- XMAJ x XMAJ, 4 waves of tiles at 8192 wide -- measured 2-3 %
    // faster in row-major order: profiles/gemm_wide8192_pp256_variants.json)
    const int dflt = g_pp_order[EPI];
    // 19..24: the ring twin -- 10 slots / 8 slots, one half per phase; 10 / 8 slots, two
    // halves in each light phase; 6 slots, one / two (all GM 4)
    static const K rfns[6] = {gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 10, 0>,
                              gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 8, 0>,
                              gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 10, 1>,
                              gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 8, 1>,
                              gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 6, 0>,
                              gemm_bf16_pp256_ring_kernel<LA, LB, EPI, ACT, BG, 6, 1>};
    static bool attr = false;
    if (!attr) {
      for (K f : kfns)
        (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_SMEM);
      for (K f : rfns)
        (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_RING_SMEM);
      attr = true;
    }
    if (variant >= 19 && variant <= 24) {
      const int smem = variant >= 23 ? 6 * PP_HALF : (variant & 1) ? PP_RING_SMEM : PP_SMEM;
      hipLaunchKernelGGL(rfns[variant - 19], grid, dim3(PP_THREADS), smem, s, p);
      return hipGetLastError();
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

static int pick_tile(int M, int N) {
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

static int wgrad_tile(int M, int N) {
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
static int make_wgrad(const WgradArgs& a, GemmParams& p, SlabReduce& pending) {
  // dW[M=out][N=in] = sum_k dZ[k][m] X[k][n]; db[m] = sum_k dZ[k][m].
  const int M = a.M, N = a.N, K = a.K;
  const int splits = wgrad_splits(M, N, K);
  const int ksteps = (K + GEMM_BK - 1) / GEMM_BK;
  p = GemmParams{};
  p.sgd_serial = sgd_serial();
  p.A = a.dZ; p.lda = a.lddz; p.B = a.X; p.ldb = a.ldx; p.M = M; p.N = N; p.K = K;
  p.k_per_split = ((ksteps + splits - 1) / splits) * GEMM_BK;
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
  // ~8 independent loads per lane: WS = S / 8 rounded up to a power of two, in [1, 16]
  int ws = 1;
  while (ws < 16 && ws * 8 < r.S) ws *= 2;
  return ws;
}

static int slab_cols(int ws) { return ws >= SLAB_NW ? 64 : 64 * (SLAB_NW / ws); }

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
    default: hipLaunchKernelGGL(slab_reduce_kernel<16>, g, t, 0, s, r, nb_main, nb_bias); break;
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
    const char* e = getenv("NNMPI_GROUP");
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
  g.wg.store_pol = g_store_pol;
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

// ---- wide backward pairs (gemm_bf16_pp256_pair_kernel) ------------------------------------
// Off by default: measured on the 8192-wide step (3 interleaved rounds, one box) 5.575 ms
// paired vs 5.540 separate -- the SGD epilogue is bound per CU (latency), not by HBM, so
// spreading it beside other CUs' main loops buys nothing, and the interleaved tile orders cost
// L2 locality (profiles/r2s2_wide_sgd_epilogue_pair_ab.txt).
static int g_pair = -1;   // 1 on, 0 off (default; NNMPI_PAIR=1 / set_wide_pair)
void set_wide_pair(int on) { g_pair = on; }
static bool pair_enabled() {
  if (g_pair < 0) {
    const char* e = std::getenv("NNMPI_PAIR");
    g_pair = (e && e[0] == '1') ? 1 : 0;
  }
  return g_pair == 1 && gemm_impl() == 2 && g_force_tile == 0 && g_variant == 0;
}
static bool tiles256_x8(int M, int N) {
  const long long t = (long long)((M + 255) / 256) * ((N + 255) / 256);
  return t >= 256 && t % 8 == 0;
}
bool wide_pair_wgrad_ok(int rows, int out_f, int in_f) {
  return pair_enabled() && wgrad_tile(out_f, in_f) == 256 && tiles256_x8(out_f, in_f) &&
         wgrad_splits(out_f, in_f, rows) == 1;
}
bool wide_pair_dgrad_ok(int rows, int out_f, int in_f) {
  // dgrad output: rows x in_f
  return pair_enabled() && pick_tile(rows, in_f) == 256 && tiles256_x8(rows, in_f);
}

template <typename F>
static void pp_attr_once(F f) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, PP_SMEM);
    done = true;
  }
}

hipError_t wide_pair(const WgradArgs& w1, const DgradArgs* dg, const WgradArgs* w2, hipStream_t s) {
  if ((dg == nullptr) == (w2 == nullptr)) return hipErrorInvalidValue;
  if (!wide_pair_wgrad_ok(w1.K, w1.M, w1.N) || !w1.db) return hipErrorInvalidValue;
  GemmParams p1, p2;
  SlabReduce r1, r2;
  make_wgrad(w1, p1, r1);
  set_extents<XMAJ, XMAJ>(p1);
  const int gx1 = (w1.N + 255) / 256, gy1 = (w1.M + 255) / 256;
  int gx2, gy2;
  if (w2) {
    if (!wide_pair_wgrad_ok(w2->K, w2->M, w2->N) || !w2->db) return hipErrorInvalidValue;
    make_wgrad(*w2, p2, r2);
    set_extents<XMAJ, XMAJ>(p2);
    gx2 = (w2->N + 255) / 256; gy2 = (w2->M + 255) / 256;
  } else {
    // dZ[M rows][K out] x W[K out][N in] -> dX[M][N], times act'(Aprev)
    if (!wide_pair_dgrad_ok(dg->M, dg->K, dg->N)) return hipErrorInvalidValue;
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
