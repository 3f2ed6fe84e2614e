// Device-side building blocks of the bf16 MFMA GEMMs (gemm_bf16.hip): operand layouts, LDS
// images, the LDS-DMA plan, the 128x128 DMA main loop and the 256x256 ping-pong tile with their
// fused epilogues.  Shared by the production launchers (gemm_bf16.hip) and the experiment
// kernels (csrc/experiments/, built only with NNMPI_BUILD_EXPERIMENTS=1).  See gemm_bf16.hip for the
// design notes.
#pragma once
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
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n s_nop 1" ::"v"(ptr), "v"(d) : "memory");
  } else {
    *ptr = v;
  }
}

// 16-byte write-through store / L1-bypassing load (in-launch hand-offs -- wgrad_multi's split-K fixup, the column-split row-band kernel:
// MI355X_MICROARCH.md "Valid forms", row 1 -- every store and every load of the handed-off slab
// bytes is sc1, each storing wave drains vmcnt before the workgroup barrier, one lane's
// agent-scope atomic add signals, the workgroup whose add returned S - 1 reads)
// (an asm store of more than 8 bytes ends with s_nop 1: the data registers may otherwise be
// overwritten by the next VALU before the store has read them -- cdna_hip_programming.md, the
// inline-asm store rule; without it the column-split row-band kernel stored garbage into the first
// element of some 16-byte pieces)
__device__ __forceinline__ void st_sc1(float* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n s_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1_f(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4 ld_sc1(const float* p) {
  f32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ float ld_sc1_f(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ __forceinline__ void st_sc1_b8(void* p, uint2 v) {   // 8 bytes (4 bf16)
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ bf16x8 ld_sc1_b16(const void* p) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// (a poll: the value is waited for)
__device__ __forceinline__ int ld_sc1_i(const int* p) {
  int v;
  asm volatile("global_load_dword %0, %1, off sc1\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// s_waitcnt with only the vector-memory counter constrained (lgkm/exp counters left free).
__device__ __forceinline__ constexpr int waitcnt_vm(int n) {
  return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8);
}

template <int N>
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(waitcnt_vm(N)); }

// Retire a ring stage while min(newer, MAXN) newer stages (PT vector-memory ops each) stay in
// flight (deep DMA rings, NS > 4).
template <int PT, int MAXN>
__device__ __forceinline__ void wait_vm_newer(int newer) {
  if constexpr (MAXN > 0) {
    if (newer >= MAXN) {
      wait_vm<MAXN * PT>();
      return;
    }
    wait_vm_newer<PT, MAXN - 1>(newer);
  } else {
    wait_vm<0>();
  }
}

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
// KST (diagnostic, scripts/r5_wg_stamps.py): per k-step shader-clock stamps of wave 0 into kst
// [4 t] ring wait done, [4 t + 1] barrier passed, [4 t + 2] DMA refill issued, [4 t + 3] MFMAs
// issued (t < 32)
// RET: no epilogue -- the accumulators go to acc_out[MI * NJ] / accb_out[MI] (row-major over
// (i, j)) for a caller-side epilogue (wgrad_multi's in-launch split-K fixup)
template <int BM, int BN, int WGM, int WGN, int LA, int LB, int EPI, int ACT, bool BIASGRAD, int NS,
          int ASYNC_TR = 1, bool KST = false, bool RET = false>
__device__ __forceinline__ void dma_gemm_tile(const GemmParams& p, char* smem, int tx, int ty,
                                              int split, unsigned long long* kst = nullptr,
                                              f32x4* acc_out = nullptr, f32x4* accb_out = nullptr) {
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
    if constexpr (NS >= 5) {
      wait_vm_newer<PER_TILE, NS - 2>(newer);
    } else if constexpr (NS >= 4) {
      if (newer >= 2) wait_vm<2 * PER_TILE>();
      else if (newer == 1) wait_vm<PER_TILE>();
      else wait_vm<0>();
    } else if constexpr (NS == 3) {
      if (newer >= 1) wait_vm<PER_TILE>();
      else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    if constexpr (KST) {
      if (tid == 0 && t < 32) kst[4 * t] = __builtin_amdgcn_s_memtime();
    }
    __builtin_amdgcn_s_barrier();
    if constexpr (KST) {
      if (tid == 0 && t < 32) kst[4 * t + 1] = __builtin_amdgcn_s_memtime();
    }
    // refill the stage consumed in iteration t-1 (all waves are past its reads); ASYNC_TR 4
    // issues it between the k-halves' MFMAs below instead
    if (ASYNC_TR != 4 && t + NS - 1 < nt) {
      char* st = smem + ((t + NS - 1) % NS) * STAGE;
      da.issue(rsA, st, w, kbeg + (t + NS - 1) * BK, kend);
      db.issue(rsB, st + A_BYTES, w, kbeg + (t + NS - 1) * BK, kend);
    }
    if constexpr (KST) {
      if (tid == 0 && t < 32) kst[4 * t + 2] = __builtin_amdgcn_s_memtime();
    }
    const char* cur = smem + (t % NS) * STAGE;
    constexpr bool TR = (LA == XMAJ || LB == XMAJ);
    if constexpr (ASYNC_TR == 4 && TR && BK == 64) {
      // as 3, and the refill's DMA pieces go out between the k-halves' MFMAs: every wave's
      // pieces pass the CU's address unit (64 B/clk: 512 cycles per 32 KiB stage), so issued
      // together after the barrier they stalled each wave ~400 cycles before its first MFMA
      // (profiles/r5_wgrad_kstep_stamps.txt); here the matrix pipe runs meanwhile
      constexpr int NR = 2 * (MI + NJ);
      static_assert(NR <= 15, "lgkmcnt counts at most 15 outstanding LDS reads");
      const bool refill = t + NS - 1 < nt;
      char* rst = smem + ((t + NS - 1) % NS) * STAGE;
      bf16x8 af[2][MI], bfr[2][NJ];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[kk][i] = read_frag_async<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[kk][j] = read_frag_async<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (refill) {
          if (kk == 0) da.issue(rsA, rst, w, kbeg + (t + NS - 1) * BK, kend);
          else db.issue(rsB, rst + A_BYTES, w, kbeg + (t + NS - 1) * BK, kend);
        }
        if (kk == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NR) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(af[kk][i]));
#pragma unroll
        for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(bfr[kk][j]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
        if constexpr (BIASGRAD) {
          if (do_bg) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
              accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[kk][i], accb[i], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (ASYNC_TR == 3 && TR && BK == 64) {
      // both k-halves' fragments issued up front; the first half's MFMAs run while the second
      // half's reads are still in flight (counted lgkmcnt), so a wave's LDS latency overlaps its
      // own matrix work instead of the SIMD partner's alone.  (Per k-step stamps of the grouped
      // weight gradient under ASYNC_TR 2: reads + wait + MFMAs 1,444 cycles for 16 + 8 MFMAs,
      // profiles/r5_wgrad_kstep_stamps.txt.)  Needs the fragment registers of both halves:
      // 2 x (MI + NJ) x 4 VGPRs.
      constexpr int NR = 2 * (MI + NJ);   // asm LDS reads per k-half (tr reads: 2 per fragment)
      static_assert(NR <= 15, "lgkmcnt counts at most 15 outstanding LDS reads");
      bf16x8 af[2][MI], bfr[2][NJ];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < MI; ++i) af[kk][i] = read_frag_async<BM, LA>(cur, wm * WM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) bfr[kk][j] = read_frag_async<BN, LB>(cur + A_BYTES, wn * WN + j * 16, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (kk == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NR) : "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < MI; ++i) asm volatile("" : "+v"(af[kk][i]));
#pragma unroll
        for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(bfr[kk][j]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
        if constexpr (BIASGRAD) {
          if (do_bg) {
#pragma unroll
            for (int i = 0; i < MI; ++i)
              accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[kk][i], accb[i], 0, 0, 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (ASYNC_TR == 2 && TR) {
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
    if constexpr (KST) {
      if (tid == 0 && t < 32) kst[4 * t + 3] = __builtin_amdgcn_s_memtime();
    }
    // all of this wave's LDS reads of stage t are consumed before the next barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if constexpr (RET) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc_out[i * NJ + j] = acc[i][j];
      accb_out[i] = accb[i];
    }
    return;
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
// ISSUE: DMA placement over the four phases.  0: halves 1 / 0 / 2 / 1 (A1(t+1) | - | A0(t+2),
// B0(t+2) | B1(t+2)); 1: one half per phase (B0(t+2) moves to P2: its buffer was last read in
// P4 of the previous K-tile, the same two-phase WAR margin as A0's), so no memory section
// carries four DMA instructions beside eight fragment reads.
// PF (weight gradient with the fused SGD update, ISSUE 0 only): the update's master and
// momentum rows are pulled toward the chip DURING the main loop -- one LDS-DMA instruction per
// wave per K-tile, 4 bytes per lane from one 64-byte granule each, landing in a 256-byte dummy
// slot per wave behind the ring (PP_PF_SMEM) -- so the epilogue, which otherwise has every CU
// read 512 KiB from HBM at the same moment (measured HBM-bound: scripts/r4_wgrad_sgd_ab.py),
// finds them in the memory-side cache.  PF 1 default policy, PF 2 `nt`.  The prefetch is one more
// vector-memory op per K-tile, so the counted waits of P1..P3 allow one (two) more.
constexpr int PP_PF_SMEM = 128 * 1024 + 8 * 256;
template <int LA, int LB, int EPI, int ACT, bool BIASGRAD, bool LATE_LGKM = true, int GM = 4,
          int ISSUE = 0, int PF = 0>
__device__ __forceinline__ void pp256_tile(const GemmParams& p, char* smem, int bid, int gx, int gy,
                                           int split) {
  static_assert(PF == 0 || (ISSUE == 0 && EPI == EPI_F32), "prefetch: wgrad + SGD, issue order 0");
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

  // prefetch plan (PF): granule g of 4096 per array (256 rows x 16 x 64 B), K-tile t serves
  // array t & 1, granules ((t >> 1) * 8 + w) * pf_lpw + lane, spread to finish ~4 K-tiles early
  __amdgpu_buffer_rsrc_t rsP = rsA, rsM = rsA;
  bool pf_on = false;
  int pf_lpw = 0;
  if constexpr (PF > 0) {
    pf_on = p.sg.g_base && !p.c16 && p.sgd_serial == 0 && m0 + 256 <= p.M && n0 + 256 <= p.N;
    if (pf_on) {
      const long long o = (reinterpret_cast<const float*>(p.C) + split * p.c_split_stride - p.sg.g_base) +
                          (long long)m0 * p.ldc + n0;
      const int bytes = (255 * p.ldc + 256) * 4;
      rsP = __builtin_amdgcn_make_buffer_rsrc((void*)(p.sg.p_base + o), (short)0, bytes, 0x00020000);
      rsM = __builtin_amdgcn_make_buffer_rsrc((void*)(p.sg.m_base + o), (short)0, bytes, 0x00020000);
    }
    const int span = max(nt - 4, 2) / 2;   // K-tiles per array
    pf_lpw = min(64, (4096 / 8 + span - 1) / span);
  }
  auto prefetch = [&](int t) {
    if constexpr (PF > 0) {
      const int g = ((t >> 1) * 8 + w) * pf_lpw + lane;
      const bool ok = pf_on && t >= 0 && lane < pf_lpw && g < 4096;
      const unsigned v = ok ? (unsigned)((g >> 4) * p.ldc * 4 + (g & 15) * 64) : DMA_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds((t & 1) ? rsM : rsP,
          (__attribute__((address_space(3))) void*)(smem + 128 * 1024 + w * 256), 4, v, 0, 0,
          PF == 2 ? 2 : 0);
    }
  };

  // prologue: K-tile 0 whole, K-tile 1's A0, B0, B1 (the steady-state issue order); retire
  // K-tile 0's A0 + B0 (five newer halves may stay in flight)
  pa0.issue(rsA, A0(0), w, kof(0), kend);
  pb0.issue(rsB, B0(0), w, kof(0), kend);
  pb1.issue(rsB, B1(0), w, kof(0), kend);
  prefetch(-1);   // (PF: the slot K-tile -1 would have used; no traffic)
  pa1.issue(rsA, A1(0), w, kof(0), kend);
  if constexpr (ISSUE == 1) {   // the steady-state order of K-tile "-1": B0, A0, B1
    pb0.issue(rsB, B0(1), w, kof(1), kend);
    pa0.issue(rsA, A0(1), w, kof(1), kend);
  } else {
    pa0.issue(rsA, A0(1), w, kof(1), kend);
    pb0.issue(rsB, B0(1), w, kof(1), kend);
  }
  pb1.issue(rsB, B1(1), w, kof(1), kend);
  wait_vm<PF ? 11 : 10>();
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
      // P2 -> A1(t) [8], P3 -> A0 + B0 (t+1) [8] (read in P4 and in the next P1).
      // ISSUE 1: P1 A1(t+1) | P2 B0(t+2) | P3 A0(t+2) | P4 B1(t+2); retire: P1 -> B1(t) [10],
      // P2 -> A1(t) [10], P3 -> B0 + A0 (t+1) [8]
      // PF: prefetch(t) sits in front of A1(t+1); newer than the retired half: P1 two
      // prefetches (t-1, t), P2 and P3 one (t)
      if (ph == 0) {
        prefetch(t);
        pa1.issue(rsA, A1(nb), w, kof(t + 1), kend);
        wait_vm<PF ? 12 : 10>();
      } else if (ph == 1) {
        if constexpr (ISSUE == 1) {
          pb0.issue(rsB, B0(b), w, kof(t + 2), kend);
          wait_vm<10>();
        } else {
          wait_vm<PF ? 9 : 8>();
        }
      } else if (ph == 2) {
        pa0.issue(rsA, A0(b), w, kof(t + 2), kend);
        if constexpr (ISSUE == 0) pb0.issue(rsB, B0(b), w, kof(t + 2), kend);
        wait_vm<PF ? 9 : 8>();
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

template <int LA, int LB, int EPI, int ACT, bool BIASGRAD, bool LATE_LGKM = true, int GM = 4,
          int ISSUE = 0, int PF = 0>
__global__ void __launch_bounds__(PP_THREADS) gemm_bf16_pp256_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int gx = gridDim.x, gy = gridDim.y;
  pp256_tile<LA, LB, EPI, ACT, BIASGRAD, LATE_LGKM, GM, ISSUE, PF>(
      p, smem, xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gy), gx, gy, blockIdx.z);
}

// ---- experiment kernels (csrc/experiments/gemm_experiments.hip) ------------------------------
// Built into the library only with NNMPI_EXPERIMENTS=1 (_build.py); weak references here, so a
// production build links without them and every entry point below is a null pointer.
// variant 19..24: the deep-ring twin of the 256x256 kernel (docs/PERF.md §4)
__attribute__((weak)) hipError_t exp_pp256_ring(int variant, int la, int lb, int epi, int act,
                                                int bg, GemmParams p, dim3 grid, hipStream_t s);
// gemm_bf16_pp256_pair_kernel (off by default even when built: NNMPI_PAIR=1)
__attribute__((weak)) void exp_set_wide_pair(int on);
__attribute__((weak)) bool exp_wide_pair_wgrad_ok(int rows, int out_f, int in_f);
__attribute__((weak)) bool exp_wide_pair_dgrad_ok(int rows, int out_f, int in_f);
__attribute__((weak)) hipError_t exp_wide_pair(const WgradArgs& w1, const DgradArgs* dg,
                                               const WgradArgs* w2, hipStream_t s);
__attribute__((weak)) hipError_t exp_fwd_stamped(const bf16* X, int ldx, const bf16* W, int ldw,
                                                 const float* bias, bf16* Y, int ldy, int M, int N,
                                                 int K, unsigned long long* stamps, hipStream_t s);

// ---- host helpers shared with csrc/experiments (defined in gemm_bf16.hip) ----
namespace gemm_host {
// the weight-gradient GEMM of a WgradArgs and its pending split-K combine (returns the splits)
int make_wgrad(const WgradArgs& a, GemmParams& p, SlabReduce& pending);
int pick_tile(int M, int N);
int wgrad_tile(int M, int N);
// the production kernel selection is in effect (LDS-DMA path, no forced tile or variant)
bool default_path();
}  // namespace gemm_host

template <int LA, int LB>
static inline void set_extents(GemmParams& p) {
  // storage extents (bytes) of the operands, for the buffer-resource range checks
  const long long a = (LA == KMAJ) ? ((long long)(p.M - 1) * p.lda + p.K) : ((long long)(p.K - 1) * p.lda + p.M);
  const long long b = (LB == KMAJ) ? ((long long)(p.N - 1) * p.ldb + p.K) : ((long long)(p.K - 1) * p.ldb + p.N);
  p.a_bytes = (unsigned)std::min<long long>(a * 2, DMA_OOB - 16);
  p.b_bytes = (unsigned)std::min<long long>(b * 2, DMA_OOB - 16);
}

}  // namespace nnmpi
