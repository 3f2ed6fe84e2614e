// Fused optimizer and elementwise kernels over the flat arena.
//
// sgd_momentum replaces torch.optim.SGD's per-tensor `_single_tensor_sgd` loop (ref.py:91,211;
// torch/optim/sgd.py) with ONE memory-bound pass over the whole arena: it folds the gradient
// average (1/P of the all-reduced SUM; ref.py:197's /nprocs), weight decay, momentum with
// dampening / Nesterov, the update of the fp32 master weights, the refresh of the bf16 compute
// shadow, and zeroes the gradient for the next step.  16-byte vector accesses, grid-stride.
// Hyper-parameters are read from device memory so a captured hipGraph picks up LR changes.
#include "common.h"
#include "kernels.h"
#include "knobs.h"

#include <algorithm>

namespace nnmpi {

template <typename TG>
__device__ __forceinline__ f32x4 load_grad4(TG* g, long long i) {
  if constexpr (sizeof(TG) == 2) {
    const bf16x4 v = reinterpret_cast<const bf16x4*>(g)[i];
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  } else {
    return reinterpret_cast<const f32x4*>(g)[i];
  }
}

// TG = bf16: the gradient is read straight from the bf16 all-reduce payload (the overlapped
// schedule's bf16 buckets: no cast back to fp32 and no fp32 gradient round trip; the fp32
// gradient arena is not touched -- every step rewrites it before reading it).
template <typename TG>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, TG* __restrict__ g,
                                                  float* __restrict__ buf, bf16* __restrict__ shadow,
                                                  long long n4, const float* __restrict__ hp,
                                                  int nesterov, int first, int zero_grad, SgdPack pk) {
  const float lr = hp[0], mom = hp[1], damp = hp[2], wd = hp[3], gs = hp[4];
  // (the momentum load is gated by kernel arguments only, not by the hyper-parameters in device
  // memory: gated by hp[1] it waited for that load's round trip before issuing -- two dependent
  // round trips per element.  sgd_elem reads buf only when mom != 0 and not first: same bits)
  const bool ldb = buf != nullptr && !first;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gv = load_grad4(g, i);
    f32x4 bv = ldb ? reinterpret_cast<f32x4*>(buf)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float bb = bv[r];
      pv[r] = sgd_elem(pv[r], gv[r], bb, lr, mom, damp, wd, gs, nesterov != 0, first != 0);
      bv[r] = bb;
    }
    if (mom != 0.f) reinterpret_cast<f32x4*>(buf)[i] = bv;
    reinterpret_cast<f32x4*>(p)[i] = pv;
    if (shadow) {
      bf16x4 s;
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = (bf16)pv[r];
      reinterpret_cast<bf16x4*>(shadow)[i] = s;
    }
    if constexpr (sizeof(TG) == 4) {
      if (zero_grad) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    for (int t = 0; t < pk.n; ++t) {   // row-band v2 weight images of the updated weights
      const long long loc = i * 4 - pk.start[t];
      if (loc >= 0 && loc < (long long)pk.M[t] * pk.N[t]) {
        const int m = (int)(loc / pk.N[t]), c = (int)(loc % pk.N[t]);
        rb_pack_store4(pk.pkf[t], pk.pkd[t], m, c, pk.M[t], pk.N[t], pv);
      }
    }
  }
}

// The optimizer pass that also refreshes the row-band v2 weight images (the multi-rank row-band
// step: its update follows the all-reduce, so the combines cannot apply it).  The matrices that
// have images are cut into 32 x 32 tiles, one per block: each thread updates one float4 of a row
// (master, momentum, bf16 shadow, the forward image's 8-byte piece) and parks the new bf16 values
// in LDS; the transposed image is then written as 16-byte pieces (8 rows of one column) -- where
// the element-wise pass above does one 64-bit division per float4 per matrix to place it and
// four scattered 2-byte stores for the transposed image.  Blocks past the tiles run the
// element-wise update over the rest of the range (biases, the head, padding).
struct SgdTileJob {
  int n;                               // matrices with images
  long long start[RB_MAXL_PK];         // element offset in the pass's range (% 4 == 0)
  int M[RB_MAXL_PK], N[RB_MAXL_PK];    // (% 32 == 0)
  bf16* pkf[RB_MAXL_PK];
  bf16* pkd[RB_MAXL_PK];
  int tx[RB_MAXL_PK], t0[RB_MAXL_PK + 1];   // tiles per row of tiles; first tile of matrix t
  long long ps[RB_MAXL_PK + 1], pe[RB_MAXL_PK + 1];   // the other float4 ranges [ps, pe)
  int np;
};

template <typename TG, int RT>
__global__ void __launch_bounds__(256) sgd_tiles_kernel(float* __restrict__ p, TG* __restrict__ g,
                                                        float* __restrict__ buf, bf16* __restrict__ shadow,
                                                        const float* __restrict__ hp, int nesterov,
                                                        int first, int zero_grad, SgdTileJob j) {
  // RT: 32-row groups per tile (a thread updates RT float4s, every load of the tile in flight
  // before the first update)
  const float lr = hp[0], mom = hp[1], damp = hp[2], wd = hp[3], gs = hp[4];
  // (momentum loads gated by kernel arguments only, as in sgd_kernel: no wait for hp[1])
  const bool useb = buf != nullptr && !first;
  auto apply = [&](long long i, f32x4 pv, f32x4 gv, f32x4 bv) -> f32x4 {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float bb = bv[r];
      pv[r] = sgd_elem(pv[r], gv[r], bb, lr, mom, damp, wd, gs, nesterov != 0, first != 0);
      bv[r] = bb;
    }
    if (mom != 0.f) reinterpret_cast<f32x4*>(buf)[i] = bv;
    reinterpret_cast<f32x4*>(p)[i] = pv;
    if (shadow) {
      bf16x4 sv;
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = (bf16)pv[r];
      reinterpret_cast<bf16x4*>(shadow)[i] = sv;
    }
    if constexpr (sizeof(TG) == 4) {
      if (zero_grad) reinterpret_cast<f32x4*>(g)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    return pv;
  };
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x;
  const int bid = blockIdx.x;
  if (bid >= j.t0[j.n]) {   // the element-wise rest, grid-stride over its blocks
    const long long nb = gridDim.x - j.t0[j.n];
    for (int q = 0; q < j.np; ++q)
      for (long long i = j.ps[q] + (long long)(bid - j.t0[j.n]) * 256 + tid; i < j.pe[q]; i += nb * 256)
        (void)apply(i, reinterpret_cast<f32x4*>(p)[i], load_grad4(g, i),
                    useb ? reinterpret_cast<f32x4*>(buf)[i] : z4);
    return;
  }
  int t = 0;
  while (t + 1 < j.n && bid >= j.t0[t + 1]) ++t;
  const int tile = bid - j.t0[t], M = j.M[t], N = j.N[t];
  const int m0 = (tile / j.tx[t]) * (32 * RT), n0 = (tile % j.tx[t]) * 32;
  const int r = tid >> 3, c4 = tid & 7, n = n0 + 4 * c4;
  __shared__ bf16 tb[32 * RT][32 + 8];   // (+8: the column reads below hit different banks)
  long long idx[RT];
  f32x4 pv[RT], gv[RT], bv[RT];
#pragma unroll
  for (int q = 0; q < RT; ++q) {
    idx[q] = (j.start[t] + (long long)(m0 + r + 32 * q) * N + n) / 4;
    pv[q] = reinterpret_cast<f32x4*>(p)[idx[q]];
    gv[q] = load_grad4(g, idx[q]);
    bv[q] = useb ? reinterpret_cast<f32x4*>(buf)[idx[q]] : z4;
  }
#pragma unroll
  for (int q = 0; q < RT; ++q) {
    const int m = m0 + r + 32 * q;
    const f32x4 nv = apply(idx[q], pv[q], gv[q], bv[q]);
    bf16x4 hv;
#pragma unroll
    for (int e = 0; e < 4; ++e) hv[e] = (bf16)nv[e];
    if (j.pkf[t]) *reinterpret_cast<bf16x4*>(j.pkf[t] + rb_pk_off(m, n, N)) = hv;
    if (j.pkd[t]) *reinterpret_cast<bf16x4*>(&tb[r + 32 * q][4 * c4]) = hv;
  }
  if (j.pkd[t]) {
    __syncthreads();
    if (tid < 128 * RT) {   // column c, rows m0 + 8 g8 .. + 7 -> one 16-byte piece of the W^T image
      const int c = tid & 31, g8 = tid >> 5;
      bf16x8 col;
#pragma unroll
      for (int e = 0; e < 8; ++e) col[e] = tb[8 * g8 + e][c];
      *reinterpret_cast<bf16x8*>(j.pkd[t] + rb_pk_off(n0 + c, m0 + 8 * g8, M)) = col;
    }
  }
}

// The tile job of a pass over n elements with the images of `pk` (false: a shape the tiles do not
// cover -- the element-wise kernel takes it).
static bool sgd_tile_job(const SgdPack& pk, long long n, SgdTileJob& j, int rt) {
  j = SgdTileJob{};
  j.n = pk.n;
  int tiles = 0;
  // matrices in arena order, each inside the range
  int ord[RB_MAXL_PK];
  for (int t = 0; t < pk.n; ++t) ord[t] = t;
  std::sort(ord, ord + pk.n, [&](int a, int b) { return pk.start[a] < pk.start[b]; });
  long long at = 0;
  for (int k = 0; k < pk.n; ++k) {
    const int t = ord[k];
    const long long s = pk.start[t], e = s + (long long)pk.M[t] * pk.N[t];
    if (s < at || e > n || pk.M[t] % (32 * rt) || pk.N[t] % 32 || s % 4) return false;
    j.start[k] = s; j.M[k] = pk.M[t]; j.N[k] = pk.N[t];
    j.pkf[k] = pk.pkf[t]; j.pkd[k] = pk.pkd[t];
    j.tx[k] = pk.N[t] / 32;
    j.t0[k] = tiles;
    tiles += (pk.M[t] / (32 * rt)) * (pk.N[t] / 32);
    if (s > at) { j.ps[j.np] = at / 4; j.pe[j.np] = s / 4; ++j.np; }
    at = e;
  }
  j.t0[pk.n] = tiles;
  if (at < n) { j.ps[j.np] = at / 4; j.pe[j.np] = n / 4; ++j.np; }
  return true;
}

template <typename TG>
static hipError_t sgd_tiles_launch(float* p, TG* g, float* buf, bf16* shadow, long long n,
                                   const float* hp, int nesterov, int first, int zero_grad,
                                   const SgdTileJob& j, int rt, hipStream_t s) {
  long long rest = 0;
  for (int q = 0; q < j.np; ++q) rest += j.pe[q] - j.ps[q];
  const int nb_rest = rest > 0 ? (int)std::min<long long>((rest + 255) / 256, 64) : 0;
  auto* f = rt == 2 ? sgd_tiles_kernel<TG, 2> : sgd_tiles_kernel<TG, 1>;
  hipLaunchKernelGGL(f, dim3(j.t0[j.n] + nb_rest), dim3(256), 0, s, p, g, buf, shadow, hp, nesterov,
                     first, zero_grad, j);
  return hipGetLastError();
}

// 32-row groups per tile (NNMPI_SGD_TILE_RT=1 / 2, experiments): one per thread measured 6.16 vs
// 6.39 us with two at 3.15 M parameters (profiles/r6_wgrad_small_ksplit_ab.txt)
static int sgd_tile_rt() {
  static const int v = [] {
    const char* e = knob_env("NNMPI_SGD_TILE_RT");
    return (e && e[0] == '2') ? 2 : 1;
  }();
  return v;
}

static int g_sgd_tiles = -1;   // NNMPI_SGD_TILES=0: the element-wise image refresh (A/B)
void set_sgd_tiles(int v) { g_sgd_tiles = v; }   // -1: re-read the knob
static bool sgd_tiles_on() {
  if (g_sgd_tiles < 0) {
    const char* e = knob_env("NNMPI_SGD_TILES");
    g_sgd_tiles = (e && e[0] == '0') ? 0 : 1;
  }
  return g_sgd_tiles == 1;
}

static int grid_for(long long n, int per_thread = 1) {
  const long long b = (n / per_thread + 255) / 256;
  return (int)std::max<long long>(1, std::min<long long>(b, 2048));
}

static bool pack_ok(const SgdPack* pk) {
  if (!pk) return true;
  if (pk->n < 0 || pk->n > RB_MAXL_PK) return false;
  for (int t = 0; t < pk->n; ++t)   // whole float4 groups inside one matrix row, 16x32 tiles
    if (pk->start[t] % 4 || pk->N[t] % 32 || pk->M[t] % 32) return false;
  return true;
}

hipError_t sgd_momentum(float* p, float* g, float* buf, bf16* shadow, long long n,
                        const float* hp, int nesterov, int first, int zero_grad, hipStream_t s,
                        const SgdPack* pack) {
  if (n % 4 != 0 || !pack_ok(pack)) return hipErrorInvalidValue;
  const SgdPack pk = pack ? *pack : SgdPack{};
  SgdTileJob j;
  int rt = sgd_tile_rt();
  if (pk.n > 0 && sgd_tiles_on() && (sgd_tile_job(pk, n, j, rt) || sgd_tile_job(pk, n, j, rt = 1)))
    return sgd_tiles_launch<float>(p, g, buf, shadow, n, hp, nesterov, first, zero_grad, j, rt, s);
  hipLaunchKernelGGL(sgd_kernel<float>, dim3(grid_for(n / 4)), dim3(256), 0, s, p, g, buf, shadow,
                     n / 4, hp, nesterov, first, zero_grad, pk);
  return hipGetLastError();
}

// The same update as a "background" launch: a fixed grid of `blocks` grid-stride blocks (one
// 4-wave block per CU at 256), so that it can run beside a 2-waves-per-SIMD GEMM whose
// blocks leave 64 VGPRs per SIMD free, instead of queueing behind / in front of it.
hipError_t sgd_momentum_bg(float* p, float* g, float* buf, bf16* shadow, long long n,
                           const float* hp, int nesterov, int first, int zero_grad, int blocks,
                           hipStream_t s) {
  if (n % 4 != 0 || blocks < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sgd_kernel<float>, dim3(blocks), dim3(256), 0, s, p, g, buf, shadow, n / 4,
                     hp, nesterov, first, zero_grad, SgdPack{});
  return hipGetLastError();
}

hipError_t sgd_momentum_bf16grad(float* p, const bf16* g, float* buf, bf16* shadow, long long n,
                                 const float* hp, int nesterov, int first, hipStream_t s,
                                 const SgdPack* pack) {
  if (n % 4 != 0 || !pack_ok(pack)) return hipErrorInvalidValue;
  const SgdPack pk = pack ? *pack : SgdPack{};
  SgdTileJob j;
  int rt = sgd_tile_rt();
  if (pk.n > 0 && sgd_tiles_on() && (sgd_tile_job(pk, n, j, rt) || sgd_tile_job(pk, n, j, rt = 1)))
    return sgd_tiles_launch<const bf16>(p, g, buf, shadow, n, hp, nesterov, first, 0, j, rt, s);
  hipLaunchKernelGGL(sgd_kernel<const bf16>, dim3(grid_for(n / 4)), dim3(256), 0, s, p, g, buf,
                     shadow, n / 4, hp, nesterov, first, 0, pk);
  return hipGetLastError();
}

// Casts: 4 elements per lane per iteration (16-B fp32 / 8-B bf16 accesses) when both pointers
// are 16/8-byte aligned, scalar otherwise and for the tail.
__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((((uintptr_t)x) & 15) == 0) && ((((uintptr_t)y) & 7) == 0);
  const long long nv = vec ? n / 4 : 0;
  for (long long i = t0; i < nv; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    bf16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (bf16)v[r];
    reinterpret_cast<bf16x4*>(y)[i] = o;
  }
  for (long long i = nv * 4 + t0; i < n; i += stride) y[i] = (bf16)x[i];
}

__global__ void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = ((((uintptr_t)x) & 7) == 0) && ((((uintptr_t)y) & 15) == 0);
  const long long nv = vec ? n / 4 : 0;
  for (long long i = t0; i < nv; i += stride) {
    const bf16x4 v = reinterpret_cast<const bf16x4*>(x)[i];
    f32x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = (float)v[r];
    reinterpret_cast<f32x4*>(y)[i] = o;
  }
  for (long long i = nv * 4 + t0; i < n; i += stride) y[i] = (float)x[i];
}

__global__ void scale_kernel(float* __restrict__ x, long long n, float a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= a;
}

// Order-fixed fp64 checksum (replica-consistency check): per-block partial sums in LDS, then a
// single block combines them in block order.
__global__ void checksum_kernel(const float* __restrict__ x, long long n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    s += (double)x[i] * (double)((i % 7) + 1);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void checksum_final(double* part, int nb, double* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < nb; ++i) s += part[i];
    *out = s;
  }
}

hipError_t cast_f32_bf16(const float* x, bf16* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t cast_bf16_f32(const bf16* x, float* y, long long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t scale_f32(float* x, long long n, float a, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, n, a);
  return hipGetLastError();
}

// out must hold 65 doubles (64 partials + the result at out[64]).
hipError_t checksum_f32(const float* x, long long n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(checksum_kernel, dim3(64), dim3(256), 0, s, x, n, out);
  hipLaunchKernelGGL(checksum_final, dim3(1), dim3(64), 0, s, out, 64, out + 64);
  return hipGetLastError();
}

// Owner step of the one-rounding bf16 all-reduce (rccl_comm.cpp): P bf16 copies of a slice,
// summed in fp32 in rank order (the same order on every owner, so the result is a pure function
// of the inputs), rounded once.  8 elements (16 B) per lane when the slice allows it.
__global__ void __launch_bounds__(256) sum_slices_bf16_kernel(bf16* __restrict__ out,
                                                              const bf16* __restrict__ sc, int P,
                                                              int me, long long stride,
                                                              long long n) {
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long step = (long long)gridDim.x * blockDim.x;
  const bool vec = ((((uintptr_t)out) | ((uintptr_t)sc)) & 15) == 0 && (stride % 8) == 0;
  const long long n8 = vec ? n / 8 : 0;
  for (long long i = t0; i < n8; i += step) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int q = 0; q < P; ++q) {
      const bf16* src = (q == me) ? out : sc + (long long)q * stride;
      const uint4 w = reinterpret_cast<const uint4*>(src)[i];
      const unsigned ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += __uint_as_float(ws[e] << 16);
        acc[2 * e + 1] += __uint_as_float(ws[e] & 0xffff0000u);
      }
    }
    bf16x4 lo, hi;
#pragma unroll
    for (int e = 0; e < 4; ++e) { lo[e] = (bf16)acc[e]; hi[e] = (bf16)acc[4 + e]; }
    reinterpret_cast<bf16x4*>(out)[2 * i] = lo;
    reinterpret_cast<bf16x4*>(out)[2 * i + 1] = hi;
  }
  for (long long j = n8 * 8 + t0; j < n; j += step) {
    float acc = 0.f;
    for (int q = 0; q < P; ++q) acc += (float)((q == me) ? out[j] : sc[(long long)q * stride + j]);
    out[j] = (bf16)acc;
  }
}

hipError_t sum_slices_bf16(bf16* out, const bf16* scratch, int P, int me, long long stride,
                           long long n, hipStream_t s) {
  if (P < 1 || me < 0 || me >= P || n < 0 || stride < n) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sum_slices_bf16_kernel, dim3(grid_for((n + 7) / 8)), dim3(256), 0, s, out,
                     scratch, P, me, stride, n);
  return hipGetLastError();
}

// Owner step of the ordered fp32 all-reduce (rccl_comm.cpp allreduce_f32_ordered): the P fp32
// copies of a slice summed in rank order, so an element's sum does not depend on where it sits
// in the buffer (a ring's order does: at P >= 3 two bucketings of one gradient differ in bits).
__global__ void __launch_bounds__(256) sum_slices_f32_kernel(float* __restrict__ out,
                                                             const float* __restrict__ sc, int P,
                                                             int me, long long stride, long long n) {
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long step = (long long)gridDim.x * blockDim.x;
  const bool vec = ((((uintptr_t)out) | ((uintptr_t)sc)) & 15) == 0 && (stride % 4) == 0;
  const long long n4 = vec ? n / 4 : 0;
  for (long long i = t0; i < n4; i += step) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < P; ++q) {
      const float* src = (q == me) ? out : sc + (long long)q * stride;
      acc += reinterpret_cast<const f32x4*>(src)[i];
    }
    reinterpret_cast<f32x4*>(out)[i] = acc;
  }
  for (long long j = n4 * 4 + t0; j < n; j += step) {
    float acc = 0.f;
    for (int q = 0; q < P; ++q) acc += (q == me) ? out[j] : sc[(long long)q * stride + j];
    out[j] = acc;
  }
}

hipError_t sum_slices_f32(float* out, const float* scratch, int P, int me, long long stride,
                          long long n, hipStream_t s) {
  if (P < 1 || me < 0 || me >= P || n < 0 || stride < n) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sum_slices_f32_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, out,
                     scratch, P, me, stride, n);
  return hipGetLastError();
}

// Bitwise replica hash: sum over i of mix64((i << 32) | word_i) mod 2^64 (splitmix64 finaliser).
// A value sum (checksum_f32) can coincide for different bits (-0.0 vs 0.0, compensating
// errors); this one changes with any flipped bit of any word, and integer addition makes the
// result independent of the reduction order.  HASH_BLOCKS partials, then one block sums them.
constexpr int HASH_BLOCKS = 1024;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) hash_u32_kernel(const unsigned* __restrict__ x, long long n,
                                                       unsigned long long* __restrict__ part) {
  __shared__ unsigned long long red[256];
  unsigned long long h = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  // 16-byte loads, two in flight per lane (the callers' buffers are 16-byte aligned), then the
  // scalar tail
  const bool vec = (((uintptr_t)x) & 15) == 0;
  const long long n4 = vec ? n / 4 : 0;
  long long q = t0;
  for (; q + stride < n4; q += 2 * stride) {
    const uint4 a = reinterpret_cast<const uint4*>(x)[q];
    const uint4 b = reinterpret_cast<const uint4*>(x)[q + stride];
    const unsigned long long i = (unsigned long long)(4 * q), j = (unsigned long long)(4 * (q + stride));
    h += mix64((i << 32) | a.x) + mix64(((i + 1) << 32) | a.y) + mix64(((i + 2) << 32) | a.z) +
         mix64(((i + 3) << 32) | a.w);
    h += mix64((j << 32) | b.x) + mix64(((j + 1) << 32) | b.y) + mix64(((j + 2) << 32) | b.z) +
         mix64(((j + 3) << 32) | b.w);
  }
  for (; q < n4; q += stride) {
    const uint4 a = reinterpret_cast<const uint4*>(x)[q];
    const unsigned long long i = (unsigned long long)(4 * q);
    h += mix64((i << 32) | a.x) + mix64(((i + 1) << 32) | a.y) + mix64(((i + 2) << 32) | a.z) +
         mix64(((i + 3) << 32) | a.w);
  }
  for (long long i = n4 * 4 + t0; i < n; i += stride)
    h += mix64(((unsigned long long)i << 32) | x[i]);
  red[threadIdx.x] = h;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) hash_final_kernel(const unsigned long long* __restrict__ part,
                                                         unsigned long long* __restrict__ out) {
  __shared__ unsigned long long red[256];
  unsigned long long h = 0;
  for (int i = threadIdx.x; i < HASH_BLOCKS; i += 256) h += part[i];
  red[threadIdx.x] = h;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

// out must hold HASH_BLOCKS + 1 = 1025 uint64 (partials + the result at out[HASH_BLOCKS]).
hipError_t hash_u32(const unsigned* x, long long n, unsigned long long* out, hipStream_t s) {
  if (n < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(hash_u32_kernel, dim3(HASH_BLOCKS), dim3(256), 0, s, x, n, out);
  hipLaunchKernelGGL(hash_final_kernel, dim3(1), dim3(256), 0, s, out, out + HASH_BLOCKS);
  return hipGetLastError();
}

}  // namespace nnmpi
