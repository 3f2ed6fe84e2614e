// Host-side launch API of the gfx950 kernels (all launches are asynchronous on `stream`, make
// no allocation and no host synchronisation, so every one of them is hipGraph-capturable).
#pragma once
#include "knobs.h"
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace nnmpi {

typedef __bf16 bf16;

constexpr int RB_MAXL_PK = 4;   // == RB_MAXL (row-band hidden layers), see below

// Optional optimizer fusion for kernels that produce final (already reduced) gradients: the
// parameter / momentum / bf16-shadow arrays share the gradient arena's layout, so an element's
// position is found from its offset to g_base.  g_base == nullptr disables the fusion.
struct SgdFuse {
  const float* g_base;
  float* p_base;
  float* m_base;
  bf16* s_base;
  const float* hp;   // {lr, momentum, dampening, weight_decay, grad_scale}
  int nesterov;
  int first;
};

// A split-K / partial-slab combine (see slab_reduce in gemm_bf16.hip), described so that its
// launch can be deferred and merged into a later grouped launch (bwd_group).
struct SlabReduce {
  const float* ws;          // S slabs of M x N (stride elements apart); null = none
  int S;
  long long stride;
  int M, N;
  float* out;
  int ldo;
  const float* bws;         // S slabs of M bias partials (bstride apart); null = none
  long long bstride;
  float* bout;
  const float* loss_part;   // loss partials (null = none)
  int n_loss_part;
  float loss_scale;
  float* loss_out;
  SgdFuse sg;               // sg.g_base != null: apply the optimizer update instead of storing
  int sgd_serial = 0;       // 1: optimizer operands loaded after the sums (A/B, NNMPI_SGD_SERIAL)
  // with sg: also write the updated [M][N] matrix into its fragment-major image (pkf) and that
  // of its transpose (pkd) -- the row-band v2 weight images (rowband.hip); null = none
  bf16* pkf = nullptr;
  bf16* pkd = nullptr;
};

enum Epi : int { EPI_BIAS_ACT = 0, EPI_DACT = 1, EPI_F32 = 2 };
enum Loss : int { LOSS_MSE = 0, LOSS_XENT = 1 };

// ---- GEMM (gemm_bf16.hip) ----
hipError_t linear_fwd_bf16(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                           bf16* Y, int ldy, int M, int N, int K, int act, hipStream_t s);
// experiment (csrc/experiments/gemm_w4.hip, NNMPI_BUILD_EXPERIMENTS=1 builds only; a weak
// reference, null otherwise): the forward on a 4-wave 256 x 256 tile (M, N % 256, K % 64)
__attribute__((weak)) hipError_t gemm_w4_fwd(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias, bf16* Y,
                       int ldy, int M, int N, int K, int act, hipStream_t s);
hipError_t linear_dgrad_bf16(const bf16* dZ, int lddz, const bf16* W, int ldw, const bf16* Aprev,
                             int lda_prev, bf16* dX, int lddx, int M, int N, int K, int act,
                             hipStream_t s);
int wgrad_splits(int M, int N, int K);
void set_gemm_impl(int impl);  // 1 = register-staged main loop, 2 = LDS-DMA ring
int get_gemm_impl();
void set_gemm_tile(int t);     // 0 = heuristic, 64 / 128 = force (experiments)
void set_gemm_variant(int v);  // DMA-path main-loop variant (experiments), 0 = default
// step-level kernel-selection knobs (-1 / 0 = built-in default; scripts/step_ab.py)
void set_fwd_variant(int v);   // forward GEMM (128x128 tiles) main-loop variant
void set_pp_prefetch(int v);            // SGD-operand prefetch in the 256x256 wgrad (0 / 1 / 2)
void set_pp256_order(int epi, int idx);   // 256x256 kernel tile order per epilogue (A/B)
void set_store_policy(int p);
void set_slab_store_policy(int p);   // split-K slab stores of the grouped backward (-2: env)  // LDS-epilogue output stores: 0 plain, 1 nt, 2 sc1 (experiments)
void set_head_xcd_rows(int v);  // head kernels: rows of XCD-remapped logical blocks (experiment)
// diagnostic (experiments library): the default 128x128 forward kernel with per-block
// entry/exit real-time stamps (stamps: 2 * grid uint64, 100 MHz counter)
hipError_t linear_fwd_bf16_stamped(const bf16* X, int ldx, const bf16* W, int ldw, const float* bias,
                                   bf16* Y, int ldy, int M, int N, int K, unsigned long long* stamps,
                                   hipStream_t s);
void set_group_async(int m);   // grouped backward LDS read mode: 0 compiler, 1 stage, 2 k-half
void set_wgrad_splits(int s);  // upper bound on the weight-gradient split-K factor
size_t wgrad_workspace_bytes(int M, int N, int K);
hipError_t linear_wgrad_bf16(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                             float* db, int M, int N, int K, float* ws, hipStream_t s,
                             const SgdFuse* sgd = nullptr);
hipError_t gemm_bf16_generic(const bf16* A, int lda, int la, const bf16* B, int ldb, int lb,
                             int M, int N, int K, float* C, int ldc, hipStream_t s);
hipError_t gemm_bf16_generic_tile(const bf16* A, int lda, int la, const bf16* B, int ldb, int lb,
                                  int M, int N, int K, float* C, int ldc, int tile, hipStream_t s);
// sgd != nullptr: instead of storing the reduced gradients, apply the optimizer update to the
// parameters at the same arena positions (single-rank fast path: gradient final once reduced).
hipError_t splitk_reduce(const float* ws, int S, long long stride, int M, int N, float* out,
                         int ldo, const float* bws, long long bstride, float* bout,
                         const float* loss_part, int n_loss_part, float loss_scale,
                         float* loss_out, hipStream_t s, const SgdFuse* sgd = nullptr);
hipError_t slab_reduce(const SlabReduce& r, hipStream_t s);
// Weight gradient whose split-K combine is NOT launched: *pending describes it (S == 0: the
// GEMM wrote dW / db directly, nothing pending).
// Un-split weight gradient stored as bf16 (dW16 / db16, same leading dimension as dW) instead of
// fp32: the bf16 all-reduce payload written by the GEMM epilogue itself (no fp32 round trip and
// no cast pass).  Refused (hipErrorInvalidValue) with an SGD fusion or when the launch would split.
hipError_t linear_wgrad_bf16_ex(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                                float* db, int M, int N, int K, float* ws, hipStream_t s,
                                const SgdFuse* sgd, SlabReduce* pending, bf16* dW16, bf16* db16);
hipError_t linear_wgrad_bf16_deferred(const bf16* dZ, int lddz, const bf16* X, int ldx, float* dW,
                                      float* db, int M, int N, int K, float* ws, hipStream_t s,
                                      const SgdFuse* sgd, SlabReduce* pending);
// Grouped backward launch: dgrad of layer i, wgrad of layer i and the pending combine of layer
// i+1 (three independent jobs) in ONE grid, so each job's tail is filled by the others and two
// launch gaps disappear.  Any argument may be null.  The wgrad's own combine is returned in
// *wg_pending (deferred to the next group).  Shapes the grouped kernel does not cover run as
// separate launches with identical results.
struct DgradArgs {
  const bf16* dZ; int lddz; const bf16* W; int ldw; const bf16* Aprev; int lda_prev;
  bf16* dX; int lddx; int M, N, K, act;
};
struct WgradArgs {
  const bf16* dZ; int lddz; const bf16* X; int ldx; float* dW; float* db; int M, N, K;
  float* ws; SgdFuse sg;
  bf16* dW16 = nullptr; bf16* db16 = nullptr;   // un-split only: bf16 gradient outputs
};
void set_bwd_group(int on);   // 1 = grouped kernel (default), 0 = separate launches (A/B)
bool bwd_group_supported(int rows, int out_f, int in_f);   // this layer shape runs grouped
hipError_t bwd_group(const DgradArgs* dg, const WgradArgs* wg, const SlabReduce* red,
                     SlabReduce* wg_pending, hipStream_t s);
// Wide-model backward pair: the un-split 256x256 weight gradient w1 (with its SGD epilogue when
// w1.sg.g_base is set) and EITHER the dgrad dg OR a second weight gradient w2, in ONE launch
// whose blocks interleave the two jobs (memory-bound SGD epilogues beside compute-bound main
// loops).  Bitwise identical to the separate launches.  hipErrorInvalidValue when a job is not
// eligible (the *_ok predicates): the caller launches them separately then.
bool wide_pair_wgrad_ok(int rows, int out_f, int in_f);
bool wide_pair_dgrad_ok(int rows, int out_f, int in_f);
hipError_t wide_pair(const WgradArgs& w1, const DgradArgs* dg, const WgradArgs* w2, hipStream_t s);
void set_wide_pair(int on);
// the experiment kernels (csrc/experiments: deep ring, wide pairs, stamps) are linked in
bool experiments_built();
// SGD epilogue form of the un-split weight gradients and split-K combines (A/B; 0 default):
// 0 LDS-staged rows (256x256 tiles), 1 per fragment (operands loaded after the sums), 2 fragment
// rows batched
void set_sgd_epilogue(int form);
void set_stage_epi(int on);   // 1: LDS-staged 256x256 forward epilogue (A/B)
// Deferred update fused into a weight-gradient epilogue (several ranks, bf16 payload): the
// un-split 256x256 weight gradient [M][N] stores its own gradient as bf16 (dW16 / db16, the
// all-reduce payload) and applies SGD-momentum to ANOTHER [M][N] region whose all-reduce has
// completed: `other` holds that region's master / momentum / shadow bases (g_base unused) and
// g16o its reduced bf16 gradient.  hipErrorInvalidValue unless wgrad_defer_ok.
bool wgrad_defer_ok(int M, int N, int K);
hipError_t linear_wgrad_bf16_out16_defer(const bf16* dZ, int lddz, const bf16* X, int ldx, bf16* dW16,
                                         bf16* db16, int M, int N, int K, const SgdFuse& other,
                                         const bf16* g16o, hipStream_t s);

// ---- row-band step (rowband.hip): forward + MSE head + activation gradients of a narrow
// square MLP (input and hidden widths H = 512, out == 1) in one launch, then every weight
// gradient in one grouped launch and every combine in one more (see rowband.hip) ----
constexpr int RB_MAXL = 4;   // hidden layers
struct RowbandArgs {
  const bf16* X; int ldx;
  int rows, H, nh, act;
  int in;                   // input width (v2; v1: == H)
  const bf16* Pf[RB_MAXL];  // v2: fragment-major image of W_l (null: the v1 kernel)
  const bf16* Pd[RB_MAXL];  // v2: fragment-major image of W_l^T (l >= 1)
  const bf16* W[RB_MAXL];   // compute (bf16) weights [H][in_l]
  const float* b[RB_MAXL];  // biases [H]
  bf16* a[RB_MAXL];         // saved activations a_l [rows][H]
  bf16* dz[RB_MAXL];        // dZ_l [rows][H]
  const float* wh; const float* bh;   // head weight [H] / bias [1] (fp32)
  const float* y;           // targets [rows]
  float inv_count;
  float* wslab; float* bslab; float* loss_part;   // per-band head partials (rowband_blocks)
  int band_map;             // v2: 1 = block b runs band xcd_remap(b) (an XCD's blocks hold
                            // contiguous rows), 0 = band b
  unsigned long long* stamps = nullptr;   // v2 diagnostic phase stamps (set_rowband_stamps)
  int out_pol = 0;          // copy-out store policy of a / dZ: 0 plain, 1 nt, 2 sc1 (write-through)
  int* zero_words = nullptr;   // block 0 zeroes these (the weight-gradient fixup's tile counters)
  int n_zero = 0;
  // column-split form (small batches, rowband_split_ok): per-band exchange counters + done
  // counter + error word (zero, self-resetting) and the head's partial-dot exchange buffer
  int* xsync = nullptr;
  float* hx = nullptr;
  int rbs_bands = 0;   // (set by the launch) bands; rbs_map: XCD-grouped block map, grid padded
  int rbs_map = 0;     // to whole 8-band groups; rbs_local: plain hand-off stores for a band whose
  int rbs_local = 0;   // blocks all report one XCC id
  // Small-batch weight gradients from K-major operand images (wgrad_small's image path, null:
  // off): the split kernel also writes each band's 32-row x 16-column MFMA operand fragments of
  // its share of X (ka[0]), a_{l-1} (ka[l], l >= 1) and dZ_l (kz[l]) -- fragment (g, band) at
  // element (g * kbands + band) * 512, lane i's 8 rows of column 16 g + (i & 15) at i * 8
  bf16* ka[RB_MAXL] = {};
  bf16* kz[RB_MAXL] = {};
  int kbands = 0;
};
// the column-split row-band kernel takes this batch (H = 512, in <= 512, rows below the
// full-band threshold): 8 blocks per 32-row band, each one 64-column slice of every layer
bool rowband_split_ok(int rows, int H, int in, int nh, int act);
void set_rb_split(int v);    // NNMPI_RB_SPLIT: 0 off, 2 / 4 / 8 blocks per band, else automatic
void set_rb_wgsmall(int v);  // NNMPI_RB_WGSMALL: small-batch weight gradients with the update fused (1) or slabs (0)
int rowband_error_word();    // int index of the split kernel's sticky wait-timeout word in the workspace
int rowband_split_stamp_slots();   // diagnostic stamps per block of the split kernel (set_rowband_stamps)
void set_rb_store_policy(int pol);   // A/B of RowbandArgs::out_pol (-1: NNMPI_RB_STORE)
void set_rb_fixup(int on);   // experiments library: 1 = split-K combine inside the weight-gradient launch, 0 = own launch (default)
// diagnostic: every later v2 row-band launch records per-wave phase stamps into buf
// (rowband_blocks(rows) x rowband_stamp_slots() uint64; null = off)
void set_rowband_stamps(unsigned long long* buf);
int rowband_stamp_slots();
int rowband_blocks(int rows);
void set_rb_band_map(int v);   // A/B: XCD-contiguous band order (-1 re-reads NNMPI_RB_BANDMAP)
bool rowband2_ok(int rows, int H, int in, int nh, int out, int loss, int act);
// elements of the fragment-major weight images one model needs (rowband_pack)
size_t rowband_packed_elems(int H, int in, int nh);
// rebuild the images Pf / Pd from the row-major bf16 weights W (one launch)
hipError_t rowband_pack(const RowbandArgs& p, hipStream_t s);
hipError_t rowband_fwd_bwd(const RowbandArgs& p, hipStream_t s);
// The whole step: grads (or, with sg.g_base set, the fused SGD-momentum update at the arena
// positions of gW / gb / gWh / gbh), loss_out[0] = loss_scale * sum of squared errors.
struct RowbandStep {
  RowbandArgs fb;
  float* gW[RB_MAXL]; float* gb[RB_MAXL];
  float* gWh; float* gbh;
  float* ws;          // rowband_workspace_bytes
  float loss_scale; float* loss_out;
  SgdFuse sg;
  int splits;         // weight-gradient split-K slabs (0 = fill the chip)
  // 0: the whole step; 1: the band launch + the LAST hidden layer's and the head's weight
  // gradients (their bucket's all-reduce can start); 2: every other layer's weight gradients.
  int phase = 0;
  // split-K plan: 0 every layer `splits` (0: the count that fills the chip with all layers in one
  // launch); 1 the phased plan -- the last layer filling the chip alone, the others together.
  // Phases 1 + 2 of a plan == phase 0 of the same plan, bitwise.
  int plan = 0;
  // small batches: the column-split kernel (rowband_split_ok) -- 0 never, 1 when it takes the
  // batch, -1 the same (the engine passes 0 / 1 by its own row threshold)
  int split = -1;
};
size_t rowband_workspace_bytes(int rows, int H, int in, int nh, int splits);
hipError_t rowband_step(const RowbandStep& st, hipStream_t s);
// Weight gradients of several layers in ONE grouped launch (128x128 tiles, split-K with
// `splits` slabs each, 0 = fill the chip); pending[j] receives job j's combine.
int wgrad_multi_splits(int nj, int M, int N, int K);
// (splits: one count per job, or null = fill the chip)
hipError_t wgrad_multi(const WgradArgs* jobs, int nj, const int* splits, SlabReduce* pending,
                       hipStream_t s);
// Several independent combines in ONE launch (same per-block body as slab_reduce).
hipError_t slab_reduce_multi(const SlabReduce* r, int nr, hipStream_t s);
// The same weight gradients with the split-K combine INSIDE the launch: the split that arrives
// last at a tile sums the tile's slabs (slab_multi's order: bitwise the same result) and applies
// the update (job.sg) or stores the gradient (job.dW / job.db), plus the row-band images; `tail`
// (may be null) is one more combine run by extra blocks of the same launch.
struct WgOut {
  bf16* pkf; bf16* pkd;   // with job.sg: the updated W's fragment-major images (null: none)
  int* cnt;               // in-launch fixup (experiments library): per-tile counter words, zero
  const bf16* kA = nullptr;   // wgrad_small: K-major fragment images of dZ (A) and of the layer
  const bf16* kB = nullptr;   // input (B), RowbandArgs::kz / ka (null: the LDS-DMA tiles)
};
#if NNMPI_EXPERIMENTS_BUILD
int wgrad_fix_counters(int M, int N);
#endif
// Small-batch weight gradients of several layers in ONE launch: 64 x 64 tiles over the whole K
// (no split), SGD-momentum + the row-band v2 images (img[j], may be null) in the epilogue when
// jobs[j].sg is set (else the gradient), the head's combine `tail` (may be null) in extra blocks.
// With img[j].kA / kB set for every job (kbands bands, a multiple of 8 up to 64) the operands
// come from the K-major fragment images instead (each wave one eighth of K, summed in order).
hipError_t wgrad_small(const WgradArgs* jobs, int nj, const WgOut* img, const SlabReduce* tail,
                       hipStream_t s, int kbands = 0);
bool wgrad_kimg_ok(int rows);   // the image path takes this batch (and NNMPI_WGS_KIMG allows it)
void set_wgs_kimg(int v);       // A/B: 1 image path, 0 the LDS-DMA tiles, -1 re-read NNMPI_WGS_KIMG
#if NNMPI_EXPERIMENTS_BUILD
hipError_t wgrad_multi_fix(const WgradArgs* jobs, int nj, const int* splits, const WgOut* fix,
                           const SlabReduce* tail, hipStream_t s);
#endif

// ---- fp32 GEMM (gemm_f32.hip) ----
hipError_t linear_fwd_f32(const float* X, int ldx, const float* W, int ldw, const float* bias,
                          float* Y, int ldy, int M, int N, int K, int act, hipStream_t s);
hipError_t linear_dgrad_f32(const float* dZ, int lddz, const float* W, int ldw,
                            const float* Aprev, int lda_prev, float* dX, int lddx, int M, int N,
                            int K, int act, hipStream_t s);
size_t wgrad_f32_workspace_bytes(int M, int N, int K);
hipError_t linear_wgrad_f32(const float* dZ, int lddz, const float* X, int ldx, float* dW,
                            float* db, int M, int N, int K, float* ws, hipStream_t s);

// ---- output layer + loss (head.hip) ----
// a: [rows][in] activations (bf16 if a_bf16 else fp32); W: [out][in] fp32; y: [rows][out] fp32
// (MSE) or labels int64 (XENT).  Writes dlogits [rows][out] fp32, dz_prev [rows][in] (same dtype
// as a; may be null), loss partials [n_part].
int head_fwd_parts(int rows, int in, int out = 1);   // loss partials (= blocks) of head_fwd
hipError_t head_fwd(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                    int out, const float* y, const int64_t* labels, int loss, float inv_count,
                    int act_prev, void* dz_prev, float* dlogits, float* loss_part, hipStream_t s);
bool head_can_fuse(int out, int in, int loss);
size_t head_fused_workspace_bytes(int rows, int in);
hipError_t head_fused(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                      const float* y, float inv_count, int act_prev, void* dz_prev, float* gW,
                      float* gb, float* ws, float* loss_part, float loss_scale, float* loss_out,
                      hipStream_t s, const SgdFuse* sgd = nullptr, SlabReduce* pending = nullptr);
size_t head_wgrad_workspace_bytes(int rows, int in, int out);
// Multi-output head (1 < out <= 16, in 512 / 1024, bf16) with its weight gradient in one
// kernel + the deferred/immediate combine (head.hip head_mo_fused_kernel)
bool head_mo_fused_ok(int a_bf16, int rows, int in, int out, int loss);
void set_head_fused(int on);   // 0: two launches (A/B), 1: fused, -1: environment
size_t head_mo_workspace_bytes(int rows, int in, int out);
hipError_t head_mo_fused(const bf16* a, int rows, int in, const float* W, const float* b, int out,
                         const float* y, const int64_t* labels, int loss, float inv_count,
                         int act_prev, void* dz_prev, float* gW, float* gb, float* ws,
                         float* loss_part, float loss_scale, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd = nullptr, SlabReduce* pending = nullptr,
                         unsigned long long* stamps = nullptr);   // stamps: 8 per block (diagnostic)
// General head on the matrix cores (head.hip): bf16 activations, in % 256 == 0, out <= 128
bool head_general_mfma_ok(int a_bf16, int in, int out);
void set_head_general_valu(int on);   // 1: the VALU general head for bf16 heads too (A/B)
size_t head_general_mfma_workspace_bytes(int rows, int in, int out);
hipError_t head_general_mfma(const bf16* a, int rows, int in, const float* W, const float* b,
                             int out, const float* y, const int64_t* labels, int loss,
                             float inv_count, int act_prev, bf16* dz_out, float* gW, float* gb,
                             float* dlogits_out, float* ws, float loss_scale, float* loss_out,
                             hipStream_t s);
// sgd: apply the optimizer update in the combine; pending: return the combine unlaunched (see
// bwd_group) instead of running it
hipError_t head_wgrad(const void* a, int a_bf16, int rows, int in, const float* dlogits, int out,
                      float* gW, float* gb, float* ws, const float* loss_part, int n_loss_part,
                      float loss_scale, float* loss_out, hipStream_t s, const SgdFuse* sgd = nullptr,
                      SlabReduce* pending = nullptr);

// ---- output layer + loss of any shape (head_general.hip): logits GEMM, loss + dlogits, dZ GEMM,
// weight/bias gradient (split partials + ordered reduce), loss_out[0] = sum * loss_scale.
// dlogits_out (may be null) receives a copy of dlogits [rows][out].
size_t head_general_workspace_bytes(int rows, int in, int out);
hipError_t head_general(const void* a, int a_bf16, int rows, int in, const float* W, const float* b,
                        int out, const float* y, const int64_t* labels, int loss, float inv_count,
                        int act_prev, void* dz_out, float* gW, float* gb, float* dlogits_out,
                        float* ws, float loss_scale, float* loss_out, hipStream_t s);

// ---- whole tiny MLP in one launch (tiny_mlp.hip), fp32, widths <= 16, layers <= 4 ----
struct TinyMLPDesc {
  int n_layers;
  int widths[5];
  int w_off[4];   // arena offsets of W_l
  int b_off[4];   // arena offsets of b_l
  int act;
  int loss;
};
size_t tiny_mlp_workspace_bytes(int rows, int arena_numel);
// sgd != nullptr (single block, i.e. rows <= 256, single rank): the kernel applies the optimizer
// update itself instead of storing the gradient (the whole step is ONE launch).  loss_scale < 0:
// the reported loss is the mean over these rows (else sum * loss_scale, e.g. micro-batches).
hipError_t tiny_mlp_step(const TinyMLPDesc& d, const float* params, const float* X,
                         const float* y, const int64_t* labels, int rows, float inv_count,
                         float* grad, int arena_numel, float* ws, float* loss_out, hipStream_t s,
                         const SgdFuse* sgd = nullptr, float loss_scale = -1.f);
bool tiny_mlp_can_fuse_sgd(int rows);
// CPU twins (csrc/host/tiny_host.cpp): the same step and update on host memory (the CPU /
// gloo path of BASELINE config 1).  Returns nonzero on a bad description.
int tiny_mlp_step_host(const TinyMLPDesc& d, float* params, const float* X, const float* y,
                       const int64_t* labels, int rows, float inv_count, float* grad,
                       int arena_numel, float* loss_out, float loss_scale, const SgdFuse* sgd);
void sgd_momentum_host(float* p, float* g, float* buf, long long n, const float* hp, int nesterov,
                       int first, int zero_grad);

// ---- optimizer / elementwise (optim.hip) ----
// Row-band v2 weight images refreshed by the optimizer pass itself (rowband.hip): matrix t
// ([M][N] row-major, starting `start` elements after the pass's first element -- may be
// negative when the pass begins inside it) is also written into its fragment-major image pkf
// and that of its transpose pkd (either may be null).
struct SgdPack {
  int n;
  long long start[RB_MAXL_PK];
  int M[RB_MAXL_PK], N[RB_MAXL_PK];
  bf16* pkf[RB_MAXL_PK];
  bf16* pkd[RB_MAXL_PK];
};
// hp = {lr, momentum, dampening, weight_decay, grad_scale}
hipError_t sgd_momentum(float* p, float* g, float* buf, bf16* shadow, long long n,
                        const float* hp, int nesterov, int first, int zero_grad, hipStream_t s,
                        const SgdPack* pack = nullptr);
// the same update on a fixed grid of `blocks` blocks (runs beside a GEMM, see optim.hip)
hipError_t sgd_momentum_bg(float* p, float* g, float* buf, bf16* shadow, long long n,
                           const float* hp, int nesterov, int first, int zero_grad, int blocks,
                           hipStream_t s);
// the same update with the gradient read from a bf16 buffer (the bf16 all-reduce payload)
hipError_t sgd_momentum_bf16grad(float* p, const bf16* g, float* buf, bf16* shadow, long long n,
                                 const float* hp, int nesterov, int first, hipStream_t s,
                                 const SgdPack* pack = nullptr);
hipError_t cast_f32_bf16(const float* x, bf16* y, long long n, hipStream_t s);
hipError_t scale_f32(float* x, long long n, float a, hipStream_t s);
hipError_t cast_bf16_f32(const bf16* x, float* y, long long n, hipStream_t s);
hipError_t checksum_f32(const float* x, long long n, double* out, hipStream_t s);
// out[j] = bf16(sum over q = 0..P-1, in order, of (q == me ? out[j] : scratch[q * stride + j]))
// for j < n, accumulated in fp32 (the owner step of RcclComm::allreduce_bf16_acc32)
hipError_t sum_slices_bf16(bf16* out, const bf16* scratch, int P, int me, long long stride,
                           long long n, hipStream_t s);
// fp32 twin (RcclComm::allreduce_f32_ordered): out[j] = sum_q (q == me ? out : scratch[q])[j]
hipError_t sum_slices_f32(float* out, const float* scratch, int P, int me, long long stride,
                          long long n, hipStream_t s);
// diagnostic: `blocks` 256-thread blocks holding their CUs (and a full wave's VGPRs) for
// `seconds` of wall time, then exiting (standin.hip; the collective stand-in)
// (csrc/experiments/standin.hip: experiments builds only; weak, null otherwise)
__attribute__((weak)) hipError_t cu_hold(int blocks, double seconds, hipStream_t s);
// a stream restricted to a CU mask (csrc/experiments/exp_host.cpp; weak, null otherwise)
__attribute__((weak)) hipError_t exp_cu_mask_stream(const uint32_t* mask, int words, hipStream_t* out);
// bitwise replica hash of n 32-bit words; out: 1025 uint64, result at out[1024]
hipError_t hash_u32(const unsigned* x, long long n, unsigned long long* out, hipStream_t s);

// ---- data (data.hip) ----
// dst[r] = src[idx[r]] for r < n, rows of row_bytes (multiple of 4); indices clamped to n_src
hipError_t gather_rows(const void* src, void* dst, const int64_t* idx, int n, long long row_bytes,
                       long long n_src, hipStream_t s);

}  // namespace nnmpi
