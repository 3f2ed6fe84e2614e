// Native runtime check, built with HOST AddressSanitizer + UndefinedBehaviorSanitizer (device
// code is not instrumented; `-fsanitize=` only after `-Xarch_host`): SURVEY.md §5.2 "host ASan on
// the C++ runtime".  Drives the C++ pieces the Python engine uses inside every step, from C++:
//   * RcclComm   — every collective of the runtime on a single-rank communicator (identity
//                  semantics, so each result is known exactly);
//   * GradSync   — per-bucket ready events, the comm stream, join;
//   * GraphRunner — stream capture of asynchronous launchers and repeated replay, compared
//                  bitwise with the same launches run eagerly;
//   * the optimizer / cast / checksum / gather launchers (host argument handling, odd sizes).
// Build: scripts/build_runtime_check.sh (in-tree binary, run on the GPU box by
// tests/test_kernels_gpu.py::test_native_runtime_under_host_asan).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "comm/rccl_comm.h"
#include "kernels/kernels.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d: %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static int g_fails = 0;

static void expect(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++g_fails;
  }
}

template <typename T>
static bool same_bits(const std::vector<T>& a, const std::vector<T>& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(T)) == 0;
}

static int check_collectives(hipStream_t s) {
  const std::string uid = nnmpi::RcclComm::get_unique_id();
  nnmpi::RcclComm comm(uid, 1, 0, 0);
  expect(comm.size() == 1 && comm.rank() == 0, "communicator rank/size");
  const size_t n = 1003;   // odd element count
  std::vector<float> h(2 * n);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.5f * (float)i - 7.f;
  float* d = nullptr;
  CK(hipMalloc(&d, h.size() * sizeof(float)));
  CK(hipMemcpyAsync(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice, s));
  comm.allreduce(d, n, 0, 0, s);                 // one rank: sum == identity
  comm.broadcast(d, n, 0, 0, s);
  comm.reduce(d, n, 0, 0, 0, s);
  comm.allgather(d, d, n, 0, s);                 // in place
  comm.reduce_scatter(d, d, n, 0, 0, s);         // in place
  std::vector<long long> counts{(long long)n}, displs{0};
  comm.scatterv(d, counts, displs, d + n, 0, 0, s);   // first half -> second half
  {
    nnmpi::GradSync gs(&comm, 3, -1);
    gs.bucket_ready(0, d, 300, 0, s);
    gs.bucket_ready(1, d + 300, 400, 0, s);
    gs.bucket_ready(2, d + 700, n - 700, 0, s);
    gs.join(s);
  }
  CK(hipStreamSynchronize(s));
  std::vector<float> out(2 * n);
  CK(hipMemcpy(out.data(), d, out.size() * sizeof(float), hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t i = 0; i < n; ++i) ok = ok && out[i] == h[i] && out[n + i] == h[i];
  expect(ok, "single-rank collectives are the identity; scatterv copies the root's rows");
  expect(comm.poll_error(false) == 0, "no RCCL async error");
  CK(hipFree(d));
  return 0;
}

struct SgdBufs {
  float *p, *g, *m, *hp;
  nnmpi::bf16* sh;
};

static int alloc_sgd(SgdBufs& b, long long n, const std::vector<float>& p0,
                     const std::vector<float>& g0, const std::vector<float>& hp) {
  CK(hipMalloc(&b.p, n * 4));
  CK(hipMalloc(&b.g, n * 4));
  CK(hipMalloc(&b.m, n * 4));
  CK(hipMalloc(&b.sh, n * 2));
  CK(hipMalloc(&b.hp, hp.size() * 4));
  CK(hipMemcpy(b.p, p0.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b.g, g0.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(b.m, 0, n * 4));
  CK(hipMemcpy(b.hp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  return 0;
}

static int check_graph_replay(hipStream_t s) {
  const long long n = 4100;   // multiple of 4 (vector SGD), not of the block size
  std::mt19937 rng(7);
  std::normal_distribution<float> nd;
  std::vector<float> p0(n), g0(n);
  for (long long i = 0; i < n; ++i) { p0[i] = nd(rng); g0[i] = nd(rng); }
  const std::vector<float> hp{0.01f, 0.9f, 0.f, 0.f, 0.5f, 0.f, 0.f, 0.f};
  SgdBufs a{}, b{};
  if (alloc_sgd(a, n, p0, g0, hp) || alloc_sgd(b, n, p0, g0, hp)) return 1;
  const int steps = 5;
  // eager: first step initialises the momentum, then `steps` plain steps
  CK(nnmpi::sgd_momentum(a.p, a.g, a.m, a.sh, n, a.hp, 0, 1, 0, s));
  for (int k = 0; k < steps; ++k) CK(nnmpi::sgd_momentum(a.p, a.g, a.m, a.sh, n, a.hp, 0, 0, 0, s));
  // graph: same first step eagerly, the plain step captured once and replayed
  CK(nnmpi::sgd_momentum(b.p, b.g, b.m, b.sh, n, b.hp, 0, 1, 0, s));
  {
    nnmpi::GraphRunner gr;
    gr.begin(s);
    CK(nnmpi::sgd_momentum(b.p, b.g, b.m, b.sh, n, b.hp, 0, 0, 0, s));
    gr.end();
    expect(gr.ready() && gr.num_nodes() >= 1, "graph captured");
    for (int k = 0; k < steps; ++k) gr.launch(s);
  }
  CK(hipStreamSynchronize(s));
  std::vector<float> pa(n), pb(n), ma(n), mb(n);
  std::vector<uint16_t> sa(n), sb(n);
  CK(hipMemcpy(pa.data(), a.p, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(pb.data(), b.p, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ma.data(), a.m, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(mb.data(), b.m, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sa.data(), a.sh, n * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(sb.data(), b.sh, n * 2, hipMemcpyDeviceToHost));
  expect(same_bits(pa, pb) && same_bits(ma, mb) && same_bits(sa, sb),
         "graph replay == eager launches (parameters, momentum, bf16 shadow)");
  // host reference of torch.optim.SGD (dampening 0): buf = g*s (first), buf = mu*buf + g*s
  double err = 0.0;
  for (long long i = 0; i < n; ++i) {
    double p = p0[i], m = 0.0;
    const double gs = (double)g0[i] * hp[4];
    for (int k = 0; k <= steps; ++k) {
      m = (k == 0) ? gs : hp[1] * m + gs;
      p -= hp[0] * m;
    }
    err = std::fmax(err, std::fabs(p - pa[i]));
  }
  expect(err < 1e-5, "SGD momentum matches the host reference");
  for (SgdBufs* x : {&a, &b}) {
    CK(hipFree(x->p)); CK(hipFree(x->g)); CK(hipFree(x->m)); CK(hipFree(x->sh)); CK(hipFree(x->hp));
  }
  return 0;
}

static int check_data_and_casts(hipStream_t s) {
  const int rows = 257, cols = 13, n = 300;   // 52-byte rows: the 4-byte gather path
  std::vector<float> src(rows * cols);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (float)i * 0.25f;
  std::vector<int64_t> idx(n);
  std::mt19937 rng(3);
  for (int i = 0; i < n; ++i) idx[i] = (int64_t)(rng() % rows);
  float *dsrc = nullptr, *ddst = nullptr;
  int64_t* didx = nullptr;
  double* dsum = nullptr;
  nnmpi::bf16* dh = nullptr;
  CK(hipMalloc(&dsrc, src.size() * 4));
  CK(hipMalloc(&ddst, (size_t)n * cols * 4));
  CK(hipMalloc(&didx, n * 8));
  CK(hipMalloc(&dsum, 65 * 8));   // 64 partials + the result
  CK(hipMalloc(&dh, src.size() * 2));
  CK(hipMemcpy(dsrc, src.data(), src.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(didx, idx.data(), n * 8, hipMemcpyHostToDevice));
  CK(nnmpi::gather_rows(dsrc, ddst, didx, n, cols * 4, rows, s));
  CK(nnmpi::checksum_f32(dsrc, (long long)src.size(), dsum, s));
  CK(nnmpi::cast_f32_bf16(dsrc + 1, dh + 1, (long long)src.size() - 1, s));   // misaligned tail path
  CK(hipStreamSynchronize(s));
  std::vector<float> dst((size_t)n * cols);
  CK(hipMemcpy(dst.data(), ddst, dst.size() * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < cols; ++c) ok = ok && dst[(size_t)r * cols + c] == src[(size_t)idx[r] * cols + c];
  expect(ok, "gather_rows");
  double sum = 0.0, ref = 0.0;
  CK(hipMemcpy(&sum, dsum + 64, 8, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < src.size(); ++i) ref += (double)src[i] * (double)((i % 7) + 1);   // position-weighted
  expect(std::fabs(sum - ref) <= 1e-6 * std::fabs(ref), "checksum_f32");
  std::vector<uint16_t> hb(src.size());
  CK(hipMemcpy(hb.data(), dh, hb.size() * 2, hipMemcpyDeviceToHost));
  bool cok = true;
  for (size_t i = 1; i < src.size(); ++i) {
    uint32_t bits = (uint32_t)hb[i] << 16;
    float back;
    std::memcpy(&back, &bits, 4);
    cok = cok && std::fabs(back - src[i]) <= std::fabs(src[i]) * (1.f / 128.f);
  }
  expect(cok, "cast_f32_bf16 (unaligned)");
  // invalid arguments are rejected on the host, before any launch
  expect(nnmpi::sgd_momentum(ddst, ddst, ddst, nullptr, 3, nullptr, 0, 0, 0, s) == hipErrorInvalidValue,
         "sgd_momentum rejects n % 4 != 0");
  CK(hipFree(dsrc)); CK(hipFree(ddst)); CK(hipFree(didx)); CK(hipFree(dsum)); CK(hipFree(dh));
  return 0;
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (check_collectives(s) || check_graph_replay(s) || check_data_and_casts(s)) return 2;
  CK(hipStreamDestroy(s));
  if (g_fails) {
    std::fprintf(stderr, "runtime_check: %d failure(s)\n", g_fails);
    return 1;
  }
  std::printf("runtime_check: ALL OK\n");
  return 0;
}
