// pybind11 bindings of the native runtime (kernels, RCCL communicator, gradient synchroniser,
// graph runner).  Tensors cross the boundary as raw device addresses + the caller's HIP stream
// (torch owns the memory; this library owns the compute/comm schedule).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>

#include "comm/rccl_comm.h"
#include "kernels/common.h"
#include "kernels/kernels.h"

namespace py = pybind11;
using namespace nnmpi;

typedef uintptr_t uptr;

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <typename T>
static T* P(uptr p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uptr s) { return reinterpret_cast<hipStream_t>(s); }

// (g_base, p_base, m_base, s_base, hp, nesterov, first) -> SgdFuse, or none
static bool to_sgd(const py::object& o, SgdFuse& f) {
  if (o.is_none()) return false;
  auto t = o.cast<py::tuple>();
  if (t.size() != 7) throw std::runtime_error("sgd fusion tuple needs 7 entries");
  f.g_base = P<const float>(t[0].cast<uptr>());
  f.p_base = P<float>(t[1].cast<uptr>());
  f.m_base = P<float>(t[2].cast<uptr>());
  f.s_base = P<bf16>(t[3].cast<uptr>());
  f.hp = P<const float>(t[4].cast<uptr>());
  f.nesterov = t[5].cast<int>();
  f.first = t[6].cast<int>();
  return true;
}

PYBIND11_MODULE(_nnmpi_hip, m) {
  m.doc() = "MI355X-native kernels and RCCL runtime for nnmpi_amd";

  m.def("arch", []() {
    int dev = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    hipDeviceProp_t prop;
    check(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
    return std::string(prop.gcnArchName);
  });
  m.def("cu_count", []() {
    int dev = 0, n = 0;
    check(hipGetDevice(&dev), "hipGetDevice");
    check(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev), "attr");
    return n;
  });
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });

  // ---- GEMMs ----
  m.def("linear_fwd_bf16", [](uptr X, int ldx, uptr W, int ldw, uptr bias, uptr Y, int ldy, int M,
                              int N, int K, int act, uptr s) {
    check(linear_fwd_bf16(P<const bf16>(X), ldx, P<const bf16>(W), ldw, P<const float>(bias),
                          P<bf16>(Y), ldy, M, N, K, act, S(s)), "linear_fwd_bf16");
  });
  m.def("linear_dgrad_bf16", [](uptr dZ, int lddz, uptr W, int ldw, uptr Ap, int ldap, uptr dX,
                                int lddx, int M, int N, int K, int act, uptr s) {
    check(linear_dgrad_bf16(P<const bf16>(dZ), lddz, P<const bf16>(W), ldw, P<const bf16>(Ap), ldap,
                            P<bf16>(dX), lddx, M, N, K, act, S(s)), "linear_dgrad_bf16");
  });
  m.def("set_gemm_impl", &set_gemm_impl);
  m.def("get_gemm_impl", &get_gemm_impl);
  m.def("set_gemm_tile", &set_gemm_tile);
  m.def("set_gemm_variant", &set_gemm_variant);
  m.def("set_fwd_variant", &set_fwd_variant);
  m.def("set_store_policy", &set_store_policy);
  m.def("set_pp256_order", &set_pp256_order);
  m.def("set_head_xcd_rows", &set_head_xcd_rows);
  m.def("linear_fwd_bf16_stamped", [](uptr X, int ldx, uptr W, int ldw, uptr bias, uptr Y, int ldy,
                                      int M, int N, int K, uptr st, uptr s) {
    check(linear_fwd_bf16_stamped(P<const bf16>(X), ldx, P<const bf16>(W), ldw, P<const float>(bias),
                                  P<bf16>(Y), ldy, M, N, K, P<unsigned long long>(st), S(s)),
          "linear_fwd_bf16_stamped");
  });
  m.def("set_group_async", &set_group_async);
  m.def("set_wgrad_splits", &set_wgrad_splits);
  m.def("wgrad_workspace_bytes", &wgrad_workspace_bytes);
  m.def("wgrad_splits", &wgrad_splits);
  m.def("linear_wgrad_bf16", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW, uptr db, int M, int N,
                                int K, uptr ws, uptr s, py::object sgd) {
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    check(linear_wgrad_bf16(P<const bf16>(dZ), lddz, P<const bf16>(X), ldx, P<float>(dW), P<float>(db),
                            M, N, K, P<float>(ws), S(s), fu ? &f : nullptr), "linear_wgrad_bf16");
  }, py::arg("dZ"), py::arg("lddz"), py::arg("X"), py::arg("ldx"), py::arg("dW"), py::arg("db"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("ws"), py::arg("s"), py::arg("sgd") = py::none());
  m.def("wide_pair_wgrad_ok", &wide_pair_wgrad_ok);
  m.def("wide_pair_dgrad_ok", &wide_pair_dgrad_ok);
  m.def("set_wide_pair", &set_wide_pair);
  m.def("set_sgd_epilogue", &set_sgd_epilogue);
  m.def("set_stage_epi", &set_stage_epi);
  m.def("wgrad_defer_ok", &wgrad_defer_ok);
  m.def("linear_wgrad_bf16_out16_defer", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW16, uptr db16,
                                            int M, int N, int K, py::object other, uptr g16o, uptr s) {
    SgdFuse f{};
    if (!to_sgd(other, f)) throw std::runtime_error("deferred update needs its SGD operands");
    check(linear_wgrad_bf16_out16_defer(P<const bf16>(dZ), lddz, P<const bf16>(X), ldx, P<bf16>(dW16),
                                        P<bf16>(db16), M, N, K, f, P<const bf16>(g16o), S(s)),
          "linear_wgrad_bf16_out16_defer");
  });
  m.def("wide_pair_wgrad_dgrad_bf16", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW, uptr db, int M,
                                         int N, int K, py::object sgd, uptr dZ2, int lddz2, uptr W2,
                                         int ldw2, uptr Ap2, int ldap2, uptr dX2, int lddx2, int M2,
                                         int N2, int K2, int act2, uptr s) {
    WgradArgs w{P<const bf16>(dZ), lddz, P<const bf16>(X), ldx, P<float>(dW), P<float>(db), M, N, K,
                nullptr, SgdFuse{}};
    to_sgd(sgd, w.sg);
    DgradArgs d{P<const bf16>(dZ2), lddz2, P<const bf16>(W2), ldw2, P<const bf16>(Ap2), ldap2,
                P<bf16>(dX2), lddx2, M2, N2, K2, act2};
    check(wide_pair(w, &d, nullptr, S(s)), "wide_pair_wgrad_dgrad_bf16");
  });
  m.def("wide_pair_wgrad_wgrad_bf16", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW, uptr db, int M,
                                         int N, int K, py::object sgd, uptr dZ2, int lddz2, uptr X2,
                                         int ldx2, uptr dW2, uptr db2, int M2, int N2, int K2,
                                         py::object sgd2, uptr s) {
    WgradArgs w{P<const bf16>(dZ), lddz, P<const bf16>(X), ldx, P<float>(dW), P<float>(db), M, N, K,
                nullptr, SgdFuse{}};
    to_sgd(sgd, w.sg);
    WgradArgs w2{P<const bf16>(dZ2), lddz2, P<const bf16>(X2), ldx2, P<float>(dW2), P<float>(db2), M2,
                 N2, K2, nullptr, SgdFuse{}};
    to_sgd(sgd2, w2.sg);
    check(wide_pair(w, nullptr, &w2, S(s)), "wide_pair_wgrad_wgrad_bf16");
  });
  m.def("linear_wgrad_bf16_out16", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW16, uptr db16,
                                      int M, int N, int K, uptr s) {
    check(linear_wgrad_bf16_ex(P<const bf16>(dZ), lddz, P<const bf16>(X), ldx, nullptr, nullptr,
                               M, N, K, nullptr, S(s),
                               nullptr, nullptr, P<bf16>(dW16), P<bf16>(db16)),
          "linear_wgrad_bf16_out16");
  });
  m.def("gemm_bf16_tile", [](uptr A, int lda, int la, uptr B, int ldb, int lb, int M, int N, int K,
                             uptr C, int ldc, int tile, uptr s) {
    check(gemm_bf16_generic_tile(P<const bf16>(A), lda, la, P<const bf16>(B), ldb, lb, M, N, K,
                                 P<float>(C), ldc, tile, S(s)), "gemm_bf16_tile");
  });
  m.def("gemm_bf16", [](uptr A, int lda, int la, uptr B, int ldb, int lb, int M, int N, int K, uptr C,
                        int ldc, uptr s) {
    check(gemm_bf16_generic(P<const bf16>(A), lda, la, P<const bf16>(B), ldb, lb, M, N, K, P<float>(C),
                            ldc, S(s)), "gemm_bf16");
  });
  m.def("linear_fwd_f32", [](uptr X, int ldx, uptr W, int ldw, uptr bias, uptr Y, int ldy, int M,
                             int N, int K, int act, uptr s) {
    check(linear_fwd_f32(P<const float>(X), ldx, P<const float>(W), ldw, P<const float>(bias),
                         P<float>(Y), ldy, M, N, K, act, S(s)), "linear_fwd_f32");
  });
  m.def("linear_dgrad_f32", [](uptr dZ, int lddz, uptr W, int ldw, uptr Ap, int ldap, uptr dX,
                               int lddx, int M, int N, int K, int act, uptr s) {
    check(linear_dgrad_f32(P<const float>(dZ), lddz, P<const float>(W), ldw, P<const float>(Ap), ldap,
                           P<float>(dX), lddx, M, N, K, act, S(s)), "linear_dgrad_f32");
  });
  m.def("wgrad_f32_workspace_bytes", &wgrad_f32_workspace_bytes);
  m.def("linear_wgrad_f32", [](uptr dZ, int lddz, uptr X, int ldx, uptr dW, uptr db, int M, int N,
                               int K, uptr ws, uptr s) {
    check(linear_wgrad_f32(P<const float>(dZ), lddz, P<const float>(X), ldx, P<float>(dW), P<float>(db),
                           M, N, K, P<float>(ws), S(s)), "linear_wgrad_f32");
  });
  m.def("splitk_reduce", [](uptr ws, int S_, long long stride, int M, int N, uptr out, int ldo,
                            uptr bws, long long bstride, uptr bout, uptr lp, int nlp, float lscale,
                            uptr lout, uptr s) {
    check(splitk_reduce(P<const float>(ws), S_, stride, M, N, P<float>(out), ldo, P<const float>(bws),
                        bstride, P<float>(bout), P<const float>(lp), nlp, lscale, P<float>(lout), S(s)),
          "splitk_reduce");
  });

  // ---- head ----
  m.def("head_fwd_parts", &head_fwd_parts, py::arg("rows"), py::arg("in"), py::arg("out") = 1);
  m.def("head_fwd", [](uptr a, int a_bf16, int rows, int in, uptr W, uptr b, int out, uptr y,
                       uptr labels, int loss, float inv_count, int act_prev, uptr dz, uptr dl,
                       uptr lp, uptr s) {
    check(head_fwd(P<const void>(a), a_bf16, rows, in, P<const float>(W), P<const float>(b), out,
                   P<const float>(y), P<const int64_t>(labels), loss, inv_count, act_prev, P<void>(dz),
                   P<float>(dl), P<float>(lp), S(s)), "head_fwd");
  });
  m.def("head_general_workspace_bytes", &head_general_workspace_bytes);
  m.def("head_general", [](uptr a, int a_bf16, int rows, int in, uptr W, uptr b, int out, uptr y,
                           uptr labels, int loss, float inv_count, int act_prev, uptr dz, uptr gW,
                           uptr gb, uptr dlogits, uptr ws, float loss_scale, uptr loss_out, uptr s) {
    check(head_general(P<const void>(a), a_bf16, rows, in, P<const float>(W), P<const float>(b), out,
                       P<const float>(y), P<const int64_t>(labels), loss, inv_count, act_prev,
                       P<void>(dz), P<float>(gW), P<float>(gb), P<float>(dlogits), P<float>(ws),
                       loss_scale, P<float>(loss_out), S(s)),
          "head_general");
  });
  m.def("head_can_fuse", &head_can_fuse);
  m.def("head_fused_workspace_bytes", &head_fused_workspace_bytes);
  m.def("head_fused", [](uptr a, int a_bf16, int rows, int in, uptr W, uptr b, uptr y, float inv_count,
                         int act_prev, uptr dz, uptr gW, uptr gb, uptr ws, uptr lp, float lscale,
                         uptr lout, uptr s, py::object sgd) {
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    check(head_fused(P<const void>(a), a_bf16, rows, in, P<const float>(W), P<const float>(b),
                     P<const float>(y), inv_count, act_prev, P<void>(dz), P<float>(gW), P<float>(gb),
                     P<float>(ws), P<float>(lp), lscale, P<float>(lout), S(s), fu ? &f : nullptr),
          "head_fused");
  }, py::arg("a"), py::arg("a_bf16"), py::arg("rows"), py::arg("in"), py::arg("W"), py::arg("b"),
     py::arg("y"), py::arg("inv_count"), py::arg("act_prev"), py::arg("dz"), py::arg("gW"),
     py::arg("gb"), py::arg("ws"), py::arg("lp"), py::arg("lscale"), py::arg("lout"), py::arg("s"),
     py::arg("sgd") = py::none());
  // ---- deferred combines + grouped backward launch ----
  py::class_<SlabReduce>(m, "SlabReduce")
      .def(py::init<>())
      .def_readonly("S", &SlabReduce::S)
      .def("pending", [](const SlabReduce& r) { return r.S > 0 || r.loss_out != nullptr; });
  m.def("slab_reduce", [](const SlabReduce& r, uptr s) { check(slab_reduce(r, S(s)), "slab_reduce"); });
  m.def("set_bwd_group", &set_bwd_group);
  m.def("bwd_group_supported", &bwd_group_supported);
  m.def("head_fused_deferred", [](uptr a, int a_bf16, int rows, int in, uptr W, uptr b, uptr y,
                                  float inv_count, int act_prev, uptr dz, uptr gW, uptr gb, uptr ws,
                                  uptr lp, float lscale, uptr lout, uptr s, py::object sgd) {
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    SlabReduce r{};
    check(head_fused(P<const void>(a), a_bf16, rows, in, P<const float>(W), P<const float>(b),
                     P<const float>(y), inv_count, act_prev, P<void>(dz), P<float>(gW), P<float>(gb),
                     P<float>(ws), P<float>(lp), lscale, P<float>(lout), S(s), fu ? &f : nullptr, &r),
          "head_fused_deferred");
    return r;
  });
  // dgrad: (dZ, lddz, W, ldw, Aprev, lda_prev, dX, lddx, M, N, K, act) or None
  // wgrad: (dZ, lddz, X, ldx, dW, db, M, N, K, ws) or None; sgd: fusion tuple or None
  // red: SlabReduce or None.  Returns the wgrad's pending combine.
  m.def("bwd_group", [](py::object dgo, py::object wgo, py::object sgd, py::object redo, uptr s) {
    DgradArgs d{};
    WgradArgs w{};
    SlabReduce red{}, pend{};
    const bool hd = !dgo.is_none(), hw = !wgo.is_none(), hr = !redo.is_none();
    if (hd) {
      auto t = dgo.cast<py::tuple>();
      if (t.size() != 12) throw std::runtime_error("dgrad tuple needs 12 entries");
      d = DgradArgs{P<const bf16>(t[0].cast<uptr>()), t[1].cast<int>(), P<const bf16>(t[2].cast<uptr>()),
                    t[3].cast<int>(), P<const bf16>(t[4].cast<uptr>()), t[5].cast<int>(),
                    P<bf16>(t[6].cast<uptr>()), t[7].cast<int>(), t[8].cast<int>(), t[9].cast<int>(),
                    t[10].cast<int>(), t[11].cast<int>()};
    }
    if (hw) {
      auto t = wgo.cast<py::tuple>();
      if (t.size() != 10) throw std::runtime_error("wgrad tuple needs 10 entries");
      w = WgradArgs{P<const bf16>(t[0].cast<uptr>()), t[1].cast<int>(), P<const bf16>(t[2].cast<uptr>()),
                    t[3].cast<int>(), P<float>(t[4].cast<uptr>()), P<float>(t[5].cast<uptr>()),
                    t[6].cast<int>(), t[7].cast<int>(), t[8].cast<int>(), P<float>(t[9].cast<uptr>()),
                    SgdFuse{}};
      to_sgd(sgd, w.sg);
    }
    if (hr) red = redo.cast<SlabReduce>();
    check(bwd_group(hd ? &d : nullptr, hw ? &w : nullptr, hr ? &red : nullptr, &pend, S(s)), "bwd_group");
    return pend;
  }, py::arg("dgrad"), py::arg("wgrad"), py::arg("sgd"), py::arg("red"), py::arg("s"));
  m.def("wgrad_will_split", [](int M, int N, int K) { return wgrad_splits(M, N, K) > 1; });
  m.def("head_wgrad_workspace_bytes", &head_wgrad_workspace_bytes);
  m.def("head_wgrad", [](uptr a, int a_bf16, int rows, int in, uptr dl, int out, uptr gW, uptr gb,
                         uptr ws, uptr lp, int nlp, float lscale, uptr lout, uptr s, py::object sgd) {
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    check(head_wgrad(P<const void>(a), a_bf16, rows, in, P<const float>(dl), out, P<float>(gW),
                     P<float>(gb), P<float>(ws), P<const float>(lp), nlp, lscale, P<float>(lout), S(s),
                     fu ? &f : nullptr),
          "head_wgrad");
  }, py::arg("a"), py::arg("a_bf16"), py::arg("rows"), py::arg("in"), py::arg("dl"), py::arg("out"),
     py::arg("gW"), py::arg("gb"), py::arg("ws"), py::arg("lp"), py::arg("nlp"), py::arg("lscale"),
     py::arg("lout"), py::arg("s"), py::arg("sgd") = py::none());
  m.def("head_wgrad_deferred", [](uptr a, int a_bf16, int rows, int in, uptr dl, int out, uptr gW,
                                  uptr gb, uptr ws, uptr lp, int nlp, float lscale, uptr lout, uptr s,
                                  py::object sgd) {
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    SlabReduce r{};
    check(head_wgrad(P<const void>(a), a_bf16, rows, in, P<const float>(dl), out, P<float>(gW),
                     P<float>(gb), P<float>(ws), P<const float>(lp), nlp, lscale, P<float>(lout), S(s),
                     fu ? &f : nullptr, &r),
          "head_wgrad_deferred");
    return r;
  });

  // ---- tiny fused MLP ----
  m.def("tiny_mlp_workspace_bytes", &tiny_mlp_workspace_bytes);
  m.def("tiny_mlp_step", [](std::vector<int> widths, std::vector<int> w_off, std::vector<int> b_off,
                            int act, int loss, uptr params, uptr X, uptr y, uptr labels, int rows,
                            float inv_count, uptr grad, int numel, uptr ws, uptr lout, uptr s,
                            py::object sgd, float loss_scale) {
    TinyMLPDesc d{};
    d.n_layers = (int)widths.size() - 1;
    if (d.n_layers < 1 || d.n_layers > 4 || (int)w_off.size() != d.n_layers || (int)b_off.size() != d.n_layers)
      throw std::runtime_error("tiny_mlp_step: bad layer description");
    for (size_t i = 0; i < widths.size(); ++i) d.widths[i] = widths[i];
    for (int i = 0; i < d.n_layers; ++i) { d.w_off[i] = w_off[i]; d.b_off[i] = b_off[i]; }
    d.act = act;
    d.loss = loss;
    SgdFuse f{};
    const bool fu = to_sgd(sgd, f);
    check(tiny_mlp_step(d, P<const float>(params), P<const float>(X), P<const float>(y),
                        P<const int64_t>(labels), rows, inv_count, P<float>(grad), numel, P<float>(ws),
                        P<float>(lout), S(s), fu ? &f : nullptr, loss_scale), "tiny_mlp_step");
  }, py::arg("widths"), py::arg("w_off"), py::arg("b_off"), py::arg("act"), py::arg("loss"),
     py::arg("params"), py::arg("X"), py::arg("y"), py::arg("labels"), py::arg("rows"),
     py::arg("inv_count"), py::arg("grad"), py::arg("numel"), py::arg("ws"), py::arg("lout"),
     py::arg("s"), py::arg("sgd") = py::none(), py::arg("loss_scale") = -1.f);
  m.def("tiny_mlp_can_fuse_sgd", &tiny_mlp_can_fuse_sgd);

  // ---- optimizer / elementwise ----
  m.def("sgd_momentum", [](uptr p, uptr g, uptr buf, uptr shadow, long long n, uptr hp, int nesterov,
                           int first, int zero_grad, uptr s) {
    check(sgd_momentum(P<float>(p), P<float>(g), P<float>(buf), P<bf16>(shadow), n, P<const float>(hp),
                       nesterov, first, zero_grad, S(s)), "sgd_momentum");
  });
  m.def("sgd_momentum_bg", [](uptr p, uptr g, uptr buf, uptr shadow, long long n, uptr hp,
                              int nesterov, int first, int zero_grad, int blocks, uptr s) {
    check(sgd_momentum_bg(P<float>(p), P<float>(g), P<float>(buf), P<bf16>(shadow), n,
                          P<const float>(hp), nesterov, first, zero_grad, blocks, S(s)),
          "sgd_momentum_bg");
  });
  m.def("sgd_momentum_bf16grad", [](uptr p, uptr g, uptr buf, uptr shadow, long long n, uptr hp,
                                    int nesterov, int first, uptr s) {
    check(sgd_momentum_bf16grad(P<float>(p), P<const bf16>(g), P<float>(buf), P<bf16>(shadow), n,
                                P<const float>(hp), nesterov, first, S(s)),
          "sgd_momentum_bf16grad");
  });
  m.def("cast_f32_bf16", [](uptr x, uptr y, long long n, uptr s) {
    check(cast_f32_bf16(P<const float>(x), P<bf16>(y), n, S(s)), "cast_f32_bf16");
  });
  m.def("cast_bf16_f32", [](uptr x, uptr y, long long n, uptr s) {
    check(cast_bf16_f32(P<const bf16>(x), P<float>(y), n, S(s)), "cast_bf16_f32");
  });
  m.def("scale_f32", [](uptr x, long long n, float a, uptr s) {
    check(scale_f32(P<float>(x), n, a, S(s)), "scale_f32");
  });
  m.def("checksum_f32", [](uptr x, long long n, uptr out, uptr s) {
    check(checksum_f32(P<const float>(x), n, P<double>(out), S(s)), "checksum_f32");
  });
  m.def("hash_u32", [](uptr x, long long n, uptr out, uptr s) {
    check(hash_u32(P<const unsigned>(x), n, P<unsigned long long>(out), S(s)), "hash_u32");
  });

  // ---- data ----
  m.def("gather_rows", [](uptr src, uptr dst, uptr idx, int n, long long row_bytes, long long n_src,
                          uptr s) {
    check(gather_rows(P<const void>(src), P<void>(dst), P<const int64_t>(idx), n, row_bytes, n_src,
                      S(s)), "gather_rows");
  });

  // ---- RCCL runtime ----
  m.def("rccl_unique_id", []() { return py::bytes(RcclComm::get_unique_id()); });
  py::class_<RcclComm>(m, "RcclComm")
      // bytes -> std::string is converted by pybind11 while the GIL is held; no Python object
      // lives inside the GIL-free body (ncclCommInitRank blocks until every rank has joined)
      .def(py::init([](const std::string& uid, int nranks, int rank, int device) {
             return new RcclComm(uid, nranks, rank, device);
           }), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def("allreduce", [](RcclComm& c, uptr buf, size_t n, int dt, int op, uptr s) {
        c.allreduce(P<void>(buf), n, dt, op, S(s));
      })
      .def("broadcast", [](RcclComm& c, uptr buf, size_t n, int dt, int root, uptr s) {
        c.broadcast(P<void>(buf), n, dt, root, S(s));
      })
      .def("reduce", [](RcclComm& c, uptr buf, size_t n, int dt, int op, int root, uptr s) {
        c.reduce(P<void>(buf), n, dt, op, root, S(s));
      })
      .def("allgather", [](RcclComm& c, uptr sb, uptr rb, size_t n, int dt, uptr s) {
        c.allgather(P<const void>(sb), P<void>(rb), n, dt, S(s));
      })
      .def("reduce_scatter", [](RcclComm& c, uptr sb, uptr rb, size_t n, int dt, int op, uptr s) {
        c.reduce_scatter(P<const void>(sb), P<void>(rb), n, dt, op, S(s));
      })
      .def("scatterv", [](RcclComm& c, uptr sb, std::vector<long long> counts,
                          std::vector<long long> displs, uptr rb, int dt, int root, uptr s) {
        c.scatterv(P<const void>(sb), counts, displs, P<void>(rb), dt, root, S(s));
      })
      .def("broadcast_pieces", [](RcclComm& c, uptr base, std::vector<long long> offsets,
                                  std::vector<long long> counts, std::vector<int> roots, int dt,
                                  uptr s) {
        c.broadcast_pieces(P<void>(base), offsets, counts, roots, dt, S(s));
      })
      .def("poll_error", &RcclComm::poll_error, py::arg("abort_on_error") = true)
      .def("abort", &RcclComm::abort);
  py::class_<GradSync>(m, "GradSync")
      .def(py::init([](RcclComm* c, int nb, int prio) { return new GradSync(c, nb, prio); }),
           py::keep_alive<1, 2>())
      .def("bucket_ready", [](GradSync& g, int b, uptr ptr, size_t n, int dt, uptr s) {
        g.bucket_ready(b, P<void>(ptr), n, dt, S(s));
      })
      .def("join", [](GradSync& g, uptr s) { g.join(S(s)); })
      .def_property_readonly("comm_stream", [](GradSync& g) { return (uptr)g.comm_stream(); });
  py::class_<GraphRunner>(m, "GraphRunner")
      .def(py::init<>())
      .def("begin", [](GraphRunner& g, uptr s, int mode) { g.begin(S(s), mode); },
           py::arg("s"), py::arg("mode") = 1)
      .def("end", &GraphRunner::end)
      .def("cancel", &GraphRunner::cancel)
      .def("launch", [](GraphRunner& g, uptr s) { g.launch(S(s)); })
      .def_property_readonly("ready", &GraphRunner::ready)
      .def_property_readonly("num_nodes", &GraphRunner::num_nodes);
}
