// CPU (host) twin of the one-launch tiny-MLP step (tiny_mlp.hip) and of the fused SGD pass
// (optim.hip), for BASELINE config 1: the reference's own 2 -> 3 -> 1 regressor on 16 rows per
// rank in fp32 on the CPU (ref.py:41-45,72,155-211), where the step is pure per-op overhead --
// the plain-PyTorch op path (ops/torch_ops.py, the numerics oracle) issues ~170 Python / ATen
// calls per step (0.28 ms) for a few hundred flops.  One call here runs forward, loss, backward
// and (one rank) the SGD-momentum update over the model's arena region; the arena layout, the
// update arithmetic (fmaf-pinned sgd_elem) and the loss contract (loss_out = sum * loss_scale,
// dlogits = d loss / d logits * inv_count) are those of the GPU kernel.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../kernels/kernels.h"

namespace nnmpi {

namespace {

constexpr int HW = 16;   // widths <= 16
constexpr int HL = 4;    // layers <= 4

inline float act_f(float z, int act) {
  if (act == 1) return z > 0.f ? z : 0.f;
  if (act == 2) return std::tanh(z);
  return z;
}

// derivative through the activation's OUTPUT a = act(z) (threshold_backward semantics)
inline float act_b(float a, int act) {
  if (act == 1) return a > 0.f ? 1.f : 0.f;
  if (act == 2) return 1.f - a * a;
  return 1.f;
}

// torch.optim.SGD update of one element, the arithmetic of sgd_elem (common.h)
inline float sgd_host(float p, float g, float& buf, float lr, float mom, float damp, float wd,
                      float gs, bool nesterov, bool first) {
  float d = g * gs;
  if (wd != 0.f) d = std::fmaf(wd, p, d);
  if (mom != 0.f) {
    buf = first ? d : std::fmaf(mom, buf, (1.f - damp) * d);
    d = nesterov ? std::fmaf(mom, buf, d) : buf;
  }
  return std::fmaf(-lr, d, p);
}

}  // namespace

void sgd_momentum_host(float* p, float* g, float* buf, long long n, const float* hp, int nesterov,
                       int first, int zero_grad) {
  const float lr = hp[0], mom = hp[1], damp = hp[2], wd = hp[3], gs = hp[4];
  for (long long i = 0; i < n; ++i) {
    float b = buf[i];
    p[i] = sgd_host(p[i], g[i], b, lr, mom, damp, wd, gs, nesterov != 0, first != 0);
    if (mom != 0.f) buf[i] = b;
    if (zero_grad) g[i] = 0.f;
  }
}

int tiny_mlp_step_host(const TinyMLPDesc& d, float* P, const float* X, const float* Y,
                       const int64_t* labels, int rows, float inv_count, float* grad,
                       int arena_numel, float* loss_out, float loss_scale, const SgdFuse* sgd) {
  const int L = d.n_layers;
  if (L < 1 || L > HL) return 1;
  for (int l = 0; l <= L; ++l)
    if (d.widths[l] < 1 || d.widths[l] > HW) return 1;
  // the model occupies arena[w_off[L-1] .. arena_numel) (reverse layer order, W_{L-1} first)
  const int base = d.w_off[L - 1];
  std::fill(grad + base, grad + arena_numel, 0.f);
  const int out_w = d.widths[L];
  float loss = 0.f;
  float a[HL + 1][HW];
  float delta[HW], dp[HW];
  for (int r = 0; r < rows; ++r) {
    const int w0 = d.widths[0];
    for (int k = 0; k < w0; ++k) a[0][k] = X[(long long)r * w0 + k];
    for (int l = 0; l < L; ++l) {
      const int win = d.widths[l], wout = d.widths[l + 1];
      const float* W = P + d.w_off[l];
      const float* B = P + d.b_off[l];
      for (int o = 0; o < wout; ++o) {
        float z = B[o];
        for (int i = 0; i < win; ++i) z += W[o * win + i] * a[l][i];
        a[l + 1][o] = (l < L - 1) ? act_f(z, d.act) : z;
      }
    }
    const float* z = a[L];
    float row_loss = 0.f;
    if (d.loss == LOSS_MSE) {
      for (int o = 0; o < out_w; ++o) {
        const float df = z[o] - Y[(long long)r * out_w + o];
        row_loss += df * df;
        delta[o] = 2.f * df * inv_count;
      }
    } else {
      float mx = -INFINITY;
      for (int o = 0; o < out_w; ++o) mx = std::max(mx, z[o]);
      float se = 0.f;
      for (int o = 0; o < out_w; ++o) se += std::exp(z[o] - mx);
      const float lse = mx + std::log(se);
      const int lab = (int)labels[r];
      for (int o = 0; o < out_w; ++o)
        delta[o] = (std::exp(z[o] - lse) - (o == lab ? 1.f : 0.f)) * inv_count;
      row_loss = lse - z[lab];
    }
    loss += row_loss;
    for (int l = L - 1; l >= 0; --l) {
      const int win = d.widths[l], wout = d.widths[l + 1];
      const float* W = P + d.w_off[l];
      float* gw = grad + d.w_off[l];
      float* gb = grad + d.b_off[l];
      for (int o = 0; o < wout; ++o) {
        for (int i = 0; i < win; ++i) gw[o * win + i] += delta[o] * a[l][i];
        gb[o] += delta[o];
      }
      if (l > 0) {
        for (int i = 0; i < win; ++i) {
          float s = 0.f;
          for (int o = 0; o < wout; ++o) s += delta[o] * W[o * win + i];
          dp[i] = s * act_b(a[l][i], d.act);
        }
        std::memcpy(delta, dp, sizeof(float) * win);
      }
    }
  }
  if (loss_out) loss_out[0] = loss * loss_scale;
  if (sgd && sgd->g_base) {
    // one rank: the gradient is final -- update the model's region right here
    const long long off = (grad + base) - sgd->g_base;
    sgd_momentum_host(sgd->p_base + off, grad + base, sgd->m_base + off, arena_numel - base,
                      sgd->hp, sgd->nesterov, sgd->first, 0);
  }
  return 0;
}

}  // namespace nnmpi
