"""HIP (gfx950) implementation of the engine's op set — thin wrappers over ``_nnmpi_hip``.

Every method launches hand-written CDNA4 kernels on the current HIP stream; none of them
allocates, synchronises or falls back to PyTorch compute (so a step built from them can be
captured into a hipGraph).  Workspaces are provided by the caller (the engine sizes them once).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
from ..utils.knobs import knob

from .. import native
from .torch_ops import ACT_CODES

LOSS_CODES = {"mse": 0, "xent": 1}


def _p(t):
    return native.ptr(t)


def _check(cond, msg):
    if not cond:
        raise ValueError(msg)


class HipOps:
    name = "hip"

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.lib = native.lib()

    @property
    def stream(self) -> int:
        return native.stream_handle()

    # ---------------- hidden layers ----------------
    def linear_act(self, x, W, b, act: str, out):
        M, K = x.shape
        N = W.shape[0]
        if x.dtype == torch.bfloat16:
            _check(K % 8 == 0 and N % 4 == 0, f"bf16 linear needs K%8==0, N%4==0 (K={K}, N={N})")
            self.lib.linear_fwd_bf16(_p(x), x.stride(0), _p(W), W.stride(0), _p(b), _p(out),
                                     out.stride(0), M, N, K, ACT_CODES[act], self.stream)
        else:
            self.lib.linear_fwd_f32(_p(x), x.stride(0), _p(W), W.stride(0), _p(b), _p(out),
                                    out.stride(0), M, N, K, ACT_CODES[act], self.stream)

    def linear_dgrad(self, dz, W, a_prev, act: str, out):
        M, K = dz.shape          # K = out features of this layer
        N = W.shape[1]           # in features
        if dz.dtype == torch.bfloat16:
            _check(K % 8 == 0 and N % 8 == 0, f"bf16 dgrad needs K%8==0, N%8==0 (K={K}, N={N})")
            self.lib.linear_dgrad_bf16(_p(dz), dz.stride(0), _p(W), W.stride(0), _p(a_prev),
                                       a_prev.stride(0), _p(out), out.stride(0), M, N, K,
                                       ACT_CODES[act], self.stream)
        else:
            self.lib.linear_dgrad_f32(_p(dz), dz.stride(0), _p(W), W.stride(0), _p(a_prev),
                                      a_prev.stride(0), _p(out), out.stride(0), M, N, K,
                                      ACT_CODES[act], self.stream)

    @staticmethod
    def _check_ws(ws, need: int, what: str):
        """Host-side guard: a split-K workspace smaller than the launch needs would be written
        out of bounds by the kernel (a GPU memory fault), so refuse the launch instead."""
        have = 0 if ws is None else ws.numel() * ws.element_size()
        _check(have >= int(need), f"{what} workspace too small: {have} < {int(need)} bytes")

    def wgrad_workspace_bytes(self, rows, out_f, in_f, dtype) -> int:
        if dtype == torch.bfloat16:
            return int(self.lib.wgrad_workspace_bytes(out_f, in_f, rows))
        return int(self.lib.wgrad_f32_workspace_bytes(out_f, in_f, rows))

    def wgrad_can_fuse_sgd(self, rows, out_f, in_f, dtype, epilogue: bool = False) -> bool:
        """True when the wgrad can apply the optimizer update itself: in its split-K reducer, or
        (``epilogue=True``: the caller guarantees nothing reads this layer's weights afterwards)
        in the GEMM epilogue when there is no split."""
        if dtype != torch.bfloat16:
            return False
        return epilogue or bool(self.lib.wgrad_will_split(out_f, in_f, rows))

    @staticmethod
    def sgd_fusion(arena, hp, nesterov: bool, first: bool):
        sh = _p(arena.shadow) if arena.shadow is not None else 0
        return (_p(arena.grad), _p(arena.master), _p(arena.momentum), sh, _p(hp), int(nesterov),
                int(first))

    def wgrad_can_write_bf16(self, rows, out_f, in_f) -> bool:
        """True when the (un-split) weight gradient can store bf16 gradients itself."""
        return bool(out_f % 8 == 0 and in_f % 8 == 0 and
                    int(self.lib.wgrad_splits(out_f, in_f, rows)) == 1)

    def linear_wgrad(self, dz, x, gW, gb, ws=None, sgd=None, out_bf16=None):
        """``out_bf16=(gW16, gb16)``: store the gradient as bf16 there instead of into gW / gb
        (un-split shapes only, see wgrad_can_write_bf16)."""
        rows, M = dz.shape
        N = x.shape[1]
        if out_bf16 is not None:
            gW16, gb16 = out_bf16
            _check(dz.dtype == torch.bfloat16 and sgd is None and
                   self.wgrad_can_write_bf16(rows, M, N), "bf16 wgrad output: un-split bf16 only")
            _check(gW16.dtype == torch.bfloat16 and tuple(gW16.shape) == (M, N) and
                   gW16.stride(0) == N and gW16.stride(1) == 1, "bf16 wgrad output: dense [M, N]")
            _check(gb16 is None or (gb16.dtype == torch.bfloat16 and gb16.numel() == M),
                   "bf16 wgrad bias output")
            self.lib.linear_wgrad_bf16_out16(_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW16),
                                             _p(gb16), M, N, rows, self.stream)
            return
        if dz.dtype == torch.bfloat16:
            _check(M % 8 == 0 and N % 8 == 0, f"bf16 wgrad needs out%8==0, in%8==0 ({M}, {N})")
            self._check_ws(ws, self.lib.wgrad_workspace_bytes(M, N, rows), "wgrad")
            self.lib.linear_wgrad_bf16(_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW), _p(gb),
                                       M, N, rows, _p(ws), self.stream, sgd)
        else:
            self._check_ws(ws, self.lib.wgrad_f32_workspace_bytes(M, N, rows), "wgrad")
            self.lib.linear_wgrad_f32(_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW), _p(gb),
                                      M, N, rows, _p(ws), self.stream)

    # ---------------- head ----------------
    def head_parts(self, rows: int, in_f: int, out_f: int = 1) -> int:
        return int(self.lib.head_fwd_parts(rows, in_f, out_f))

    def _head_split(self, rows, in_f, out_f=1):
        parts = self.head_parts(rows, in_f, out_f)
        return parts, (parts + 3) // 4 * 4 + 4   # keep the slab region 16-byte aligned

    @staticmethod
    def head_is_general(out_f: int, in_f: int) -> bool:
        """Heads the skinny kernels (head.hip: out <= 16, an fp32 weight image within 64 KiB of
        LDS, in % 8 == 0) do not take run on the general path (head_general.hip)."""
        return out_f > 16 or out_f * in_f * 4 > 65536 or in_f % 8 != 0

    def head_workspace_bytes(self, rows, in_f, out_f, loss="mse") -> int:
        if self.head_is_general(out_f, in_f):
            return int(self.lib.head_general_workspace_bytes(max(rows, 1), in_f, out_f))
        _, off = self._head_split(rows, in_f, out_f)
        return max(int(self.lib.head_wgrad_workspace_bytes(rows, in_f, out_f)),
                   int(self.lib.head_fused_workspace_bytes(rows, in_f)),
                   int(self.lib.head_mo_workspace_bytes(rows, in_f, out_f))) + 4 * off

    def _head_mo(self, a, W, b, y, labels, loss, inv_count, act_prev, dz_out, gW, gb, loss_out,
                 loss_scale, ws, sgd, deferred):
        """Multi-output head with its weight gradient in one kernel (head.hip
        head_mo_fused_kernel); None when the shape is not one it takes."""
        rows, in_f = a.shape
        out_f = W.shape[0]
        if a.dtype != torch.bfloat16 or not self.lib.head_mo_fused_ok(1, rows, in_f, out_f,
                                                                      LOSS_CODES[loss]):
            return None
        _check(a.is_contiguous() and (dz_out is None or dz_out.is_contiguous()),
               "fused head needs contiguous activations")
        parts, off = self._head_split(rows, in_f, out_f)
        return self.lib.head_mo_fused(_p(a), rows, in_f, _p(W), _p(b), out_f, _p(y), _p(labels),
                                      LOSS_CODES[loss], float(inv_count), ACT_CODES[act_prev],
                                      _p(dz_out), _p(gW), _p(gb), _p(ws[off:]), _p(ws[:parts]),
                                      float(loss_scale), _p(loss_out), self.stream, sgd, deferred)

    def head_can_fuse_sgd(self, out_f, in_f, loss) -> bool:
        # both skinny head forms end in a slab combine that can apply the update: the fused
        # regression kernel's (out == 1, MSE) and the separate weight-gradient kernel's; the
        # general head's reducer does not (its update is a separate pass)
        return not self.head_is_general(out_f, in_f)

    def head(self, a, W, b, y, labels, loss: str, inv_count: float, act_prev: str, dz_out,
             gW, gb, dlogits, loss_out, loss_scale: float, ws=None, sgd=None):
        rows, in_f = a.shape
        out_f = W.shape[0]
        if self.head_is_general(out_f, in_f):
            _check(sgd is None, "the general head does not fuse the optimizer update")
            self._check_ws(ws, self.head_workspace_bytes(rows, in_f, out_f), "head")
            _check(a.is_contiguous() and (dz_out is None or dz_out.is_contiguous()),
                   "general head needs contiguous activations")
            self.lib.head_general(_p(a), 1 if a.dtype == torch.bfloat16 else 0, rows, in_f, _p(W),
                                  _p(b), out_f, _p(y), _p(labels), LOSS_CODES[loss],
                                  float(inv_count), ACT_CODES[act_prev], _p(dz_out), _p(gW),
                                  _p(gb), _p(dlogits), _p(ws), float(loss_scale), _p(loss_out),
                                  self.stream)
            return
        _check(in_f % 8 == 0, f"head needs in%8==0 (in={in_f})")
        parts, off = self._head_split(rows, in_f, out_f)
        self._check_ws(ws, self.head_workspace_bytes(rows, in_f, out_f), "head")
        lp = ws[:parts]
        wws = ws[off:]
        a_bf16 = 1 if a.dtype == torch.bfloat16 else 0
        if self._head_mo(a, W, b, y, labels, loss, inv_count, act_prev, dz_out, gW, gb, loss_out,
                         loss_scale, ws, sgd, False) is not None:
            return
        if self.lib.head_can_fuse(out_f, in_f, LOSS_CODES[loss]):
            # regression head: fwd + loss + dZ + wgrad partials in one kernel, then one reduce
            self.lib.head_fused(_p(a), a_bf16, rows, in_f, _p(W), _p(b), _p(y), float(inv_count),
                                ACT_CODES[act_prev], _p(dz_out), _p(gW), _p(gb), _p(wws), _p(lp),
                                float(loss_scale), _p(loss_out), self.stream, sgd)
            return
        self.lib.head_fwd(_p(a), a_bf16, rows, in_f, _p(W), _p(b), out_f, _p(y), _p(labels),
                          LOSS_CODES[loss], float(inv_count), ACT_CODES[act_prev], _p(dz_out),
                          _p(dlogits), _p(lp), self.stream)
        self.lib.head_wgrad(_p(a), a_bf16, rows, in_f, _p(dlogits), out_f, _p(gW), _p(gb),
                            _p(wws), _p(lp), parts, float(loss_scale), _p(loss_out), self.stream,
                            sgd)

    # ---------------- grouped backward (bf16) ----------------
    def head_deferred(self, a, W, b, y, inv_count: float, act_prev: str, dz_out, gW, gb, loss_out,
                      loss_scale: float, ws, sgd=None, labels=None, loss: str = "mse",
                      dlogits=None):
        """Head whose final slab combine (gW, gb, loss; optionally the optimizer update) is
        deferred: returned as a SlabReduce for the next grouped backward launch (bwd_group)."""
        rows, in_f = a.shape
        out_f = W.shape[0]
        parts, off = self._head_split(rows, in_f, out_f)
        self._check_ws(ws, self.head_workspace_bytes(rows, in_f, out_f), "head")
        a_bf16 = 1 if a.dtype == torch.bfloat16 else 0
        if self.lib.head_can_fuse(out_f, in_f, LOSS_CODES[loss]):
            return self.lib.head_fused_deferred(_p(a), a_bf16, rows, in_f, _p(W), _p(b), _p(y),
                                                float(inv_count), ACT_CODES[act_prev], _p(dz_out),
                                                _p(gW), _p(gb), _p(ws[off:]), _p(ws[:parts]),
                                                float(loss_scale), _p(loss_out), self.stream, sgd)
        r = self._head_mo(a, W, b, y, labels, loss, inv_count, act_prev, dz_out, gW, gb, loss_out,
                          loss_scale, ws, sgd, True)
        if r is not None:
            return r
        _check(dlogits is not None, "multi-output head needs a dlogits buffer")
        self.lib.head_fwd(_p(a), a_bf16, rows, in_f, _p(W), _p(b), out_f, _p(y), _p(labels),
                          LOSS_CODES[loss], float(inv_count), ACT_CODES[act_prev], _p(dz_out),
                          _p(dlogits), _p(ws[:parts]), self.stream)
        return self.lib.head_wgrad_deferred(_p(a), a_bf16, rows, in_f, _p(dlogits), out_f, _p(gW),
                                            _p(gb), _p(ws[off:]), _p(ws[:parts]), parts,
                                            float(loss_scale), _p(loss_out), self.stream, sgd)

    def bwd_group_supported(self, rows, out_f, in_f) -> bool:
        return bool(self.lib.bwd_group_supported(rows, out_f, in_f))

    # ---- deferred update fused into a weight-gradient epilogue (several ranks, bf16 payload) ---
    def wgrad_defer_ok(self, rows, out_f, in_f) -> bool:
        return bool(self.lib.wgrad_defer_ok(out_f, in_f, rows))

    def linear_wgrad_defer(self, dz, x, gW16, gb16, arena, hp, nesterov: bool, first: bool,
                           other_offset: int, g16):
        """Weight gradient ``dz^T x`` stored as bf16 into (gW16, gb16) -- the all-reduce payload --
        while its epilogue applies SGD-momentum to the arena weights at ``other_offset`` (a region
        of the same [out, in] shape whose reduced bf16 gradient is in ``g16`` at that offset)."""
        rows, M = dz.shape
        N = x.shape[1]
        _check(self.wgrad_defer_ok(rows, M, N), "deferred update: weight gradient not eligible")
        _check(tuple(gW16.shape) == (M, N) and gW16.stride(0) == N and gb16.numel() == M,
               "deferred update: dense bf16 outputs")
        _check(other_offset + M * N <= arena.numel and g16.numel() >= other_offset + M * N,
               "deferred update: region out of range")
        e, o = 4, other_offset
        sh = _p(arena.shadow) + 2 * o if arena.shadow is not None else 0
        other = (_p(arena.grad) + e * o, _p(arena.master) + e * o, _p(arena.momentum) + e * o, sh,
                 _p(hp), int(nesterov), int(first))
        self.lib.linear_wgrad_bf16_out16_defer(_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW16),
                                               _p(gb16), M, N, rows, other, _p(g16) + 2 * o,
                                               self.stream)

    # ---- wide-model backward pairs (one launch: weight gradient + SGD beside a dgrad) -------
    def wide_pair_wgrad_ok(self, rows, out_f, in_f) -> bool:
        return bool(self.lib.wide_pair_wgrad_ok(rows, out_f, in_f))

    def wide_pair_dgrad_ok(self, rows, out_f, in_f) -> bool:
        return bool(self.lib.wide_pair_dgrad_ok(rows, out_f, in_f))

    def wide_pair(self, wgrad, sgd, dgrad=None, wgrad2=None, sgd2=None):
        """``wgrad = (dz, x, gW, gb)`` (un-split, SGD epilogue ``sgd``) in one launch with EITHER
        ``dgrad = (dz, W, a_prev, act, out)`` OR ``wgrad2`` (same form as wgrad, ``sgd2``)."""
        dz, x, gW, gb = wgrad
        rows, M = dz.shape
        N = x.shape[1]
        _check(dz.dtype == torch.bfloat16 and gb is not None and
               self.wide_pair_wgrad_ok(rows, M, N), "wide pair: weight gradient not eligible")
        _check(tuple(gW.shape) == (M, N) and gW.stride(0) == N, "wide pair: dense dW")
        w = (_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW), _p(gb), M, N, rows, sgd)
        if dgrad is not None:
            dz2, W, a_prev, act, out = dgrad
            r2, K2 = dz2.shape
            N2 = W.shape[1]
            _check(self.wide_pair_dgrad_ok(r2, K2, N2) and tuple(out.shape) == (r2, N2),
                   "wide pair: dgrad not eligible")
            self.lib.wide_pair_wgrad_dgrad_bf16(*w, _p(dz2), dz2.stride(0), _p(W), W.stride(0),
                                                _p(a_prev), a_prev.stride(0), _p(out),
                                                out.stride(0), r2, N2, K2, ACT_CODES[act],
                                                self.stream)
            return
        dz2, x2, gW2, gb2 = wgrad2
        r2, M2 = dz2.shape
        N2 = x2.shape[1]
        _check(gb2 is not None and self.wide_pair_wgrad_ok(r2, M2, N2) and
               tuple(gW2.shape) == (M2, N2) and gW2.stride(0) == N2,
               "wide pair: second weight gradient not eligible")
        self.lib.wide_pair_wgrad_wgrad_bf16(*w, _p(dz2), dz2.stride(0), _p(x2), x2.stride(0),
                                            _p(gW2), _p(gb2), M2, N2, r2, sgd2, self.stream)

    def bwd_group(self, dgrad, wgrad, sgd, pending):
        """One grouped launch: dgrad of layer i (``(dz, W, a_prev, act, out)`` or None), wgrad of
        layer i (``(dz, x, gW, gb, ws)`` or None, optional optimizer fusion ``sgd``) and the
        pending combine of layer i+1.  Returns layer i's pending combine."""
        dg = wg = None
        if dgrad is not None:
            dz, W, a_prev, act, out = dgrad
            rows, K = dz.shape
            N = W.shape[1]
            _check(dz.dtype == torch.bfloat16 and K % 8 == 0 and N % 8 == 0, "bf16 dgrad shapes")
            dg = (_p(dz), dz.stride(0), _p(W), W.stride(0), _p(a_prev), a_prev.stride(0), _p(out),
                  out.stride(0), rows, N, K, ACT_CODES[act])
        if wgrad is not None:
            dz, x, gW, gb, ws = wgrad
            rows, M = dz.shape
            N = x.shape[1]
            _check(dz.dtype == torch.bfloat16 and M % 8 == 0 and N % 8 == 0, "bf16 wgrad shapes")
            self._check_ws(ws, self.lib.wgrad_workspace_bytes(M, N, rows), "wgrad")
            wg = (_p(dz), dz.stride(0), _p(x), x.stride(0), _p(gW), _p(gb), M, N, rows, _p(ws))
        return self.lib.bwd_group(dg, wg, sgd, pending, self.stream)

    def slab_reduce(self, pending):
        if pending is not None:
            self.lib.slab_reduce(pending, self.stream)

    # ---------------- row-band step (rowband.hip) ----------------
    def rowband_version(self, rows: int, widths, act: str, loss: str) -> int:
        """2: the row-band step (fragment-major weight images, rowband.hip) runs this model --
        hidden widths all equal (H in 256 / 384 / 512 / 768 / 1024), input width % 64 == 0,
        out == 1, MSE, everything in the LDS; 0: it does not."""
        widths = list(widths)
        if len(widths) < 3 or any(w != widths[1] for w in widths[1:-1]):
            return 0
        H, in_, nh, out = widths[1], widths[0], len(widths) - 2, widths[-1]
        lc, ac = LOSS_CODES.get(loss, -1), ACT_CODES[act]
        return 2 if self.lib.rowband2_ok(int(rows), H, in_, nh, out, lc, ac) else 0

    def rowband_ok(self, rows: int, widths, act: str, loss: str) -> bool:
        """The whole forward + head + activation-gradient chain runs as one launch per step
        (see rowband.hip)."""
        return self.rowband_version(rows, widths, act, loss) > 0

    def rowband_split_ok(self, rows: int, H: int, in_: int, nh: int, act: str = "relu") -> bool:
        """A row-band step of ``rows`` rows runs the column-split kernel (rowband.hip
        rowband_split_kernel: H = 512, 256 <= in <= 512, in % 256 == 0, 1-4 hidden layers,
        <= 128 bands of 32 rows, any activation; the C++ predicate also requires the grid to fit
        the chip at its occupancy, so every block of a band can be resident together)."""
        return bool(self.lib.rowband_split_ok(int(rows), int(H), int(in_), int(nh), ACT_CODES[act]))

    def rowband_error_word(self) -> int:
        """Index (int32 words) of the split kernel's sticky wait-timeout word in the workspace."""
        return int(self.lib.rowband_error_word())

    def rowband_workspace_bytes(self, rows: int, H: int, nh: int, splits: int = 0,
                                in_: Optional[int] = None) -> int:
        return int(self.lib.rowband_workspace_bytes(int(rows), int(H), int(H if in_ is None else in_),
                                                    int(nh), int(splits)))

    def rowband_packed(self, H: int, in_: int, nh: int, device) -> Tuple[torch.Tensor, list]:
        """The v2 weight images of one model: one bf16 buffer and, per hidden layer, the
        (forward image, dgrad image) views (layer 0 has no dgrad image)."""
        buf = torch.zeros(int(self.lib.rowband_packed_elems(H, in_, nh)), dtype=torch.bfloat16,
                          device=device)
        views, o = [], 0
        for l in range(nh):
            k = in_ if l == 0 else H
            pf = buf[o:o + H * k]
            o += H * k
            pd = None
            if l >= 1:
                pd = buf[o:o + H * H]
                o += H * H
            views.append((pf, pd))
        return buf, views

    @staticmethod
    def _packed_ptrs(packed):
        return None if packed is None else [(_p(pf), _p(pd) if pd is not None else 0)
                                            for pf, pd in packed]

    def rowband_pack(self, weights, packed):
        """Rebuild the v2 weight images from the row-major bf16 weights (one launch)."""
        H, in_ = weights[0].shape
        self.lib.rowband_pack(int(H), int(in_), [_p(W) for W in weights], self._packed_ptrs(packed),
                              self.stream)

    def rowband_step(self, X, layers, wh, bh, y, inv_count: float, gWh, gbh, ws, loss_scale: float,
                     loss_out, act: str, sgd=None, splits: int = 0, packed=None, phase: int = 0,
                     plan: int = 0, split: int = -1):
        """One step body of a narrow MSE regressor in three launches.  ``layers``: per hidden
        layer ``(W16, b, a_out, dz_out, gW, gb)``.  Writes every activation and dZ, the
        gradients (or, with ``sgd``, applies the fused update at their arena positions -- and
        rewrites the ``packed`` v2 weight images from the new weights) and
        ``loss_out[0] = loss_scale * sum of squared errors``.  ``packed``: the v2 weight images
        (must match the weights); None runs the v1 kernel.  ``phase`` 1 / 2: the band launch with
        the last hidden layer's and the head's gradients / the other layers' gradients (the
        overlapped multi-rank schedule); ``plan``: the split-K plan (RowbandStep, kernels.h);
        ``split``: the column-split kernel for small batches -- 0 never, 1 / -1 where it takes the
        batch (rowband_split_ok)."""
        rows, in_ = X.shape
        nh = len(layers)
        H = layers[0][0].shape[0]
        _check(X.dtype == torch.bfloat16 and X.stride(1) == 1, "rowband: bf16 rows")
        _check(packed is not None, "rowband: the fragment-major weight images (rowband_packed)")
        _check(self.lib.rowband2_ok(rows, H, in_, nh, 1, LOSS_CODES["mse"], ACT_CODES[act]),
               "rowband: shape")
        self._check_ws(ws, self.rowband_workspace_bytes(rows, H, nh, splits, in_), "rowband")
        lay = []
        for l, (W, b, a, dz, gW, gb) in enumerate(layers):
            k = in_ if l == 0 else H
            _check(tuple(W.shape) == (H, k) and W.is_contiguous() and W.dtype == torch.bfloat16,
                   "rowband: bf16 [H, in] weights")
            # (a may be None for the last hidden layer: its activations stay inside the band)
            _check((a is None and l == nh - 1) or (a.shape[0] >= rows and a.stride(0) == H and
                                                   a.dtype == torch.bfloat16),
                   "rowband: dense bf16 activation buffers")
            _check(dz.shape[0] >= rows and dz.stride(0) == H and dz.dtype == torch.bfloat16,
                   "rowband: dense bf16 activation buffers")
            _check(gW.is_contiguous() and gW.numel() == H * k and gb.numel() == H and
                   b.numel() == H, "rowband: gradient / bias shapes")
            lay.append((_p(W), _p(b), _p(a), _p(dz), _p(gW), _p(gb)))
        _check(y.numel() >= rows and wh.numel() == H, "rowband: head shapes")
        if packed is not None:
            _check(len(packed) == nh, "rowband: one (forward, dgrad) image pair per hidden layer")
        self.lib.rowband_step(_p(X), X.stride(0), rows, H, in_, ACT_CODES[act], lay, _p(wh),
                              _p(bh), _p(y), float(inv_count), _p(gWh), _p(gbh), _p(ws),
                              float(loss_scale), _p(loss_out), sgd, int(splits),
                              self._packed_ptrs(packed), int(phase), int(plan), int(split),
                              self.stream)

    # ---------------- tiny fused MLP ----------------
    def tiny_workspace_bytes(self, rows, numel) -> int:
        return int(self.lib.tiny_mlp_workspace_bytes(rows, numel))

    def tiny_can_fuse_sgd(self, rows: int) -> bool:
        return bool(self.lib.tiny_mlp_can_fuse_sgd(rows))

    def tiny_step(self, spec, arena, X, y, labels, inv_count, loss_out, ws, sgd=None,
                  loss_scale=None):
        L = spec.n_layers
        w_off = [arena.by_name[f"layers.{2 * i}.weight"].offset for i in range(L)]
        b_off = [arena.by_name[f"layers.{2 * i}.bias"].offset for i in range(L)]
        self.lib.tiny_mlp_step(list(spec.widths), w_off, b_off, ACT_CODES[spec.activation],
                               LOSS_CODES[spec.loss], _p(arena.master), _p(X), _p(y), _p(labels),
                               X.shape[0], float(inv_count), _p(arena.grad), arena.numel,
                               _p(ws), _p(loss_out), self.stream, sgd,
                               -1.0 if loss_scale is None else float(loss_scale))

    # ---------------- data ----------------
    def gather_rows(self, src, idx, dst):
        """dst[r] = src[idx[r]] (one launch; rows are copied as raw bytes)."""
        n = idx.numel()
        row_bytes = src[0].numel() * src.element_size() if src.shape[0] else 0
        _check(src.is_contiguous() and dst.is_contiguous() and idx.dtype == torch.int64,
               "gather_rows needs contiguous src/dst and int64 indices")
        _check(dst.shape[0] >= n and dst[0].numel() * dst.element_size() == row_bytes,
               "gather_rows: destination rows do not match the source rows")
        self.lib.gather_rows(_p(src), _p(dst), _p(idx), n, row_bytes, src.shape[0], self.stream)

    # ---------------- optimizer ----------------
    def sgd(self, arena, hp, nesterov: bool, first: bool, zero_grad: bool = True, offset: int = 0,
            numel: int = None, grad_bf16=None, images=None):
        """``grad_bf16``: read the gradient from this bf16 buffer (same layout as the arena)
        instead of ``arena.grad`` -- the bf16 all-reduce payload, updated from directly.
        ``images``: {layer: (pkf, pkd)} row-band v2 weight images to refresh from the updated
        weights of those layers (the parts inside this pass's range)."""
        n = arena.numel - offset if numel is None else numel
        e = 4  # bytes per fp32 element
        sh = _p(arena.shadow) + 2 * offset if arena.shadow is not None else 0
        pack = None
        if images:
            pack = []
            for li, (pf, pd) in images.items():
                slot = arena.by_name[f"layers.{2 * li}.weight"]
                M, N = slot.shape
                if slot.offset < offset + n and slot.offset + M * N > offset:
                    pack.append((slot.offset - offset, M, N, _p(pf), _p(pd) if pd is not None else 0))
        if grad_bf16 is not None:
            _check(grad_bf16.dtype == torch.bfloat16 and grad_bf16.numel() >= offset + n,
                   "sgd: bf16 gradient buffer too small")
            self.lib.sgd_momentum_bf16grad(_p(arena.master) + e * offset, _p(grad_bf16) + 2 * offset,
                                           _p(arena.momentum) + e * offset, sh, n, _p(hp),
                                           int(nesterov), int(first), self.stream, pack)
            return
        self.lib.sgd_momentum(_p(arena.master) + e * offset, _p(arena.grad) + e * offset,
                              _p(arena.momentum) + e * offset, sh, n, _p(hp), int(nesterov),
                              int(first), int(zero_grad), self.stream, pack)
