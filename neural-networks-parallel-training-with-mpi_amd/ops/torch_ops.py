"""Plain-PyTorch implementation of the engine's op set.

This is (a) the CPU compute path (BASELINE config 1 runs on CPU with gloo, like the
reference's CPU-only script) and (b) the numerics oracle every HIP kernel is tested against.
It computes in fp32 (upcasting bf16 operands) and rounds results to the destination dtype,
which is exactly the contract of the HIP kernels (bf16 in, fp32 accumulate, bf16/fp32 out).

The forward uses ``torch.addmm(b, x, W.t())`` and the backward the same products autograd's
``AddmmBackward0``/``MseLossBackward0`` use, so in fp32 the CPU path
reproduces the reference's golden losses to reorder tolerance.
"""
from __future__ import annotations

import torch

ACT_CODES = {"none": 0, "relu": 1, "tanh": 2}


def act_fwd(z: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return torch.relu(z)
    if act == "tanh":
        return torch.tanh(z)
    return z


def act_bwd_from_out(a: torch.Tensor, act: str) -> torch.Tensor:
    if act == "relu":
        return (a > 0).to(torch.float32)
    if act == "tanh":
        return 1.0 - a * a
    return torch.ones_like(a)


class TorchOps:
    name = "torch"

    def __init__(self, device="cpu"):
        self.device = torch.device(device)

    # y = act(x @ W^T + b)
    def linear_act(self, x, W, b, act: str, out):
        z = torch.addmm(b.float(), x.float(), W.float().t())
        out.copy_(act_fwd(z, act))

    # out = (dz @ W) * act'(a_prev)
    def linear_dgrad(self, dz, W, a_prev, act: str, out):
        g = dz.float().mm(W.float())
        out.copy_(g * act_bwd_from_out(a_prev.float(), act))

    # gW = dz^T @ x ; gb = sum(dz, 0)
    def linear_wgrad(self, dz, x, gW, gb, ws=None, out_bf16=None):
        if out_bf16 is not None:
            gW, gb = out_bf16
        gW.copy_(dz.float().t().mm(x.float()))
        if gb is not None:
            gb.copy_(dz.float().sum(0))

    def head(self, a, W, b, y, labels, loss: str, inv_count: float, act_prev: str, dz_out,
             gW, gb, dlogits, loss_out, loss_scale: float, ws=None):
        """Output layer + loss fwd/bwd.  Writes gW, gb, dz_out (if not None), loss_out[0]."""
        af = a.float()
        logits = torch.addmm(b.float(), af, W.float().t())
        if loss == "mse":
            d = logits - y.float()
            total = (d * d).sum()
            dl = 2.0 * d * inv_count
        else:
            lse = torch.logsumexp(logits, dim=1, keepdim=True)
            total = (lse.squeeze(1) - logits.gather(1, labels.view(-1, 1)).squeeze(1)).sum()
            p = torch.exp(logits - lse)
            p[torch.arange(p.shape[0], device=p.device), labels] -= 1.0
            dl = p * inv_count
        if dlogits is not None:
            dlogits.copy_(dl)
        loss_out.fill_(0.0)
        loss_out.add_(total * loss_scale)
        gW.copy_(dl.t().mm(af))
        gb.copy_(dl.sum(0))
        if dz_out is not None:
            dz_out.copy_(dl.mm(W.float()) * act_bwd_from_out(af, act_prev))

    def gather_rows(self, src, idx, dst):
        dst[:idx.numel()].copy_(src.index_select(0, idx))

    def sgd(self, arena, hp, nesterov: bool, first: bool, zero_grad: bool = True, offset: int = 0,
            numel: int = None, grad_bf16=None):
        lr, mom, damp, wd, gs = [float(v) for v in hp.tolist()[:5]]
        n = arena.numel - offset if numel is None else numel
        sl = slice(offset, offset + n)
        p, g, buf = arena.master[sl], arena.grad[sl], arena.momentum[sl]
        if grad_bf16 is not None:
            g = grad_bf16[sl].float()
            zero_grad = False
        with torch.no_grad():
            d = g * gs
            if wd != 0:
                d = d + wd * p
            if mom != 0:
                if first:
                    buf.copy_(d)
                else:
                    buf.mul_(mom).add_(d, alpha=1.0 - damp)
                d = d + mom * buf if nesterov else buf
            p.sub_(lr * d)
            if arena.shadow is not None:
                arena.shadow[sl].copy_(p)
            if zero_grad:
                g.zero_()
