"""The producer of the per-Gaussian offsets: the reference's live deformation network
``DirectTemporalNeRF`` (scene/gaussian_model.py:242-316, with the NeRF positional encoding of :33-82).

Inputs: canonical means (P,3) and a per-view time (P,1, one value); the encoding maps x to
[x, sin(2^k x), cos(2^k x)]_{k<10} (63 channels) and t likewise (21); an 8-layer, 256-wide ReLU MLP with the
encoded x re-injected after layer 4 feeds four linear heads: dx (3), d log-scale (3), d quaternion (4) and
dSH (48).  Before iteration 3000 the reference returns zeros (:302-307).  The module keeps the reference's
parameter names and shapes (``_time.{0..7}``, ``_time_out``, ``_time_out_scale``, ``_time_out_rot``,
``_time_out_shs``), so ``offset_model.pth`` state dicts load as they are (``torch.load(...,
weights_only=True)``).  Its output plugs into ``render()`` as ``pc.offset_model`` and reaches the fused
preamble / split-SH rasterizer directly.

The ≈511k multiply-adds per Gaussian are plain GEMMs, so they go to hipBLASLt through torch.matmul (f32 by
default, like the reference; ``dtype=torch.bfloat16`` runs the hidden layers in bf16 on the MFMA cores with
f32 accumulation).  The encoding is one fused elementwise HIP-friendly torch expression.
"""
from __future__ import annotations

import torch
import torch.nn as nn


# Weight gradients reduce over all P rows (K = P, a 256 x 256 output): one GEMM of that shape gets ~16 output
# tiles -- 16 workgroups on 256 CUs (hipBLASLt picked MT64x64x256 / MT32x64x128 without split-K: 1.8-2.3 ms per
# layer at P = 1M).  Split-K by hand instead: a batched GEMM over row chunks, then a sum over the chunks.
_SPLITK_ROWS = 8192


def _weight_grad(g: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """g^T h summed over the rows, as float32: (N, out), (N, in) -> (out, in)."""
    N = g.shape[0]
    S = N // _SPLITK_ROWS
    if S < 2:
        return (g.t() @ h).float()
    main = S * _SPLITK_ROWS
    dw = torch.bmm(g[:main].view(S, _SPLITK_ROWS, -1).transpose(1, 2), h[:main].view(S, _SPLITK_ROWS, -1))
    dw = dw.sum(0, dtype=torch.float32)
    if main < N:
        dw += (g[main:].t() @ h[main:]).float()
    return dw


class _Linear(torch.autograd.Function):
    """y = h W^T + b (then ReLU when `relu`), in h's dtype (f32 or bf16; W and b cast to it), with the split-K
    weight gradient above; dW and db come back in float32 (the parameters' dtype)."""

    @staticmethod
    def forward(ctx, h, W, b, relu):
        Wc, bc = W.to(h.dtype), b.to(h.dtype)
        # bias and ReLU in the GEMM's epilogue (hipBLASLt) where torch offers it
        y = torch._addmm_activation(bc, h, Wc.t()) if relu else torch.addmm(bc, h, Wc.t())
        ctx.relu = relu
        ctx.save_for_backward(h, Wc, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, Wc, y = ctx.saved_tensors
        gy = gy.to(h.dtype)
        g = torch.ops.aten.threshold_backward(gy, y, 0) if ctx.relu else gy.contiguous()  # one pass
        dh = g @ Wc if ctx.needs_input_grad[0] else None
        dW = _weight_grad(g, h) if ctx.needs_input_grad[1] else None
        db = g.sum(0, dtype=torch.float32) if ctx.needs_input_grad[2] else None
        return dh, dW, db, None


def positional_encoding(x: torch.Tensor, n_freqs: int = 10) -> torch.Tensor:
    """[x, sin(x 2^0), cos(x 2^0), ..., sin(x 2^(n-1)), cos(x 2^(n-1))] (gaussian_model.py:33-82, log sampling)."""
    freqs = 2.0 ** torch.linspace(0.0, n_freqs - 1, steps=n_freqs, device=x.device)
    xf = x[..., None, :] * freqs[:, None]                       # (P, n, d)
    sc = torch.stack((torch.sin(xf), torch.cos(xf)), dim=-2)     # (P, n, 2, d)
    return torch.cat((x, sc.flatten(start_dim=-3)), dim=-1)


class DirectTemporalNeRF(nn.Module):
    def __init__(self, D: int = 8, W: int = 256, n_freqs: int = 10, skips=(4,), zero_before: int = 3000,
                 dtype: torch.dtype = torch.float32):
        super().__init__()
        self.D, self.W, self.n_freqs, self.skips = D, W, n_freqs, tuple(skips)
        self.zero_before = zero_before
        self.compute_dtype = dtype
        self.input_ch = 3 * (1 + 2 * n_freqs)        # 63
        self.input_ch_time = 1 * (1 + 2 * n_freqs)   # 21
        layers = [nn.Linear(self.input_ch + self.input_ch_time, W)]
        for i in range(D - 1):
            layers.append(nn.Linear(W + (self.input_ch if i in self.skips else 0), W))
        self._time = nn.ModuleList(layers)
        self._time_out = nn.Linear(W, 3)
        self._time_out_scale = nn.Linear(W, 3)
        self._time_out_rot = nn.Linear(W, 4)
        self._time_out_shs = nn.Linear(W, 48)

    def forward(self, x: torch.Tensor, ts: torch.Tensor, iteration: int):
        """-> (dx (P,3), d_scale (P,3), d_rot (P,4), d_sh (P,48)) as in gaussian_model.py:290-316."""
        P = x.shape[0]
        if iteration < self.zero_before:
            z = x.new_zeros
            return z(P, 3), z(P, 3), z(P, 4), z(P, 48)
        ex = positional_encoding(x, self.n_freqs)
        et = positional_encoding(ts, self.n_freqs)
        dt = self.compute_dtype if self.compute_dtype != torch.float32 else ex.dtype  # f32: the input's own
        # the hidden layers and the heads in `dt` (as autocast would cast them), bias + ReLU fused after each GEMM;
        # the four heads as one 58-wide GEMM over the concatenated weights
        exd = ex.to(dt)
        h = torch.cat((exd, et.to(dt)), dim=-1)
        for i, layer in enumerate(self._time):
            h = _Linear.apply(h, layer.weight, layer.bias, True)
            if i in self.skips:
                h = torch.cat((exd, h), dim=-1)
        heads = (self._time_out, self._time_out_scale, self._time_out_rot, self._time_out_shs)
        W = torch.cat([m.weight for m in heads], dim=0)
        b = torch.cat([m.bias for m in heads], dim=0)
        o = _Linear.apply(h, W, b, False).float()
        return tuple(t.contiguous() for t in o.split([m.out_features for m in heads], dim=-1))
