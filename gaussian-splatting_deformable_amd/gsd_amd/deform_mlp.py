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
import torch.nn.functional as F


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
        dt = self.compute_dtype
        with torch.autocast(device_type=x.device.type, dtype=dt, enabled=dt != torch.float32):
            h = torch.cat((ex, et), dim=-1)
            for i, layer in enumerate(self._time):
                h = F.relu(layer(h))
                if i in self.skips:
                    h = torch.cat((ex, h), dim=-1)
            outs = (self._time_out(h), self._time_out_scale(h), self._time_out_rot(h), self._time_out_shs(h))
        return tuple(o.float() for o in outs)
