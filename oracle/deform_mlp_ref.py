"""Test infrastructure only.  Independent restatement of the reference's DirectTemporalNeRF forward
(scene/gaussian_model.py:33-82 Embedder / get_embedder, :242-316 the network) over a plain dict of
weights, evaluated in float64: the embedding as an explicit list of functions in the reference's order
(identity, then sin / cos per frequency 2^k), layers applied one by one with the skip re-injection."""
from __future__ import annotations

import torch


def embed(x, n=10):
    fns = [lambda v: v]
    for f in (2.0 ** k for k in range(n)):
        fns.append(lambda v, f=f: torch.sin(v * f))
        fns.append(lambda v, f=f: torch.cos(v * f))
    return torch.cat([fn(x) for fn in fns], -1)


def forward(sd, x, t, iteration, D=8, skips=(4,)):
    if iteration < 3000:
        P = x.shape[0]
        return (torch.zeros(P, 3, dtype=x.dtype), torch.zeros(P, 3, dtype=x.dtype), torch.zeros(P, 4, dtype=x.dtype),
                torch.zeros(P, 48, dtype=x.dtype))
    w = {k: v.double() for k, v in sd.items()}
    ex, et = embed(x.double()), embed(t.double())
    h = torch.cat([ex, et], -1)
    for i in range(D):
        h = torch.relu(h @ w[f"_time.{i}.weight"].t() + w[f"_time.{i}.bias"])
        if i in skips:
            h = torch.cat([ex, h], -1)
    head = lambda n: h @ w[f"{n}.weight"].t() + w[f"{n}.bias"]  # noqa: E731
    return head("_time_out"), head("_time_out_scale"), head("_time_out_rot"), head("_time_out_shs")


