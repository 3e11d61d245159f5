"""Seeded synthetic scenes for the bench and the parity tests.

Means: z ~ U(2,10), NDC u,v ~ U(-1.1,1.1) back-projected through the camera;
scales: per-axis sigma_px ~ LogUniform(0.5,4) px converted to world units at
depth z, times exp(N(0,0.3)), stored as log; rotations: normalize(N(0,1)^4);
opacity ~ U(0.05,0.95) stored as logit; SH (M=16): DC ~ N(0,0.5), rest
~ N(0,0.1).  The config list mirrors BASELINE.json "configs".
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

CONFIGS = {
    1: dict(P=10_000, sh_degree=0, W=400, H=400, se3="identity"),
    2: dict(P=100_000, sh_degree=2, W=800, H=800, se3=None),
    3: dict(P=500_000, sh_degree=3, W=1920, H=1080, se3="random"),
    4: dict(P=1_000_000, sh_degree=3, W=1920, H=1080, se3=None),
    5: dict(P=2_000_000, sh_degree=3, W=3840, H=2160, se3=None),
}


@dataclass
class GaussianParams:
    xyz: torch.Tensor          # (P,3)
    scaling: torch.Tensor      # (P,3) log-scales
    rotation: torch.Tensor     # (P,4) unnormalised quaternion (r,x,y,z)
    opacity: torch.Tensor      # (P,1) logit
    features_dc: torch.Tensor  # (P,1,3)
    features_rest: torch.Tensor  # (P,15,3)
    twist: torch.Tensor | None = None  # (P,6) SE(3) twist [w, v]

    def to(self, device):
        return GaussianParams(**{k: (None if v is None else v.to(device)) for k, v in self.__dict__.items()})

    @property
    def P(self) -> int:
        return int(self.xyz.shape[0])


def make_gaussians(P: int, W: int, H: int, seed: int = 0, fovy_deg: float = 60.0, se3: str | None = None,
                   device="cpu") -> GaussianParams:
    g = torch.Generator().manual_seed(seed)
    tany = math.tan(math.radians(fovy_deg) / 2)
    tanx = tany * W / H
    focal = H / (2.0 * tany)
    z = torch.rand(P, generator=g) * 8.0 + 2.0
    u = torch.rand(P, generator=g) * 2.2 - 1.1
    v = torch.rand(P, generator=g) * 2.2 - 1.1
    xyz = torch.stack([u * z * tanx, v * z * tany, z], dim=1)
    sig_px = torch.exp(torch.rand(P, generator=g) * (math.log(4.0) - math.log(0.5)) + math.log(0.5))
    s = (sig_px * z / focal)[:, None] * torch.exp(torch.randn(P, 3, generator=g) * 0.3)
    rot = torch.nn.functional.normalize(torch.randn(P, 4, generator=g), dim=1)
    op = torch.rand(P, 1, generator=g) * 0.9 + 0.05
    dc = torch.randn(P, 1, 3, generator=g) * 0.5
    rest = torch.randn(P, 15, 3, generator=g) * 0.1
    twist = None
    if se3 == "identity":
        twist = torch.zeros(P, 6)
    elif se3 == "random":
        twist = torch.cat([torch.randn(P, 3, generator=g) * 0.05, torch.randn(P, 3, generator=g) * 0.02], dim=1)
    p = GaussianParams(xyz=xyz, scaling=torch.log(s), rotation=rot, opacity=torch.log(op / (1 - op)),
                       features_dc=dc, features_rest=rest, twist=twist)
    return p.to(device)
