"""Camera matrices in the reference's storage convention.

Restates ``utils/graphics_utils.py:38-71`` (getWorld2View2, getProjectionMatrix)
and ``scene/cameras.py:17-71`` (Camera / MiniCam): the world->view matrix is
stored transposed (so the kernels read it column-major,
``cuda_rasterizer/auxiliary.h:58-77``), full_proj = view @ proj (both stored
transposed), camera_center = inverse(view)[3, :3].
"""
from __future__ import annotations

import math

import numpy as np
import torch


def getWorld2View2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    C2W[:3, 3] = (C2W[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(C2W))


def getProjectionMatrix(znear, zfar, fovX, fovY):
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


class Camera:
    """The attributes ``render()`` reads (gaussian_renderer/__init__.py:35-66)."""

    def __init__(self, R, T, FoVx, FoVy, width, height, time=0.0, trans=np.array([0.0, 0.0, 0.0]), scale=1.0,
                 znear=0.01, zfar=100.0, device="cpu"):
        self.R, self.T = R, T
        self.FoVx, self.FoVy = FoVx, FoVy
        self.image_width, self.image_height = int(width), int(height)
        self.time = time
        self.znear, self.zfar = znear, zfar
        self.world_view_transform = torch.tensor(getWorld2View2(R, T, trans, scale)).transpose(0, 1).to(device)
        self.projection_matrix = getProjectionMatrix(znear, zfar, FoVx, FoVy).transpose(0, 1).to(device)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3]

    def to(self, device):
        for k in ("world_view_transform", "projection_matrix", "full_proj_transform", "camera_center"):
            setattr(self, k, getattr(self, k).to(device))
        return self


def yaw_matrix(deg: float) -> np.ndarray:
    a = math.radians(deg)
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def synthetic_camera(width, height, yaw_deg=0.0, fovy_deg=60.0, time=0.0, device="cpu"):
    """SURVEY.md 8(d) camera: at the origin looking down +z, FoVy 60 deg,
    tan(FoVx/2) = tan(FoVy/2) * W/H, znear 0.01, zfar 100; optional yaw offset."""
    fovy = math.radians(fovy_deg)
    fovx = 2.0 * math.atan(math.tan(fovy / 2) * width / height)
    return Camera(yaw_matrix(yaw_deg), np.zeros(3), fovx, fovy, width, height, time=time, device=device)
