"""Test infrastructure only (tests/ may import this; the product path never does).

float32 torch restatement of the training loss, utils/loss_utils.py:17-63 and train.py:529:
l1_loss = mean|x - y| (:17-18); gaussian window (:23-25), create_window (:27-31), _ssim (:43-63) with
grouped conv2d, zero padding window_size // 2, C1 = 0.01^2, C2 = 0.03^2; loss = (1 - l) L1 + l (1 - SSIM).
Pinned against tests/golden/loss.npz (values produced by the reference module itself).  Device-agnostic:
runs on CPU here and on the GPU box as the fp32 autograd reference for gsd_amd.loss.
"""
from __future__ import annotations

from math import exp

import torch
import torch.nn.functional as F


def l1_loss(x, y):
    return torch.abs(x - y).mean()


def gaussian(window_size, sigma):
    g = torch.tensor([exp(-(k - window_size // 2) ** 2 / float(2 * sigma ** 2)) for k in range(window_size)],
                     dtype=torch.float32)
    return g / g.sum()


def create_window(window_size, channel, device):
    g1 = gaussian(window_size, 1.5).unsqueeze(1)
    g2 = g1.mm(g1.t()).float().unsqueeze(0).unsqueeze(0)
    return g2.expand(channel, 1, window_size, window_size).contiguous().to(device)


def ssim(x, y, window_size=11):
    channel = x.size(-3)
    w = create_window(window_size, channel, x.device).type_as(x)
    pad = window_size // 2
    mu1 = F.conv2d(x, w, padding=pad, groups=channel)
    mu2 = F.conv2d(y, w, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(x * x, w, padding=pad, groups=channel) - mu1_sq
    s2 = F.conv2d(y * y, w, padding=pad, groups=channel) - mu2_sq
    s12 = F.conv2d(x * y, w, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean()


def l1_ssim_loss(x, y, lambda_dssim=0.2):
    return (1.0 - lambda_dssim) * l1_loss(x, y) + lambda_dssim * (1.0 - ssim(x, y))
