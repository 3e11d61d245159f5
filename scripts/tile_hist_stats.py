import os, sys, math
sys.path[:0] = ["/root/repo/gaussian-splatting_deformable_amd", "/root/repo"]
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "gaussian-splatting_deformable_amd"), ROOT]
import torch, numpy as np
from gsd_amd import _C
from gsd_amd.introspect import decode
from gsd_amd.camera import synthetic_camera
from gsd_amd.scene import CONFIGS, make_gaussians
cfg = CONFIGS[4]; P, W, H, D = cfg["P"], cfg["W"], cfg["H"], cfg["sh_degree"]
dev = torch.device("cuda:0")
g = make_gaussians(P, W, H, seed=4); cam = synthetic_camera(W, H).to(dev)
e = torch.empty(0)
K, color, radii, geom, binning, img = _C.rasterize_gaussians(torch.zeros(3, device=dev), g.xyz.to(dev), e, torch.sigmoid(g.opacity).to(dev), torch.exp(g.scaling).to(dev), torch.nn.functional.normalize(g.rotation, dim=1).to(dev), 1.0, e, cam.world_view_transform, cam.full_proj_transform, math.tan(cam.FoVx/2), math.tan(cam.FoVy/2), H, W, torch.cat([g.features_dc, g.features_rest], 1).to(dev), D, cam.camera_center, False, False)
st = decode(P, W, H, K, geom, binning, img)
r = st["ranges"].cpu().numpy().astype(np.int64)
n = r[:, 1] - r[:, 0]
print("K", K, "tiles", len(n), "mean", n.mean(), "max", n.max())
for lo, hi in [(0, 1), (1, 128), (128, 256), (256, 512), (512, 1024), (1024, 2048), (2048, 4096), (4096, 1 << 30)]:
    m = (n >= lo) & (n < hi)
    print(f"[{lo},{hi}) tiles {m.sum()} instances {n[m].sum()}")
nc = st["n_contrib"].cpu().numpy().astype(np.int64)
print("n_contrib mean", nc.mean(), "max", nc.max())
