"""On-disk formats (gsd_amd.io): the reference's PLY layout (scene/gaussian_model.py:891-1003) and checkpoint
tuple (:686-730).  The reference writes PLY with the `plyfile` package, absent here, and ships no PLY or
checkpoint fixture, so the format is pinned by its documented layout: plyfile's binary header, the attribute
order of construct_list_of_attributes, the channel-major SH flattening -- parity unpinned beyond that."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import PKG  # noqa: F401  (sys.path)


def _pc(P=257, seed=4):
    from gsd_amd import DeformableGaussians
    from gsd_amd.scene import make_gaussians
    return DeformableGaussians(make_gaussians(P, 64, 48, seed=seed), sh_degree=3)


def test_ply_layout_and_roundtrip(tmp_path):
    from gsd_amd.io import attribute_names, load_ply, save_ply
    pc = _pc()
    path = str(tmp_path / "point_cloud" / "iteration_7" / "point_cloud.ply")
    save_ply(path, pc)
    raw = open(path, "rb").read()
    head, body = raw.split(b"end_header\n", 1)
    names = attribute_names()
    assert names[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert names[-8:] == ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]
    assert len(names) == 62
    expect = ["ply", "format binary_little_endian 1.0", "element vertex 257"] + [f"property float {n}" for n in names]
    assert head.decode().strip().split("\n") == expect
    assert len(body) == 257 * 62 * 4
    rows = np.frombuffer(body, dtype="<f4").reshape(257, 62)
    # channel-major SH: f_rest_0..14 are the 15 red coefficients (features_rest[:, :, 0])
    assert np.array_equal(rows[:, 9:24], pc._features_rest.detach()[:, :, 0].numpy())
    assert np.array_equal(rows[:, 3:6], np.zeros((257, 3), np.float32))
    g = load_ply(path, max_sh_degree=3)
    for a, b in [(g.xyz, pc._xyz), (g.features_dc, pc._features_dc), (g.features_rest, pc._features_rest),
                 (g.opacity, pc._opacity), (g.scaling, pc._scaling), (g.rotation, pc._rotation)]:
        assert a.shape == b.shape and torch.equal(a, b.detach())


def test_ply_reader_ascii_and_types(tmp_path):
    from gsd_amd.io import read_ply
    p = tmp_path / "a.ply"
    p.write_text("ply\nformat ascii 1.0\ncomment made by hand\nelement vertex 2\nproperty double x\n"
                 "property uchar red\nproperty float y\nend_header\n1.5 7 -2\n-0.25 255 3.5\n")
    v = read_ply(str(p))
    assert v["x"].tolist() == [1.5, -0.25] and v["red"].tolist() == [7, 255] and v["y"].tolist() == [-2.0, 3.5]
    bad = tmp_path / "b.ply"
    bad.write_bytes(b"nope\n")
    with pytest.raises(ValueError):
        read_ply(str(bad))


def test_load_ply_rejects_wrong_sh_degree(tmp_path):
    from gsd_amd.io import load_ply, save_ply
    path = str(tmp_path / "c.ply")
    save_ply(path, _pc(P=8))
    with pytest.raises(ValueError):
        load_ply(path, max_sh_degree=2)


def test_save_ply_t_roundtrip(tmp_path):
    """save_ply_t (gaussian_model.py:932-958): the given deformed means / activated opacities / deformed rotations
    next to the model's raw SH pieces and raw scaling, in the attribute order of construct_list_of_attributes;
    read back through read_ply bit for bit."""
    from gsd_amd.io import attribute_names, read_ply, save_ply_t
    pc = _pc(P=129, seed=6)
    g = torch.Generator().manual_seed(1)
    xyz = pc._xyz + 0.01 * torch.randn(129, 3, generator=g)
    opac = torch.sigmoid(pc._opacity)
    rot = torch.nn.functional.normalize(pc._rotation + 0.1 * torch.randn(129, 4, generator=g))
    path = str(tmp_path / "test_ply" / "point_cloud_250.ply")
    save_ply_t(path, pc, xyz=xyz, opacities=opac, rotation=rot)
    v = read_ply(path)
    assert list(v) == attribute_names()
    col = lambda *ks: np.stack([v[k] for k in ks], 1)  # noqa: E731
    assert np.array_equal(col("x", "y", "z"), xyz.detach().numpy())
    assert np.array_equal(col("nx", "ny", "nz"), np.zeros((129, 3), np.float32))
    assert np.array_equal(col("opacity"), opac.detach().numpy())
    assert np.array_equal(col("scale_0", "scale_1", "scale_2"), pc._scaling.detach().numpy())
    assert np.array_equal(col("rot_0", "rot_1", "rot_2", "rot_3"), rot.detach().numpy())
    assert np.array_equal(col(*[f"f_rest_{i}" for i in range(15)]), pc._features_rest.detach()[:, :, 0].numpy())
    assert np.array_equal(col("f_dc_0", "f_dc_1", "f_dc_2"), pc._features_dc.detach()[:, 0, :].numpy())
