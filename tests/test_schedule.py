"""The learning-rate schedule (gsd_amd.schedule) against get_expon_lr_func of the reference
(utils/general_utils.py:29-62), whose values tests/golden/lr.npz holds (tests/golden/make_golden.py), and
update_learning_rate (scene/gaussian_model.py:875-886) on a torch optimizer's param groups.  CPU only."""
from __future__ import annotations

import numpy as np
import torch

from conftest import golden


def test_expon_lr_matches_reference_fixture():
    from gsd_amd.schedule import get_expon_lr_func
    g = golden("lr.npz")
    for name in ("xyz", "offset", "delay", "zero"):
        kw = {k[len(name) + 1:]: float(g[k]) for k in g.files if k.startswith(name + "_")}
        if "max_steps" in kw:
            kw["max_steps"] = int(kw["max_steps"])
        if "lr_delay_steps" in kw:
            kw["lr_delay_steps"] = int(kw["lr_delay_steps"])
        f = get_expon_lr_func(**kw)
        got = np.array([float(f(int(s))) for s in g["steps"]])
        np.testing.assert_array_equal(got, g[name])   # the same float64 operations: bit-identical


def test_reference_defaults_and_update_learning_rate():
    from gsd_amd.schedule import offset_schedule, position_schedule, update_learning_rate
    g = golden("lr.npz")
    xyz, off = position_schedule(), offset_schedule()
    for i, s in enumerate(g["steps"]):
        assert float(xyz(int(s))) == float(g["xyz"][i]) and float(off(int(s))) == float(g["offset"][i])
    ps = [torch.nn.Parameter(torch.zeros(4)) for _ in range(4)]
    opt = torch.optim.Adam([{"params": [ps[0]], "lr": 0.00016, "name": "xyz"},
                            {"params": [ps[1]], "lr": 0.00016, "name": "offset_model"},
                            {"params": [ps[2]], "lr": 0.0025, "name": "f_dc"},
                            {"params": [ps[3]], "lr": 0.05, "name": "opacity"}], lr=0.0, eps=1e-15)
    for it in (1, 500, 7000, 40000):
        lr = update_learning_rate(opt, it, xyz, off)
        assert lr == xyz(it)
        assert [gr["lr"] for gr in opt.param_groups] == [xyz(it), off(it), 0.0025, 0.05]
    update_learning_rate(opt, 3, xyz)   # no offset schedule given: that group keeps its rate
    assert opt.param_groups[0]["lr"] == xyz(3) and opt.param_groups[1]["lr"] == off(40000)
