"""Learning-rate schedule of the training loop.

``get_expon_lr_func`` restates ``utils/general_utils.py:29-62`` (log-linear decay from lr_init to lr_final over
max_steps, with the optional reverse-cosine delay), evaluated in numpy float64 as the reference does, so the
rates are bit-identical (``tests/golden/lr.npz``, generated from the reference function).

``update_learning_rate`` restates ``scene/gaussian_model.py:875-886``: every step the "xyz" group's rate comes
from the position schedule and the "offset_model" / "offset_model_rot" groups' from the offset schedule
(``:857-864``).  It rewrites ``param_group['lr']`` of any torch optimizer; ``gsd_amd.optim.FusedAdam`` reads the
groups' rates at each step (and inside the fused backward epilogue), so the new rate is the one applied.
"""
from __future__ import annotations

import numpy as np

# arguments/__init__.py:74-77 (OptimizationParams)
POSITION_LR_INIT = 0.00016
POSITION_LR_FINAL = 0.0000016
POSITION_LR_DELAY_MULT = 0.01
POSITION_LR_MAX_STEPS = 40_000
# scene/gaussian_model.py:862-864
OFFSET_LR_INIT = 8e-4
OFFSET_LR_FINAL = 1.6e-6


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """utils/general_utils.py:29-62: a function of the step; lr_init at step 0, lr_final at max_steps,
    log-linear in between; scaled by lr_delay_mult + (1 - lr_delay_mult) sin(pi/2 clip(step / delay)) while
    step < lr_delay_steps; 0 for a negative step or when both rates are 0."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        log_lerp = np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
        return delay_rate * log_lerp

    return helper


def position_schedule(spatial_lr_scale=1.0, max_steps=POSITION_LR_MAX_STEPS):
    """The xyz schedule of training_setup (scene/gaussian_model.py:857-860) with the default arguments
    (lr_delay_steps stays at its default 0, so lr_delay_mult has no effect, as in the reference)."""
    return get_expon_lr_func(lr_init=POSITION_LR_INIT * spatial_lr_scale,
                             lr_final=POSITION_LR_FINAL * spatial_lr_scale,
                             lr_delay_mult=POSITION_LR_DELAY_MULT, max_steps=max_steps)


def offset_schedule(max_steps=POSITION_LR_MAX_STEPS):
    """The deformation network's schedule (scene/gaussian_model.py:862-864)."""
    return get_expon_lr_func(lr_init=OFFSET_LR_INIT, lr_final=OFFSET_LR_FINAL, max_steps=max_steps)


def update_learning_rate(optimizer, iteration, xyz_schedule, offset_schedule_fn=None):
    """scene/gaussian_model.py:875-886: rewrite the "xyz" group's lr (and the "offset_model" /
    "offset_model_rot" groups' when an offset schedule is given) for ``iteration``.  Returns the xyz rate."""
    lr_xyz = None
    for group in optimizer.param_groups:
        name = group.get("name")
        if name == "xyz":
            lr_xyz = xyz_schedule(iteration)
            group["lr"] = lr_xyz
        elif name in ("offset_model", "offset_model_rot") and offset_schedule_fn is not None:
            group["lr"] = offset_schedule_fn(iteration)
    return lr_xyz
