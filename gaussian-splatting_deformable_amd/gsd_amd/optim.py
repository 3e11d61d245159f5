"""The reference's optimizer step, fused.

``FusedAdam`` keeps torch.optim.Adam's interface and semantics for the Gaussian parameter groups of
``training_setup`` (scene/gaussian_model.py:839-856: one group per attribute, its own ``lr``, eps 1e-15,
``update_learning_rate`` rewriting ``param_group['lr']`` each step, :875-886), but stores every
parameter, gradient and moment in flat slabs so that one HIP launch (gsd_adam_step) updates them all.
Construction moves each parameter's data into the parameter slab (``p.data`` becomes a view) and makes
each ``p.grad`` a view of the gradient slab (``self.flat``, a ``FlatGrads``: the one buffer that the
data-parallel all-reduce sums).  There is no CPU path.
"""
from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _native
from ._C import _ptr, _stream
from .parallel import FlatGrads, dp_active, slab_view


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=0.0, betas=(0.9, 0.999), eps=1e-15, coef_major=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps))
        # coef_major: SH parameters (P, K, 3) live coefficient-major in the slab (a (K, 3, P) block; the
        # parameter is a permuted view with strides (1, 3P, P)), so one lane per Gaussian reads and writes each
        # coefficient of a wave as one contiguous 256-B run (gsd_sh_split strides) instead of 64 rows of 180 B.
        # Measured on the bench: no change in preprocess (0.06 / 0.16 ms either way -- those kernels are
        # bound by latency at 220 VGPRs, not by the row accesses), so it is off by default.
        self.coef_major = bool(coef_major)
        coef_major = self.coef_major
        ps = [p for g in self.param_groups for p in g["params"]]
        if len({id(p) for p in ps}) != len(ps):
            raise ValueError("FusedAdam: a parameter appears in more than one group")
        if any(g["betas"] != self.param_groups[0]["betas"] or g["eps"] != self.param_groups[0]["eps"]
               for g in self.param_groups):
            raise ValueError("FusedAdam: betas and eps must be the same for every group")
        if len(self.param_groups) > 16:
            raise ValueError("FusedAdam: at most 16 parameter groups")
        dev = ps[0].device
        if dev.type != "cuda" or any(p.device != dev or p.dtype != torch.float32 for p in ps):
            raise RuntimeError("FusedAdam: parameters must be float32 HIP device tensors on one device")
        total = sum(p.numel() for p in ps)
        self.param_slab = torch.empty(total, dtype=torch.float32, device=dev)
        off = 0
        for p in ps:
            n = p.numel()
            view = slab_view(self.param_slab, off, shape=tuple(p.shape), coef_major=coef_major)
            view.copy_(p.detach())
            p.grad = None
            p.data = view
            off += n
        # the gradient views take each parameter's memory order, so slab element i of the gradient belongs to
        # slab element i of the parameter (what the fused Adam pass pairs)
        self.flat = FlatGrads(ps, device=dev)
        self.flat.invalidate()   # a fresh parameter has no gradient (grad None) until a backward writes one
        self.exp_avg = torch.zeros_like(self.param_slab)
        self.exp_avg_sq = torch.zeros_like(self.param_slab)
        self._layout()
        self.steps = [0] * len(ps)   # torch's state['step'] per parameter (0: no state yet)

    def _layout(self):
        """Slab span, group index and identity of every parameter, in slab order."""
        self._params, self._span, self._gidx = [], [], []
        off = 0
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                self._params.append(p)
                self._span.append((off, off + p.numel()))
                self._gidx.append(gi)
                off += p.numel()

    @property
    def step_count(self) -> int:
        """The largest per-parameter step count (every parameter's, when all of them get gradients)."""
        return max(self.steps, default=0)

    @step_count.setter
    def step_count(self, n: int):
        self.steps = [int(n)] * len(self.steps)

    def zero_grad(self, set_to_none: bool = True):
        """torch.optim.Optimizer.zero_grad.  set_to_none=True (torch's default; the reference's call,
        train.py:683) leaves every parameter without a gradient: the slab is marked stale (FlatGrads.invalidate),
        so a parameter no backward writes before the next step is skipped by it, step count and moments
        untouched, as torch.optim.Adam skips a grad-None parameter.  set_to_none=False zeroes the gradients that
        exist and leaves grad-None parameters without one (torch zeroes only existing .grad tensors): a parameter
        with a zeroed gradient is then stepped with it, as torch does."""
        if set_to_none:
            self.flat.invalidate()
        else:
            none = set(self.flat.stale)   # the parameters without a gradient (stale views) stay so
            self.flat.zero()
            self.flat.stale = none

    def _advance(self, missing, done=frozenset()):
        """torch.optim.Adam skips a parameter whose grad is None and keeps state['step'] per parameter: count
        this step for every parameter that got a gradient (``done``: already stepped inside the backward).
        Returns their indices."""
        active = [i for i, p in enumerate(self._params) if id(p) not in missing and id(p) not in done]
        for i in active:
            self.steps[i] += 1
        return set(active)

    def _bump(self, indices):
        """Advance the autograd version counter of the parameters updated in place through raw pointers (the HIP
        Adam pass and the fused epilogue write memory torch does not see): caches keyed on (data_ptr, _version)
        -- the fused deformation-network forward's packed weights -- then repack, and autograd refuses a graph
        that saved a parameter before this step.  Called once the backward is over."""
        for i in indices:
            torch.autograd.graph.increment_version(self._params[i])

    def _adam(self, a: int, b: int, active, addends=()):
        """gsd_adam_step over slab elements [a, b) of the parameters in ``active``: one launch per contiguous
        run of them (parameters without a gradient are left out, untouched), each run cut into segments of equal
        (learning rate, step count), at most 16 per launch.  ``addends``: [(lo, hi, tensor)] slab ranges whose
        gradient steps with the tensor added (FlatGrads.addend_ranges; gsd_adam_step_ex)."""
        segs = []   # [begin, end, lr, step]
        for i, (pb, pe) in enumerate(self._span):
            lo, hi = max(pb, a), min(pe, b)
            if hi <= lo or i not in active:
                continue
            lr, st = float(self.param_groups[self._gidx[i]]["lr"]), self.steps[i]
            if segs and segs[-1][1] == lo and segs[-1][2] == lr and segs[-1][3] == st:
                segs[-1][1] = hi
            else:
                segs.append([lo, hi, lr, st])
        runs = []
        for sg in segs:
            if runs and runs[-1][-1][1] == sg[0] and len(runs[-1]) < 16:
                runs[-1].append(sg)
            else:
                runs.append([sg])
        g0 = self.param_groups[0]
        beta1, beta2 = g0["betas"]
        lib = _native.load()
        dev = self.param_slab.device
        f4 = 4  # bytes per float: the run's pointers
        with torch.cuda.device(dev):
            for run in runs:
                r0, r1 = run[0][0], run[-1][1]
                k = len(run)
                # at most one addend per launch: a run holding more is cut at the second one's start
                pieces, cuts = [], sorted(lo for lo, hi, _ in addends if r0 < hi and lo < r1)
                bounds = [r0] + [c for c in cuts[1:] if r0 < c < r1] + [r1]
                for q0, q1 in zip(bounds[:-1], bounds[1:]):
                    pieces.append((q0, q1))
                for q0, q1 in pieces:
                    segs_q = [[max(sg[0], q0), min(sg[1], q1), sg[2], sg[3]] for sg in run if sg[0] < q1 and q0 < sg[1]]
                    kq = len(segs_q)
                    add = next(((lo, hi, t) for lo, hi, t in addends if q0 < hi and lo < q1), None)
                    a_ptr, a_lo, a_hi = None, 0, 0
                    if add is not None:
                        lo, hi, t = add
                        s0 = max(lo, q0)
                        a_ptr = ctypes.c_void_p(t.data_ptr() + f4 * (s0 - lo))
                        a_lo, a_hi = s0 - q0, min(hi, q1) - q0
                    _native.check(lib.gsd_adam_step_ex(
                        q1 - q0, ctypes.c_void_p(self.param_slab.data_ptr() + f4 * q0),
                        ctypes.c_void_p(self.flat.slab.data_ptr() + f4 * q0),
                        ctypes.c_void_p(self.exp_avg.data_ptr() + f4 * q0),
                        ctypes.c_void_p(self.exp_avg_sq.data_ptr() + f4 * q0), kq,
                        (ctypes.c_int64 * kq)(*[sg[0] - q0 for sg in segs_q]),
                        (ctypes.c_float * kq)(*[sg[2] for sg in segs_q]),
                        (ctypes.c_int64 * kq)(*[sg[3] for sg in segs_q]), float(beta1), float(beta2),
                        float(g0["eps"]), 0, a_ptr, a_lo, a_hi, _stream(dev)))

    @torch.no_grad()
    def step(self, closure=None, zero_grad: bool = False):
        """One Adam step for every parameter that got a gradient.  ``zero_grad`` then marks the gradient slab
        stale instead of writing zeros (FlatGrads.invalidate): the next backward stores into it, as after
        torch's zero_grad(set_to_none=True)."""
        loss = closure() if closure is not None else None
        self.flat.collect()
        active = self._advance(self.flat.settle())
        self._adam(0, self.param_slab.numel(), active, self.flat.addend_ranges())
        self._bump(active)
        if zero_grad:
            self.flat.invalidate()
        return loss

    @torch.no_grad()
    def allreduce_step(self, zero_grad: bool = False, bucket_floats: int | None = None):
        """Data-parallel step: the gradient all-reduce (FlatGrads.allreduce) and this Adam step, overlapped.
        The all-reduce goes out in buckets on RCCL's stream; Adam runs over every range that needs no
        reduction (the SH gradient the ranks assembled from the exchanged views) at once, and over each bucket
        as soon as that bucket's sum is in -- the device updates bucket k while the links carry bucket k + 1.
        The same arithmetic per element as ``allreduce(); step()``; at world size 1 it is ``step()``.
        Which parameters got a gradient is decided per rank: every rank must produce gradients for the same
        parameters (as DistributedDataParallel requires), or their step counts diverge."""
        from .parallel import BUCKET_FLOATS
        ranges = self.flat.allreduce_buckets(bucket_floats or BUCKET_FLOATS)
        addends = self.flat.addend_ranges()   # rank-summed terms (the exchanged views' mean term): added in the pass
        active = self._advance(self.flat.missing, self.flat.fused)
        for a, b, w in ranges:        # ranges with nothing to wait for first
            if w is None:
                self._adam(a, b, active, addends)
        for a, b, w in ranges:
            if w is not None:
                w.wait()
                self._adam(a, b, active, addends)
        self._bump(active)
        if zero_grad:
            self.flat.invalidate()

    @contextlib.contextmanager
    def step_in_backward(self):
        """``with opt.step_in_backward(): loss.backward()`` is ``loss.backward(); opt.allreduce_step(zero_grad=True)``
        with the Adam step of every parameter whose gradient is final inside the rasterizer backward fused into
        that backward (``fuse``; gsd_adam_epilogue): the gradient never goes through HBM, 8 B per float saved
        (of the 28 B of the separate pass).  Such a gradient is final there when the rasterizer is its only
        producer (store mode: the parameter had no gradient yet this step) and no rank sums it (world size 1).
        The rest is stepped on leaving the block, as ``allreduce_step`` does.  Afterwards the fused parameters'
        ``.grad`` hold no gradient (as after ``zero_grad(set_to_none=True)``); a second gradient producer for
        one of them inside the block -- which the fused step would have missed -- raises."""
        if self.flat.epilogue is not None:
            raise RuntimeError("step_in_backward: already inside a step_in_backward block")
        self.flat.epilogue = self
        steps0 = list(self.steps)
        try:
            yield self
        except BaseException:
            # the step did not happen: step counts back to where they were.  A fused epilogue that was already
            # queued before the exception may have updated its parameters and moments in place (the device work
            # cannot be recalled), so after an exception here the optimizer state of the fused parameters is
            # undefined; the step counts stay torch's (no step taken).
            self.steps = steps0
            self.flat.epilogue = None
            self.flat.fused = set()
            self.flat.drain_early()
            raise
        self.flat.epilogue = None
        self.allreduce_step(zero_grad=True)
        self._bump(i for i, p in enumerate(self._params) if id(p) in self.flat.fused)
        self.flat.fused = set()

    def fuse(self, named, epi=None, summed=False):
        """Called by the rasterizer backward inside ``step_in_backward`` for sinks it is about to store into:
        ``named`` maps gsd_adam_epilogue slots ("dc", "rest", "xyz", "scaling", "rotation", "opacity") to
        parameters.  Counts their step now and returns ``epi`` (a _native.AdamEpilogue, created when None) with
        their slots filled -- or ``epi`` unchanged when the step cannot be fused here (world size > 1, a
        coefficient-major slab, a parameter this optimizer does not own or has already stepped).  ``summed``: the
        caller's gradient is already the sum over every rank (the exchanged SH views), so any world size fuses."""
        if self.flat.epilogue is not self or (dp_active() and not summed) or self.coef_major:
            return epi
        index = {id(p): i for i, p in enumerate(self._params)}
        if any(id(p) not in index or id(p) in self.flat.fused for p in named.values()):
            return epi
        if epi is None:
            g0 = self.param_groups[0]
            epi = _native.AdamEpilogue(beta1=float(g0["betas"][0]), beta2=float(g0["betas"][1]),
                                       eps=float(g0["eps"]))
        f4 = 4
        for slot, p in named.items():
            i = index[id(p)]
            self.steps[i] += 1
            a = self._span[i][0]
            setattr(epi, slot, _native.AdamSink(
                param=p.data_ptr(), exp_avg=self.exp_avg.data_ptr() + f4 * a,
                exp_avg_sq=self.exp_avg_sq.data_ptr() + f4 * a,
                lr=float(self.param_groups[self._gidx[i]]["lr"]), step=self.steps[i]))
            self.flat.fused.add(id(p))
        return epi

    def reduce_early(self, params) -> bool:
        """Called by the data-parallel rasterizer backward inside ``step_in_backward`` once it has stored the final
        per-rank gradients of ``params``: their all-reduce starts now (FlatGrads.early_allreduce), to run on the
        links while the device finishes the backward; ``allreduce_step`` then waits on it instead of issuing it.
        Inside the block a second producer of these gradients raises (it would miss the sum)."""
        if self.flat.epilogue is not self or not dp_active():
            return False
        index = {id(p) for p in self._params}
        if any(id(p) not in index or id(p) in self.flat.fused or id(p) in self.flat.early_ids for p in params):
            return False
        self.flat.early_allreduce(params)
        return True

    @staticmethod
    def fused_owner(params):
        """The FusedAdam inside ``step_in_backward`` that owns ``params`` (through their FlatGrads), or None."""
        flats = {id(getattr(p, "_gsd_flat", None)): getattr(p, "_gsd_flat", None) for p in params}
        if len(flats) != 1:
            return None
        f = next(iter(flats.values()))
        return getattr(f, "epilogue", None) if f is not None else None

    def moments(self, p: torch.Tensor):
        """(exp_avg, exp_avg_sq) views of parameter ``p`` (shaped like ``p``)."""
        off = 0
        for q in (q for g in self.param_groups for q in g["params"]):
            n = q.numel()
            if q is p:
                return slab_view(self.exp_avg, off, like=q), slab_view(self.exp_avg_sq, off, like=q)
            off += n
        raise KeyError("parameter not managed by this optimizer")

    @torch.no_grad()
    def rebuild(self, new_data, new_exp_avg, new_exp_avg_sq):
        """Give every parameter (in group order) new data and moments, whose shapes may differ from the old
        ones -- the optimizer-state surgery of densification (scene/gaussian_model.py:1027-1105:
        replace / prune / concatenate).  Parameter objects stay the same; their ``.data`` and ``.grad``
        become views of freshly allocated slabs; the gradient slab is zero."""
        ps = [p for g in self.param_groups for p in g["params"]]
        if not (len(new_data) == len(new_exp_avg) == len(new_exp_avg_sq) == len(ps)):
            raise ValueError("rebuild: one tensor per parameter expected")
        dev = self.param_slab.device
        total = sum(t.numel() for t in new_data)
        param_slab = torch.empty(total, dtype=torch.float32, device=dev)
        exp_avg = torch.empty_like(param_slab)
        exp_avg_sq = torch.empty_like(param_slab)
        off = 0
        for p, d, a, b in zip(ps, new_data, new_exp_avg, new_exp_avg_sq):
            n = d.numel()
            if a.numel() != n or b.numel() != n:
                raise ValueError("rebuild: moments must match their parameter")
            view = slab_view(param_slab, off, shape=tuple(d.shape), coef_major=self.coef_major)
            view.copy_(d)
            slab_view(exp_avg, off, like=view).copy_(a.reshape(d.shape))   # moments in the parameter's order
            slab_view(exp_avg_sq, off, like=view).copy_(b.reshape(d.shape))
            p.grad = None
            p.data = view
            off += n
        self.param_slab, self.exp_avg, self.exp_avg_sq = param_slab, exp_avg, exp_avg_sq
        # the reference's surgery makes new nn.Parameters: no gradient yet; one layout exchange per step per rank
        self.flat = self.flat.successor(ps, device=dev)
        self._layout()   # per-parameter step counts carry over (the reference keeps stored_state['step'])

    def reset_state(self):
        """Zero the moments and the step counts (as a freshly constructed torch Adam)."""
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        self.steps = [0] * len(self.steps)
