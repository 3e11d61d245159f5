"""Data parallelism over views: one process per GPU, RCCL all-reduce of the
per-Gaussian gradients.

The reference is single-GPU (train.py:106-112, utils/general_utils.py:133).
Views are independent given replicated Gaussian parameters, so each rank
renders its own view forward+backward, then the gradients are summed.  Every
parameter's ``.grad`` is a view into one flat, contiguous slab, so the
reduction is a few large all-reduces with no pack/unpack copies (xGMI rings
are per-link bound: few, large collectives).  The SH gradient -- 48 of the 59
floats per Gaussian -- is not all-reduced when the means are undeformed: it is
B(dir_v) x dL/dRGB_v per view, so the ranks all-gather the 3-float dL/dRGB
rows (12 B per Gaussian and rank) and each sums the SH gradient of every view
itself (rasterizer._backward_sh_views, gsd_sh_grad_views): 2.4x fewer bytes
on the links at 8 GPUs than the all-reduce of the full slab.
Densification statistics (visibility counts, |dL/dmean2D| sums, max radii)
are per-view quantities and must be taken before the reduction; see
``view_stats_allreduce``.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

# Failure bound of the N > 1 path: every process group (the default one and the gloo signature group) is created
# with this timeout, so a collective whose peer died or hangs raises on the waiting ranks after at most this long
# instead of torch's defaults (10 min for RCCL, 30 min for gloo); with RCCL the watchdog then tears the
# communicator down and the rank exits (TORCH_NCCL_ASYNC_ERROR_HANDLING=1, set unless the caller chose).  A peer
# that EXITS is seen sooner: gloo's connections close at once, and torch.distributed.run stops every worker when
# one fails.  GSD_DIST_TIMEOUT_S overrides the 120 s (tests/test_parallel_gloo.py::test_failed_rank_*).
DIST_TIMEOUT_S = float(os.environ.get("GSD_DIST_TIMEOUT_S", "120"))


def dist_timeout() -> datetime.timedelta:
    return datetime.timedelta(seconds=DIST_TIMEOUT_S)


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """torchrun-style env (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) -> (rank, local_rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or DP_ONE_RANK) and not dist.is_initialized():
        if world == 1:   # GSD_DP_ONE_RANK without a launcher: a one-rank group on this host
            for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29571"), ("RANK", "0"), ("WORLD_SIZE", "1")):
                os.environ.setdefault(k, v)
        # GSD_DIST_BACKEND=gloo: rehearse the data-parallel path with every rank on one GPU (gloo through host
        # memory; bench.py then maps LOCAL_RANK onto the devices present)
        backend = backend or os.environ.get("GSD_DIST_BACKEND") or None
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(backend=backend, timeout=dist_timeout())
        signature_group()   # collective: every rank creates the host-side group at the same point
    return rank, local, world


_SIG_GROUP = None


def signature_group():
    """The process group of the per-step layout check (FlatGrads.verify_layout): the default group when it is
    gloo, else a gloo group over the same ranks, so the check is a host-side exchange that never waits on the
    device.  Creating it is a collective: init_from_env does it on every rank; a caller that initialises the
    default group itself must call this on every rank before the first data-parallel step."""
    global _SIG_GROUP
    if _SIG_GROUP is None:
        _SIG_GROUP = (dist.group.WORLD if dist.get_backend() == "gloo" else
                      dist.new_group(backend="gloo", timeout=dist_timeout()))
    return _SIG_GROUP


def slab_view(slab, off, like=None, shape=None, coef_major=False):
    """A view of slab[off : off + n] shaped like ``like`` with ``like``'s memory order (any permutation of a
    contiguous layout), or, given ``shape``, contiguous -- or coefficient-major when ``coef_major`` and the
    shape is an SH tensor (P, K, 3): stored as (K, 3, P), so the (P,K,3) view has strides (1, 3P, P)."""
    if like is not None:
        shape = tuple(like.shape)
        n = like.numel()
        if not like.is_contiguous() and like.dim() > 1:
            perm = sorted(range(like.dim()), key=lambda d: -like.stride(d))
            if like.permute(perm).is_contiguous():
                inv = [perm.index(d) for d in range(like.dim())]
                return slab[off:off + n].view([shape[d] for d in perm]).permute(inv)
        return slab[off:off + n].view(shape)
    n = 1
    for d in shape:
        n *= d
    if coef_major and len(shape) == 3 and shape[2] == 3:
        return slab[off:off + n].view(shape[1], 3, shape[0]).permute(2, 0, 1)
    return slab[off:off + n].view(shape)


SH_VIEWS = os.environ.get("GSD_SH_VIEWS", "1") != "0"   # exchange per-view dL/dRGB instead of the SH gradient
# all-reduce bucket (floats) of FusedAdam.allreduce_step: 8M floats = 32 MB, a few per step at 1M Gaussians, each
# large enough for the ring to run at link rate on xGMI (GSD_BUCKET_MB overrides)
BUCKET_FLOATS = int(float(os.environ.get("GSD_BUCKET_MB", "32")) * (1 << 20) / 4)


# GSD_DP_ONE_RANK=1: a one-rank process group still takes the data-parallel path (the SH-view all-gather, the
# early and bucketed all-reduces), so that path -- RCCL's streams and asynchronous works included -- runs on a
# one-GPU box (tests/test_gpu_multiview.py::test_one_rank_rccl_matches_single_process)
DP_ONE_RANK = os.environ.get("GSD_DP_ONE_RANK", "0") == "1"


def data_parallel_world() -> int:
    """World size of the default process group (1 without torch.distributed)."""
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def dp_active() -> bool:
    """Whether the data-parallel path runs: a process group of more than one rank, or of one with
    GSD_DP_ONE_RANK=1."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size() > 1 or DP_ONE_RANK


def mark_reduced(params):
    """The gradients of ``params`` (FlatGrads views) already hold the sum over all ranks for this step."""
    for p in params:
        f = getattr(p, "_gsd_flat", None)
        if f is not None:
            f.reduced.add(id(p))


class FlatGrads:
    """Owns one contiguous gradient slab; each parameter's .grad is a view of it.

    A parameter's view can be *stale* (``invalidate``: what the fused Adam step leaves instead of writing
    zeros): its contents are a previous step's and the next gradient producer stores instead of adding --
    torch's ``zero_grad(set_to_none=True)`` semantics (the first backward assigns, later ones accumulate)
    without a memset.  The fused HIP backwards ask ``claim`` whether to store or add; any other producer
    (autograd's AccumulateGrad) goes through a hook that zeroes a stale view first; a view still stale at
    the optimizer step holds no gradient and is zeroed then."""

    def __init__(self, params, device=None):
        self.params = [p for p in params if p is not None]
        dev = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.slab = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        self.views = []
        for p in self.params:
            v = slab_view(self.slab, off, like=p)   # the parameter's memory order (FusedAdam's layouts)
            self.views.append(v)
            off += p.numel()
        self.stale = set()
        self.missing = set()   # what the last settle() found without a gradient
        self.epilogue = None   # the FusedAdam inside its step_in_backward block, if any
        self.fused = set()     # parameters that block already stepped inside the backward
        self.reduced = set()   # views already summed over the ranks this step (mark_reduced)
        self.early = []        # [(a, b, work)]: all-reduces issued inside the backward (early_allreduce)
        self.early_ids = set()
        self.addends = {}      # id(p) -> tensor: a gradient term already summed over the ranks (add_after_reduce)
        self._view_of = {id(p): v for p, v in zip(self.params, self.views)}
        self.hooks = [p.register_hook(self._before_accumulate(p)) for p in self.params if p.requires_grad]
        self._sig_pending = None
        self._verified = False   # this step's layout check is done (reset at the step boundary)
        self.attach()

    # ---- the layout check of the data-parallel path ----
    def layout_signature(self):
        """What every rank's slab must agree on before its collectives: the slab size, the parameters' shapes
        (a densification that ran on one rank only changes both), the bucket size and the SH-view exchange mode
        (which decide the collectives' sizes and count)."""
        shapes = 0
        for p in self.params:
            for d in (p.dim(),) + tuple(p.shape):
                shapes = (shapes * 1000003 + int(d)) % (1 << 61)
        return [int(self.slab.numel()), len(self.params), shapes, int(BUCKET_FLOATS), int(SH_VIEWS)]

    def post_layout_check(self):
        """Start this step's layout check: an asynchronous host-side all-gather of layout_signature() on the gloo
        signature group, its latency overlapping the forward.  The rasterizer's forward posts it for the FlatGrads
        of its inputs (gsd_amd.rasterizer), i.e. after any densification between steps, so the signature is the
        layout the step's collectives will use; at most one post per step."""
        if self._sig_pending is not None or self._verified or not dp_active():
            return
        sig = torch.tensor(self.layout_signature(), dtype=torch.int64)
        outs = [torch.empty_like(sig) for _ in range(dist.get_world_size())]
        work = dist.all_gather(outs, sig, group=signature_group(), async_op=True)
        self._sig_pending = (sig, outs, work)

    def verify_layout(self):
        """Before the first collective of a step: every rank's signature must equal this rank's -- otherwise every
        rank raises here (each sees all signatures) instead of entering collectives of different sizes, which
        would hang or sum unrelated memory.  Without a posted check (no forward went through the rasterizer) the
        exchange is made here, synchronously.  Every rank makes exactly one exchange per step, so a rank that
        rebuilt its slab (a densification on that rank only) cannot leave the signature group's collectives
        paired across different steps."""
        if self._verified or not dp_active():
            return
        if self._sig_pending is None:
            self.post_layout_check()
        sig, outs, work = self._sig_pending
        self._sig_pending = None
        self._verified = True
        work.wait()
        if any(not torch.equal(o, sig) for o in outs):
            raise RuntimeError("FlatGrads: the data-parallel ranks' gradient slabs differ (per rank [numel, "
                               f"params, shapes hash, bucket floats, SH views]: {[o.tolist() for o in outs]}); "
                               "every rank must hold the same Gaussians (densify on every rank) and settings")
        if sig.tolist() != self.layout_signature():
            raise RuntimeError("FlatGrads: this rank's gradient slab changed between the forward's layout check and "
                               "the step's collectives")

    def successor(self, params, device=None):
        """The slab replacing this one after a layout change (FusedAdam.rebuild: densification): this one's hooks
        removed, the new one stale (no gradient yet) and holding this step's layout-check state, so the rank still
        makes exactly one exchange per step -- a check posted before the change then fails on this rank."""
        self.remove_hooks()
        new = FlatGrads(params, device=device)
        new.invalidate()
        new._sig_pending, self._sig_pending = self._sig_pending, None
        new._verified = self._verified
        return new

    def _fused_guard(self, ids):
        if self.fused.intersection(ids) or self.early_ids.intersection(ids):
            raise RuntimeError("FlatGrads: a second gradient for a parameter whose Adam step already ran inside "
                               "the backward (FusedAdam.step_in_backward); leave it out of that block")

    def _before_accumulate(self, p):
        def hook(grad):
            if grad is None:   # a fused HIP backward wrote the .grad in place (it returns None to autograd)
                return grad
            self._fused_guard([id(p)])
            if id(p) in self.stale:
                self._view_of[id(p)].zero_()
                self.stale.discard(id(p))
            return grad
        return hook

    def remove_hooks(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []

    def attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v
            p._gsd_inplace_grad = True  # fused HIP backwards may add into this .grad directly
            p._gsd_flat = self

    def zero(self):
        self.drain_early()
        self.slab.zero_()
        self.stale.clear()
        self.reduced = set()
        self.addends = {}
        self.attach()
        self._verified = False   # a new step: its layout check is still to come

    def invalidate(self):
        """Mark every view stale (no memory traffic): the next gradient producer stores instead of adding."""
        self.drain_early()
        self.stale = {id(p) for p in self.params}
        self.reduced = set()
        self.addends = {}
        self._version = self.slab._version
        self._verified = False   # a new step: its layout check is still to come

    def add_after_reduce(self, p, t):
        """A term of ``p``'s gradient that is already the sum over every rank (gsd_sh_grad_views_ex's view-direction
        term of the means, from the exchanged SH views): it joins the gradient after the all-reduce of the ranks'
        own parts -- added by ``allreduce``, or handed to the consumer of ``allreduce_buckets`` (FusedAdam adds it
        inside its Adam pass: addend_ranges)."""
        if id(p) not in self._view_of or id(p) in self.addends:
            raise RuntimeError("add_after_reduce: parameter not in this slab, or already given an addend this step")
        if t.numel() != p.numel() or not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError("add_after_reduce: the addend must be a contiguous float32 tensor of p's size")
        self.addends[id(p)] = t

    def addend_ranges(self):
        """[(a, b, tensor)]: the slab ranges of the pending addends (consumed: the caller adds them)."""
        out, off = [], 0
        for p, v in zip(self.params, self.views):
            n = v.numel()
            if id(p) in self.addends:
                out.append((off, off + n, self.addends[id(p)].reshape(-1)))
            off += n
        self.addends = {}
        return out

    def _apply_addends(self):
        for a, b, t in self.addend_ranges():
            self.slab[a:b].add_(t)

    def claim(self, params) -> bool:
        """A fused backward is about to produce the gradients of ``params`` in place: True = add into the
        views, False = store (they were all stale).  A mix zeroes the stale ones and adds."""
        ids = [id(p) for p in params]
        self._fused_guard(ids)
        fresh = [i for i in ids if i in self.stale]
        if fresh and len(fresh) == len(ids):
            self.stale.difference_update(ids)
            return False
        for i in fresh:
            self._view_of[i].zero_()
            self.stale.discard(i)
        return True

    def settle(self):
        """Before the gradients are consumed: views nothing wrote since ``invalidate`` hold zero gradient --
        unless no backward ran at all and the slab was written in place (gradients set by hand, e.g.
        ``p.grad.copy_(g)``), which then stand as written.  Returns the ids of the parameters that got no
        gradient (torch's ``p.grad is None`` after ``zero_grad(set_to_none=True)``): their views are zeroed (so a
        collective sums zeros for them) but stay stale -- still "no gradient" until a producer writes them."""
        if len(self.stale) == len(self.params) and self.slab._version != getattr(self, "_version", None):
            self.stale.clear()
            self.missing = set()
            return self.missing
        for i in self.stale:
            self._view_of[i].zero_()
        self._version = self.slab._version   # the zeroing above is not a hand-written gradient
        self.missing = set(self.stale)
        return self.missing

    def collect(self):
        """Copy any .grad autograd replaced (instead of accumulating in place) back into the slab."""
        for p, v in zip(self.params, self.views):
            if p.grad is not None and p.grad.data_ptr() != v.data_ptr():
                v.copy_(p.grad)
                p.grad = v
                self.stale.discard(id(p))

    def early_allreduce(self, params, bucket_floats: int = BUCKET_FLOATS):
        """Start the all-reduce of ``params``' views now, from inside the backward that produced their final
        per-rank gradients (FusedAdam.step_in_backward guards them against a second producer), so that it runs
        on the links while the device computes what is left of the backward.  The views count as reduced for
        this step; allreduce / allreduce_buckets hand their works to the consumer instead of reducing again."""
        if not dp_active():
            return
        ids = {id(p) for p in params}
        if not ids <= set(self._view_of) or ids & self.early_ids:
            raise RuntimeError("early_allreduce: parameters not in this slab, or already reduced this step")
        self.verify_layout()
        keep = [p for p in self.params if id(p) not in ids]
        nccl = dist.get_backend() == "nccl" or not self.slab.is_cuda
        for a, b in self._runs({id(p) for p in keep}):
            for c in range(a, b, max(1, int(bucket_floats))):
                d = min(b, c + int(bucket_floats))
                if nccl:
                    self.early.append((c, d, dist.all_reduce(self.slab[c:d], op=dist.ReduceOp.SUM, async_op=True)))
                else:   # gloo on device tensors (tests): through host memory, synchronously
                    h = self.slab[c:d].cpu()
                    dist.all_reduce(h, op=dist.ReduceOp.SUM)
                    self.slab[c:d].copy_(h)
                    self.early.append((c, d, None))
        self.early_ids |= ids

    def drain_early(self):
        """Order the current stream behind any early all-reduce still in flight and forget them."""
        for _, _, w in self.early:
            if w is not None:
                w.wait()
        self.early, self.early_ids = [], set()

    def _runs(self, reduced):
        """Contiguous slab ranges [a, b) of the views not in ``reduced``."""
        runs, off = [], 0
        for p, v in zip(self.params, self.views):
            n = v.numel()
            if id(p) not in reduced:
                if runs and runs[-1][1] == off:
                    runs[-1][1] = off + n
                else:
                    runs.append([off, off + n])
            off += n
        return runs

    def allreduce(self, op=None, async_op=False):
        """Sum the slab across ranks (no-op for world size 1): one all-reduce per contiguous run of views not
        already summed (mark_reduced -- e.g. the SH gradient the rasterizer assembled from every view)."""
        self.collect()
        self.settle()
        reduced, self.reduced = self.reduced | self.early_ids, set()
        early = [w for _, _, w in self.early if w is not None]
        self.early, self.early_ids = [], set()
        if not dp_active():
            self._apply_addends()
            return None
        self.verify_layout()
        if async_op and self.addends:
            raise RuntimeError("FlatGrads.allreduce(async_op=True): pending addends need the reduced sums first")
        if not async_op:
            for w in early:
                w.wait()
        runs = self._runs(reduced)
        if dist.get_backend() != "nccl" and self.slab.is_cuda:   # gloo (tests): through host memory
            for a, b in runs:
                h = self.slab[a:b].cpu()
                dist.all_reduce(h, op=op or dist.ReduceOp.SUM)
                self.slab[a:b].copy_(h)
            self._apply_addends()
            return None
        works = [dist.all_reduce(self.slab[a:b], op=op or dist.ReduceOp.SUM, async_op=async_op) for a, b in runs]
        if async_op:
            return early + works
        self._apply_addends()
        return None

    def allreduce_buckets(self, bucket_floats: int = BUCKET_FLOATS):
        """The all-reduce of ``allreduce`` issued asynchronously in buckets of at most ``bucket_floats``, for
        a consumer that works through the slab while the later buckets are still on the links
        (FusedAdam.allreduce_step).  Returns [(a, b, work)] covering the whole slab in order: work is None for
        a range that needs no reduction (world size 1, or views already summed) or was reduced synchronously
        (gloo); otherwise the caller waits on it (``work.wait()`` only orders the current stream behind the
        collective, the host does not block).  Pending addends (add_after_reduce) stay for the caller:
        ``addend_ranges``."""
        self.collect()
        self.settle()
        reduced, self.reduced = self.reduced | self.early_ids, set()
        early, self.early, self.early_ids = self.early, [], set()
        n = self.slab.numel()
        if not dp_active():
            return [(0, n, None)]
        self.verify_layout()
        work = list(early)   # ranges whose all-reduce went out inside the backward (early_allreduce)
        nccl = dist.get_backend() == "nccl" or not self.slab.is_cuda
        for a, b in self._runs(reduced):
            for c in range(a, b, max(1, int(bucket_floats))):
                d = min(b, c + int(bucket_floats))
                if nccl:
                    work.append((c, d, dist.all_reduce(self.slab[c:d], op=dist.ReduceOp.SUM, async_op=True)))
                else:   # gloo on device tensors (tests): through host memory, synchronously
                    h = self.slab[c:d].cpu()
                    dist.all_reduce(h, op=dist.ReduceOp.SUM)
                    self.slab[c:d].copy_(h)
                    work.append((c, d, None))
        out, pos = [], 0
        for a, b, w in sorted(work, key=lambda t: t[0]):
            if a > pos:
                out.append((pos, a, None))
            out.append((a, b, w))
            pos = b
        if pos < n:
            out.append((pos, n, None))
        return out


def allreduce_(t: torch.Tensor, op=None) -> torch.Tensor:
    """In-place all-reduce of ``t`` over the default group (no-op at world size 1); gloo with a device tensor
    (the tests) goes through host memory."""
    if not dp_active():
        return t
    op = op or dist.ReduceOp.SUM
    if dist.get_backend() != "nccl" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """In-place broadcast of ``t`` from rank ``src`` (no-op at world size 1)."""
    if not dp_active():
        return t
    if dist.get_backend() != "nccl" and t.is_cuda:
        h = t.cpu()
        dist.broadcast(h, src)
        t.copy_(h)
    else:
        dist.broadcast(t, src)
    return t


def view_stats_allreduce(visible_count: torch.Tensor, grad2d_norm_sum: torch.Tensor, max_radii: torch.Tensor,
                         grad_3vec_sum: torch.Tensor | None = None):
    """Per-view densification statistics (gaussian_model.py:1252-1257, train.py:613),
    combined across ranks after each rank has accumulated its own views: sums for
    the counts / norm sums, max for the radii."""
    if dp_active():
        allreduce_(visible_count)
        allreduce_(grad2d_norm_sum)
        if grad_3vec_sum is not None:
            allreduce_(grad_3vec_sum)
        allreduce_(max_radii, dist.ReduceOp.MAX)
    return visible_count, grad2d_norm_sum, max_radii
