"""The producer of the per-Gaussian offsets: the reference's live deformation network
``DirectTemporalNeRF`` (scene/gaussian_model.py:242-316, with the NeRF positional encoding of :33-82).

Inputs: canonical means (P,3) and a per-view time (P,1, one value); the encoding maps x to
[x, sin(2^k x), cos(2^k x)]_{k<10} (63 channels) and t likewise (21); an 8-layer, 256-wide ReLU MLP with the
encoded x re-injected after layer 4 feeds four linear heads: dx (3), d log-scale (3), d quaternion (4) and
dSH (48).  Before iteration 3000 the reference returns zeros (:302-307).  The module keeps the reference's
parameter names and shapes (``_time.{0..7}``, ``_time_out``, ``_time_out_scale``, ``_time_out_rot``,
``_time_out_shs``), so ``offset_model.pth`` state dicts load as they are (``torch.load(...,
weights_only=True)``).  Its output plugs into ``render()`` as ``pc.offset_model`` and reaches the fused
preamble / split-SH rasterizer directly.

The ≈511k multiply-adds per Gaussian are GEMMs.  In float32 (the reference's training precision) on a HIP device
they run on the hand-written training path (gsd_mlp_train.hip): forward and backward, each GEMM on the bf16
matrix cores with its f32 operands split into three bf16 terms (BF16x6, f32-level accuracy).  ``dtype=
torch.bfloat16`` keeps autocast semantics: the fused bf16 forward kernel without autograd (gsd_mlp.hip), torch /
hipBLASLt GEMMs with autograd.  GSD_MLP_TORCH=1 forces the torch path (the reference's structure, f32 GEMMs).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn


# Weight gradients reduce over all P rows (K = P, a 256 x 256 output): one GEMM of that shape gets ~16 output
# tiles -- 16 workgroups on 256 CUs (hipBLASLt picked MT64x64x256 / MT32x64x128 without split-K: 1.8-2.3 ms per
# layer at P = 1M).  Split-K by hand instead: a batched GEMM over row chunks, then a sum over the chunks.
_SPLITK_ROWS = 8192


def _weight_grad(g: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    """g^T h summed over the rows, as float32: (N, out), (N, in) -> (out, in)."""
    N = g.shape[0]
    S = N // _SPLITK_ROWS
    if S < 2:
        return (g.t() @ h).float()
    main = S * _SPLITK_ROWS
    dw = torch.bmm(g[:main].view(S, _SPLITK_ROWS, -1).transpose(1, 2), h[:main].view(S, _SPLITK_ROWS, -1))
    dw = dw.sum(0, dtype=torch.float32)
    if main < N:
        dw += (g[main:].t() @ h[main:]).float()
    return dw


_RELU_ROWS = 512   # rows per workgroup of gsd_relu_backward_bias


def _relu_bias_backward(gy: torch.Tensor, y):
    """(g, db) on a HIP device in one pass (gsd_relu_backward_bias): g = gy where y > 0 (y None: gy) and the bias
    gradient db = column sums of g in float32 (per-block partials summed in a fixed order)."""
    from . import _native
    from ._C import _ptr, _stream
    lib = _native.load()
    P, N = gy.shape
    gy = gy.contiguous()
    y = None if y is None else y.contiguous()
    g = torch.empty_like(gy)
    part = torch.empty(lib.gsd_relu_backward_bias_blocks(P, _RELU_ROWS), N, dtype=torch.float32, device=gy.device)
    with torch.cuda.device(gy.device):
        _native.check(lib.gsd_relu_backward_bias(P, N, int(gy.dtype == torch.bfloat16), _ptr(gy), _ptr(y), _ptr(g),
                                                 _ptr(part), _RELU_ROWS, _stream(gy.device)))
    return g, part.sum(0)


class _Linear(torch.autograd.Function):
    """y = h W^T + b (then ReLU when `relu`), in h's dtype (f32 or bf16; W and b cast to it), with the split-K
    weight gradient above; dW and db come back in float32 (the parameters' dtype)."""

    @staticmethod
    def forward(ctx, h, W, b, relu):
        Wc, bc = W.to(h.dtype), b.to(h.dtype)
        # bias and ReLU in the GEMM's epilogue (hipBLASLt) where torch offers it
        y = torch._addmm_activation(bc, h, Wc.t()) if relu else torch.addmm(bc, h, Wc.t())
        ctx.relu = relu
        ctx.save_for_backward(h, Wc, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, Wc, y = ctx.saved_tensors
        gy = gy.to(h.dtype)
        if (gy.is_cuda and gy.dtype in (torch.float32, torch.bfloat16) and gy.dim() == 2 and gy.shape[1] % 2 == 0
                and gy.shape[1] <= 512):
            g, db = _relu_bias_backward(gy, y if ctx.relu else None)   # mask + bias gradient, one HIP pass
        else:
            g = torch.ops.aten.threshold_backward(gy, y, 0) if ctx.relu else gy.contiguous()
            db = g.sum(0, dtype=torch.float32)
        dh = g @ Wc if ctx.needs_input_grad[0] else None
        dW = _weight_grad(g, h) if ctx.needs_input_grad[1] else None
        db = db if ctx.needs_input_grad[2] else None
        return dh, dW, db, None


# ---- the fused bf16 forward (gsd_mlp.hip via gsd_deform_mlp_forward_bf16) ----
# Inside each 16-wide k-step the kernel's B operand (the previous layer's accumulator registers) holds, at logical
# position p = 8 h + j, feature 8 (j >> 2) + 4 h + (j & 3): the weights' input columns are permuted to match.
_PERM16 = (0, 1, 2, 3, 8, 9, 10, 11, 4, 5, 6, 7, 12, 13, 14, 15)


def _perm_cols(W: torch.Tensor) -> torch.Tensor:
    n = W.shape[1]
    idx = torch.arange(n, device=W.device).view(-1, 16)[:, list(_PERM16)].reshape(-1)
    return W[:, idx]


def _frag_major(W: torch.Tensor) -> torch.Tensor:
    """(RB*32, KS*16) -> [ks][rb][lane = 32 h + r][j] = W[32 rb + r][16 ks + 8 h + j], bf16."""
    M, K = W.shape
    RB, KS = M // 32, K // 16
    return W.to(torch.bfloat16).view(RB, 32, KS, 2, 8).permute(2, 0, 3, 1, 4).reshape(-1)


def _lane_bias(b: torch.Tensor, rows: int) -> torch.Tensor:
    """b padded to `rows`, rounded to bf16 (autocast's bias), as [rb][h][reg] = b[32 rb + (reg&3) + 8 (reg>>2) + 4 h]."""
    dev = b.device
    bp = torch.zeros(rows, dtype=torch.float32, device=dev)
    bp[: b.numel()] = b.detach().to(torch.bfloat16).float()
    reg = torch.arange(16, device=dev)
    row = (32 * torch.arange(rows // 32, device=dev)[:, None, None] + 4 * torch.arange(2, device=dev)[None, :, None]
           + ((reg & 3) + 8 * (reg >> 2))[None, None, :])
    return bp[row.reshape(-1)]


@torch.no_grad()
def pack_fused_mlp(net: "DirectTemporalNeRF"):
    """The network's weights and biases in the layout gsd_deform_mlp_forward_bf16 reads (gsd_mlp.hip): nine
    layers (8 hidden, the heads as one 58 -> 64-row GEMM), K padded to 16, fragment-major bf16."""
    hid = list(net._time)
    Ws, bs = [], []
    W0 = hid[0].weight
    Ws.append(torch.cat((W0, W0.new_zeros(W0.shape[0], 96 - W0.shape[1])), 1))
    bs.append(hid[0].bias)
    for i in range(1, len(hid)):
        W = hid[i].weight
        if i - 1 in net.skips:   # cat(enc(x) 63, h): the encoding in natural order, one zero column, h permuted
            W = torch.cat((W[:, :63], W.new_zeros(W.shape[0], 1), _perm_cols(W[:, 63:])), 1)
        else:
            W = _perm_cols(W)
        Ws.append(W)
        bs.append(hid[i].bias)
    heads = (net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs)
    Wh = _perm_cols(torch.cat([m.weight for m in heads], 0))
    Ws.append(torch.cat((Wh, Wh.new_zeros(64 - Wh.shape[0], Wh.shape[1])), 0))
    bs.append(torch.cat([m.bias for m in heads], 0))
    frags = torch.cat([_frag_major(W) for W in Ws])
    bias = torch.cat([_lane_bias(b, W.shape[0]) for W, b in zip(Ws, bs)])
    return frags.contiguous(), bias.contiguous()


def _fused_forward(net: "DirectTemporalNeRF", x: torch.Tensor, ts: torch.Tensor):
    from . import _native
    from ._C import _ptr, _stream
    lib = _native.load()
    P = x.shape[0]
    key = tuple((p.data_ptr(), p._version) for p in net.parameters())
    if getattr(net, "_fused_key", None) != key:   # repacked when a parameter changed (optimizer step, load)
        net._fused_pack = pack_fused_mlp(net)
        net._fused_key = key
    frags, bias = net._fused_pack
    if frags.numel() != 8 * lib.gsd_deform_mlp_fragments() or bias.numel() != lib.gsd_deform_mlp_biases():
        raise RuntimeError("deform_mlp: packed layout does not match the library")
    xc = x.detach().to(torch.float32).contiguous()
    tc = ts.detach().to(torch.float32).reshape(-1).expand(P).contiguous()
    outs = tuple(torch.empty(P, n, dtype=torch.float32, device=x.device) for n in (3, 3, 4, 48))
    with torch.cuda.device(x.device):
        _native.check(lib.gsd_deform_mlp_forward_bf16(P, _ptr(xc), _ptr(tc), _ptr(frags), _ptr(bias),
                                                      *(_ptr(o) for o in outs), _stream(x.device)))
    return outs


# ---- the f32-accurate training path (gsd_mlp_train.hip via gsd_deform_mlp_train_forward / _backward) ----
def _param_list(net: "DirectTemporalNeRF"):
    """The reference's 12 weights and 12 biases in the C-ABI's order (_time.0-7, _time_out, _scale, _rot, _shs)."""
    mods = list(net._time) + [net._time_out, net._time_out_scale, net._time_out_rot, net._time_out_shs]
    return [m.weight for m in mods], [m.bias for m in mods]


def _ptr_array(ts):
    import ctypes
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


_HEADS = (3, 3, 4, 48)   # dx, d log-scale, d quaternion, dSH


class _MLPTrainF32(torch.autograd.Function):
    """DirectTemporalNeRF forward + backward as the reference trains it (float32 with autograd), each GEMM on the
    bf16 matrix cores with the operands split into three bf16 terms (BF16x6, f32-level accuracy): three HIP
    kernels per layer direction instead of torch's GEMMs, every activation kept feature-major in one workspace.
    The four heads come out as separate tensors (no (P, 58) array to split and copy, and autograd concatenates no
    gradients for the backward, which reads the four gradients -- a missing one as zero -- in place).  Parameters
    (and x) whose .grad is a FlatGrads view get their gradients written there by the backward (stored when the view
    is stale, added otherwise: autograd's accumulation without a zero-fill and an add kernel per parameter)."""

    @staticmethod
    def forward(ctx, x, t, *params):
        from . import _native
        from ._C import _ptr, _stream
        lib = _native.load()
        P = int(x.shape[0])
        dev = x.device
        ws_, bs_ = list(params[:12]), list(params[12:])
        wc = [w.detach().contiguous() for w in ws_]
        bc = [b.detach().contiguous() for b in bs_]
        if any(w.dtype != torch.float32 or w.device != dev for w in wc + bc):
            raise RuntimeError("deform_mlp: the f32 training path needs float32 parameters on the input's device")
        xc = x.detach().to(torch.float32).contiguous()
        tc = t.detach().to(torch.float32).reshape(-1).expand(P).contiguous()
        ws = torch.empty(lib.gsd_deform_mlp_train_workspace_bytes(P), dtype=torch.uint8, device=dev)
        heads = [torch.empty(P, n, dtype=torch.float32, device=dev) for n in _HEADS]
        with torch.cuda.device(dev):
            _native.check(lib.gsd_deform_mlp_train_forward_heads(P, _ptr(xc), _ptr(tc), _ptr_array(wc),
                                                                 _ptr_array(bc), _ptr(ws), _ptr_array(heads),
                                                                 _stream(dev)))
        ctx.ws, ctx.wc, ctx.P = ws, wc, P
        ctx.shapes = [w.shape for w in wc] + [b.shape for b in bc]
        ctx.x, ctx.params = x, params
        ctx.set_materialize_grads(False)
        # saved for autograd's version check: an in-place optimizer step between this forward and its backward
        # (the activations in ws would then belong to other weights) raises instead of mixing them
        ctx.save_for_backward(*params)
        return tuple(heads)

    @staticmethod
    def backward(ctx, *g_heads):
        from . import _native
        from ._C import _ptr, _stream
        from .activate import _sinks
        lib = _native.load()
        if ctx.ws is None:
            raise RuntimeError("deform_mlp: backward through the f32 training path called a second time (its "
                               "workspace is released by the first; retain_graph is not supported)")
        ctx.saved_tensors   # noqa: B018 -- raises if a parameter was modified in place since the forward
        P, dev = ctx.P, ctx.ws.device
        gh = [None if g is None else g.detach().to(torch.float32).contiguous() for g in g_heads]
        if all(g is None for g in gh):
            ctx.ws = None
            return (None,) * (2 + len(ctx.params))
        # FlatGrads sinks for the parameters (all or none) and for x
        sinks, acc = _sinks(list(ctx.params)) if all(p.requires_grad for p in ctx.params) else (None, True)
        xs, xacc = (_sinks([ctx.x]) if ctx.needs_input_grad[0] else (None, True))
        if sinks is not None:
            dW, db = sinks[:12], sinks[12:]
        else:
            dW = [torch.empty(sh, dtype=torch.float32, device=dev) for sh in ctx.shapes[:12]]
            db = [torch.empty(sh, dtype=torch.float32, device=dev) for sh in ctx.shapes[12:]]
            acc = False
        if xs is not None:
            dx = xs[0]
        else:
            dx = torch.empty(P, 3, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
            xacc = False
        gptr = (_native.ctypes.c_void_p * 4)(*[None if g is None else g.data_ptr() for g in gh])
        with torch.cuda.device(dev):
            _native.check(lib.gsd_deform_mlp_train_backward_heads(
                P, gptr, _ptr_array(ctx.wc), _ptr(ctx.ws), None if dx is None else _ptr(dx), int(bool(xacc)),
                _ptr_array(dW), _ptr_array(db), int(bool(acc)), _stream(dev)))
        ctx.ws = None
        gx = None if (xs is not None or dx is None) else dx
        gp = (None,) * len(ctx.params) if sinks is not None else (*dW, *db)
        return (gx, None, *gp)


def _train_forward(net: "DirectTemporalNeRF", x: torch.Tensor, ts: torch.Tensor):
    ws, bs = _param_list(net)
    return _MLPTrainF32.apply(x, ts, *ws, *bs)


@torch.no_grad()
def _eval_forward_f32(net: "DirectTemporalNeRF", x: torch.Tensor, ts: torch.Tensor):
    """The f32 network without autograd (render.py:46 renders under torch.no_grad(), gaussian_model.py:290-316):
    gsd_deform_mlp_eval_forward_heads -- the training forward's layer-fused BF16x6 kernel without its hidden-output
    stores, and a workspace of the packed weights and the encoding only (~0.4 KB per Gaussian, freed on return)."""
    from . import _native
    from ._C import _ptr, _stream
    lib = _native.load()
    P = int(x.shape[0])
    dev = x.device
    ws_, bs_ = _param_list(net)
    wc = [w.detach().contiguous() for w in ws_]
    bc = [b.detach().contiguous() for b in bs_]
    xc = x.detach().to(torch.float32).contiguous()
    tc = ts.detach().to(torch.float32).reshape(-1).expand(P).contiguous()
    ws = torch.empty(lib.gsd_deform_mlp_eval_workspace_bytes(P), dtype=torch.uint8, device=dev)
    heads = [torch.empty(P, n, dtype=torch.float32, device=dev) for n in _HEADS]
    with torch.cuda.device(dev):
        _native.check(lib.gsd_deform_mlp_eval_forward_heads(P, _ptr(xc), _ptr(tc), _ptr_array(wc), _ptr_array(bc),
                                                            _ptr(ws), _ptr_array(heads), _stream(dev)))
    return tuple(heads)


def positional_encoding(x: torch.Tensor, n_freqs: int = 10) -> torch.Tensor:
    """[x, sin(x 2^0), cos(x 2^0), ..., sin(x 2^(n-1)), cos(x 2^(n-1))] (gaussian_model.py:33-82, log sampling)."""
    freqs = 2.0 ** torch.linspace(0.0, n_freqs - 1, steps=n_freqs, device=x.device)
    xf = x[..., None, :] * freqs[:, None]                       # (P, n, d)
    sc = torch.stack((torch.sin(xf), torch.cos(xf)), dim=-2)     # (P, n, 2, d)
    return torch.cat((x, sc.flatten(start_dim=-3)), dim=-1)


class DirectTemporalNeRF(nn.Module):
    def __init__(self, D: int = 8, W: int = 256, n_freqs: int = 10, skips=(4,), zero_before: int = 3000,
                 dtype: torch.dtype = torch.float32):
        super().__init__()
        self.D, self.W, self.n_freqs, self.skips = D, W, n_freqs, tuple(skips)
        self.zero_before = zero_before
        self.compute_dtype = dtype
        self.input_ch = 3 * (1 + 2 * n_freqs)        # 63
        self.input_ch_time = 1 * (1 + 2 * n_freqs)   # 21
        layers = [nn.Linear(self.input_ch + self.input_ch_time, W)]
        for i in range(D - 1):
            layers.append(nn.Linear(W + (self.input_ch if i in self.skips else 0), W))
        self._time = nn.ModuleList(layers)
        self._time_out = nn.Linear(W, 3)
        self._time_out_scale = nn.Linear(W, 3)
        self._time_out_rot = nn.Linear(W, 4)
        self._time_out_shs = nn.Linear(W, 48)

    def _reference_arch(self) -> bool:
        return (self.D, self.W, self.n_freqs, self.skips) == (8, 256, 10, (4,))

    def _hip_f32(self, x: torch.Tensor) -> bool:
        return (self.compute_dtype == torch.float32 and x.device.type == "cuda" and self._reference_arch()
                and not os.environ.get("GSD_MLP_TORCH") and all(p.dtype == torch.float32 for p in self.parameters())
                and all(p.device == x.device for p in self.parameters()))

    def _needs_grad(self, x: torch.Tensor) -> bool:
        return torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters()))

    def _use_train_f32(self, x: torch.Tensor) -> bool:
        """The f32 network on a HIP device (the reference's training precision) runs the hand-written training
        path (gsd_mlp_train.hip: BF16x6 on the matrix cores, forward and backward) when a backward can follow --
        its forward stores every hidden layer and the backward every layer's gradient (~17 KB per Gaussian).  An
        evaluation (no_grad, or nothing requiring grad) runs the same forward kernel without those stores
        (_eval_forward_f32).  GSD_MLP_TORCH=1 keeps torch for both."""
        return self._needs_grad(x) and self._hip_f32(x)

    def _use_eval_f32(self, x: torch.Tensor) -> bool:
        return not self._needs_grad(x) and self._hip_f32(x)

    def _use_fused(self, x: torch.Tensor) -> bool:
        """The fused bf16 kernel (gsd_mlp.hip) serves the bf16 evaluation without autograd on a HIP device, for
        the reference architecture (8 x 256, skip after layer 4, 10 frequencies); GSD_MLP_TORCH=1 keeps torch."""
        if self.compute_dtype != torch.bfloat16 or x.device.type != "cuda" or os.environ.get("GSD_MLP_TORCH"):
            return False
        if (self.D, self.W, self.n_freqs, self.skips) != (8, 256, 10, (4,)):
            return False
        return not (torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())))

    def forward(self, x: torch.Tensor, ts: torch.Tensor, iteration: int):
        """-> (dx (P,3), d_scale (P,3), d_rot (P,4), d_sh (P,48)) as in gaussian_model.py:290-316."""
        P = x.shape[0]
        if iteration < self.zero_before or P == 0:   # the HIP paths take P >= 1; an empty set has empty heads
            z = x.new_zeros
            return z(P, 3), z(P, 3), z(P, 4), z(P, 48)
        if self._use_fused(x):
            return _fused_forward(self, x, ts)
        if self._use_train_f32(x):
            return _train_forward(self, x, ts)
        if self._use_eval_f32(x):
            return _eval_forward_f32(self, x, ts)
        ex = positional_encoding(x, self.n_freqs)
        et = positional_encoding(ts, self.n_freqs)
        dt = self.compute_dtype if self.compute_dtype != torch.float32 else ex.dtype  # f32: the input's own
        # the hidden layers and the heads in `dt` (as autocast would cast them), bias + ReLU fused after each GEMM;
        # the four heads as one 58-wide GEMM over the concatenated weights
        exd = ex.to(dt)
        h = torch.cat((exd, et.to(dt)), dim=-1)
        for i, layer in enumerate(self._time):
            h = _Linear.apply(h, layer.weight, layer.bias, True)
            if i in self.skips:
                h = torch.cat((exd, h), dim=-1)
        heads = (self._time_out, self._time_out_scale, self._time_out_rot, self._time_out_shs)
        W = torch.cat([m.weight for m in heads], dim=0)
        b = torch.cat([m.bias for m in heads], dim=0)
        o = _Linear.apply(h, W, b, False).float()
        return tuple(t.contiguous() for t in o.split([m.out_features for m in heads], dim=-1))


class DirectTemporalNeRF_se3(nn.Module):
    """The reference's SE(3) twist producer ``DirectTemporalNeRF_se3`` (scene/gaussian_model.py:99-173; dormant in the
    reference's training loop): an 8-layer, 256-wide ReLU MLP on the raw point and time (no positional
    encoding: ``input_ch`` 3 + ``input_ch_time`` 1), the point re-injected after layer 4 (``cat([x, h])``), and two
    linear heads w (3) and v (3).  ``forward`` returns what the reference returns: the (P, 4, 4) transform
    ``exp_se3([w, v] / |w|, |w|)`` (rigid_body.py:86-93) -- the identity where |w| = 0 instead of the reference's NaN
     -- or ``zeros_like(x[:, :4])`` before iteration 3000 (:168-171).  ``twist`` returns the raw (P, 6) [w, v]
    that ``render()``'s SE(3) mode takes (``DeformableGaussians(..., deform="se3", twist_model=net.twist)``): the
    fused HIP exp-map (gsd_deform.hip) normalises it with the same |w| guard and moves means and rotations.

    Parameter names and shapes are the reference's (``_time.{0..7}``, ``_w``, ``_v``), so its state dicts load as
    they are.  In float32 on a HIP device the network runs on DirectTemporalNeRF's training kernels
    (gsd_mlp_train.hip, BF16x6): this architecture IS that one with structurally zero weights -- the raw point is
    channels 0-2 of the positional encoding and the raw time channel 63 of the layer-0 input, the skip layer's
    re-injected point columns 0-2 of its encoding block, and w / v the first two heads (dx, d log-scale) with the
    other heads zero.  Zero weights contribute exact zeros to every f32 accumulation, so the kernels compute this
    network's values; the padded weights are built from the parameters by differentiable concatenation, so autograd
    hands the real entries' gradients back to the parameters and drops the structural zeros'."""

    def __init__(self, D: int = 8, W: int = 256, input_ch: int = 3, input_ch_time: int = 1, skips=(4,),
                 zero_before: int = 3000):
        super().__init__()
        self.D, self.W, self.skips = D, W, tuple(skips)
        self.input_ch, self.input_ch_time = input_ch, input_ch_time
        self.zero_before = zero_before
        layers = [nn.Linear(input_ch + input_ch_time, W)]
        for i in range(D - 1):
            layers.append(nn.Linear(W + (input_ch if i in self.skips else 0), W))
        self._time = nn.ModuleList(layers)
        self._w = nn.Linear(W, 3)
        self._v = nn.Linear(W, 3)

    def _hip_f32(self, x: torch.Tensor) -> bool:
        return ((self.D, self.W, self.skips, self.input_ch, self.input_ch_time) == (8, 256, (4,), 3, 1)
                and x.device.type == "cuda" and not os.environ.get("GSD_MLP_TORCH")
                and all(p.dtype == torch.float32 and p.device == x.device for p in self.parameters()))

    def _padded(self):
        """The twelve weights and biases of the reference-architecture network (DirectTemporalNeRF's C-ABI order)
        that computes this one: see the class docstring."""
        W = self.W
        hid = list(self._time)
        z = lambda r, c, like: like.new_zeros(r, c)  # noqa: E731
        w0 = hid[0].weight   # (W, 4): x 0-2, t 3
        ws = [torch.cat([w0[:, :3], z(W, 60, w0), w0[:, 3:4], z(W, 20, w0)], 1)]
        for i in range(1, self.D):
            w = hid[i].weight
            if (i - 1) in self.skips:   # cat([x, h]): x into the encoding block's first three columns
                w = torch.cat([w[:, :3], z(W, 60, w), w[:, 3:]], 1)
            ws.append(w)
        ref = self._w.weight
        ws += [self._w.weight, self._v.weight, z(4, W, ref), z(48, W, ref)]
        bs = [m.bias for m in hid] + [self._w.bias, self._v.bias, ref.new_zeros(4), ref.new_zeros(48)]
        return ws, bs

    def query_time(self, x: torch.Tensor, ts: torch.Tensor):
        """gaussian_model.py:142-150 -> (w, v), each (P, 3)."""
        if self._hip_f32(x) and x.shape[0] > 0:
            ws, bs = self._padded()
            if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
                heads = _MLPTrainF32.apply(x, ts, *ws, *bs)
            else:
                with torch.no_grad():
                    heads = _MLPTrainF32.apply(x, ts, *[w.detach() for w in ws], *[b.detach() for b in bs])
            return heads[0], heads[1]
        h = torch.cat([x, ts.to(x.dtype).expand(x.shape[0], 1)], dim=-1)
        for i, layer in enumerate(self._time):
            h = torch.relu(layer(h))
            if i in self.skips:
                h = torch.cat([x, h], dim=-1)
        return self._w(h), self._v(h)

    def twist(self, x: torch.Tensor, ts: torch.Tensor, iteration: int) -> torch.Tensor:
        """(P, 6) raw [w, v] for render()'s SE(3) mode; zeros (the identity motion) before iteration 3000."""
        if iteration < self.zero_before:
            return x.new_zeros(x.shape[0], 6)
        w, v = self.query_time(x, ts)
        return torch.cat([w, v], dim=-1)

    def forward(self, x: torch.Tensor, ts: torch.Tensor, iteration: int) -> torch.Tensor:
        """gaussian_model.py:153-173: the (P, 4, 4) transform, or before iteration 3000 the reference's
        ``torch.zeros_like(input_pts[:, :4])`` -- (P, 3) zeros for (P, 3) points, as written."""
        if iteration < self.zero_before:
            return torch.zeros_like(x[:, :4])
        w, v = self.query_time(x, ts)
        return se3_transform(torch.cat([w, v], dim=-1))


def se3_transform(twist: torch.Tensor) -> torch.Tensor:
    """(P, 6) raw [w, v] -> (P, 4, 4) exp_se3 of the unit screw axis [w, v] / |w| by the angle |w|
    (rigid_body.py:61-65, 86-93, gaussian_model.py:161-165): R = I + sin t W + (1 - cos t) W^2,
    p = (t I + (1 - cos t) W + (t - sin t) W^2) v / t, W = skew(w / t); the identity where t = 0."""
    w, v = twist[:, :3], twist[:, 3:]
    th = torch.linalg.vector_norm(w, dim=-1)
    safe = torch.where(th > 0, th, torch.ones_like(th))
    wn, vn = w / safe[:, None], v / safe[:, None]
    Z = torch.zeros_like(th)
    Wm = torch.stack([torch.stack([Z, -wn[:, 2], wn[:, 1]], -1), torch.stack([wn[:, 2], Z, -wn[:, 0]], -1),
                      torch.stack([-wn[:, 1], wn[:, 0], Z], -1)], -2)
    W2 = Wm @ Wm
    s, c = torch.sin(th)[:, None, None], torch.cos(th)[:, None, None]
    eye = torch.eye(3, dtype=twist.dtype, device=twist.device).expand(twist.shape[0], 3, 3)
    R = eye + s * Wm + (1.0 - c) * W2
    t = th[:, None, None]
    p = ((t * eye + (1.0 - c) * Wm + (t - s) * W2) @ vn[:, :, None])[..., 0]
    on = (th > 0)[:, None, None]
    R = torch.where(on, R, eye)
    p = torch.where(on[..., 0], p, torch.zeros_like(p))
    T = torch.zeros(twist.shape[0], 4, 4, dtype=twist.dtype, device=twist.device)
    T[:, :3, :3] = R
    T[:, :3, 3] = p
    T[:, 3, 3] = 1.0
    return T
