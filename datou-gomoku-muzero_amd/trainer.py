"""MuZero training step of the reference on the GPU.

What the reference's trainer computes, per step (loss.py:30-158, workers.py:445-628):
  * 8-fold board augmentation of a sampled batch (one rotation k and flip per batch);
  * n-step value targets from the stored rewards / search values, bootstrapping from the target
    network's value of the last observation once the n-step window leaves the unroll;
  * an unroll of NUM_UNROLL_STEPS dynamics steps from the representation of obs[0]: policy and
    value cross-entropies at every step, reward cross-entropy and a Barlow-twins consistency loss
    (dynamics projection vs projection of the true next representation) per unrolled step, the
    hidden-state gradient halved between steps, steps masked where the game had ended (action -1);
  * PER importance weights, Adam + weight decay, warm-up + cosine LR, gradient clipping, AMP grad
    scaler, soft update of the target network;
  * |value error| at step 0 as the new PER priorities.

Here the same step runs on MI355X through PyTorch-ROCm (MIOpen convolutions, hipBLASLt GEMMs):
``TrainNet`` keeps the reference's parameter names (``network.py:109-123``), so state_dicts move
between the reference, this trainer and the inference engine (``network.GomokuNetHip``) unchanged;
``Trainer`` wraps the optimiser/scheduler/scaler/target-network bookkeeping and, when
torch.distributed is initialised, data parallelism with one flat-bucket gradient all-reduce per step
(RCCL over xGMI);
``ReplayBuffer`` keeps the slices resident in device memory and samples like
replay_buffer.py:58-94 (uniform without replacement, or stratified proportional PER).
The 128->128 residual-block convolutions (forward, input and weight gradients) and every
training-mode BatchNorm run on the HIP kernels of csrc/gmz_conv.hip / csrc/gmz_train.hip; the
trunks' first convolutions, 1x1 convolutions and Linears run on MIOpen / hipBLASLt.
"""
import collections
import math
from dataclasses import dataclass, field, asdict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class TrainConfig:
    """Trainer keys of the reference's config (config.py:57-104)."""
    BOARD_SIZE: int = 15
    NUM_RES_BLOCKS: int = 8
    NUM_FILTERS: int = 128
    HEAD_HIDDEN_DIM: int = 64
    VALUE_SUPPORT_MIN: int = -1
    VALUE_SUPPORT_MAX: int = 1
    VALUE_SUPPORT_BINS: int = 3
    REWARD_SUPPORT_MIN: int = -1
    REWARD_SUPPORT_MAX: int = 1
    REWARD_SUPPORT_BINS: int = 3
    DISCOUNT: float = 0.997
    NUM_UNROLL_STEPS: int = 5
    N_STEPS: int = 10
    PHYSICAL_BATCH_SIZE: int = 360
    GRADIENT_ACCUMULATION_STEPS: int = 1
    LEARNING_RATE: float = 5e-6
    WEIGHT_DECAY: float = 1e-5
    BARLOW_LAMBDA: float = 5e-3
    TARGET_MODEL_TAU: float = 0.995
    GRAD_CLIP_NORM: float = 5.0
    LOSS_WEIGHTS: dict = field(default_factory=lambda: {"policy": 1.0, "value": 1.0, "reward": 0.5,
                                                        "consistency": 5.0})
    TRAIN_BUFFER_SIZE: int = 1000000
    ENABLE_PER: bool = False
    PER_BETA: float = 0.4
    PER_EPSILON: float = 1e-6
    MODEL_UPDATE_INTERVAL: int = 1000

    @property
    def ACTION_SPACE_SIZE(self):
        return self.BOARD_SIZE * self.BOARD_SIZE

    @classmethod
    def from_any(cls, cfg=None, **overrides):
        vals = {}
        if cfg is not None:
            for k in cls.__dataclass_fields__:
                if hasattr(cfg, k):
                    vals[k] = getattr(cfg, k)
        vals.update(overrides)
        return cls(**vals)

    def as_dict(self):
        return asdict(self)


# ------------------------------------------------------------------------------ supports
def support_to_scalar(logits, vmin, vmax, bins):
    """network.py:9-13: expectation of softmax(logits) over linspace(vmin, vmax, bins)."""
    grid = torch.linspace(vmin, vmax, bins, device=logits.device)
    return (F.softmax(logits, dim=1) * grid).sum(dim=1, keepdim=True)


def scalar_to_support(x, vmin, vmax, bins):
    """network.py:15-25: two-hot projection of a clamped scalar onto the support grid; x of any shape
    -> [*x.shape, bins] (elementwise, so a whole [B, steps] block at once gives each column's values)."""
    shape = x.shape
    x = x.reshape(-1).clamp(vmin, vmax)
    pos = (x - vmin) * ((bins - 1) / (vmax - vmin))
    lo, hi = torch.floor(pos).long(), torch.ceil(pos).long()
    w_hi = pos - lo.float()
    out = torch.zeros(x.shape[0], bins, device=x.device)
    out.scatter_add_(1, lo[:, None], (1 - w_hi)[:, None])
    out.scatter_add_(1, hi[:, None], w_hi[:, None])
    return out.view(*shape, bins)


# ------------------------------------------------------------------------------ network
def _bn(mod, x, mask=None, segments=1):
    """``segments`` > 1: x is that many equal row segments (the batched consistency representations), each
    normalised with its own statistics and the running statistics updated segment after segment — exactly
    ``segments`` calls one after the other.
    BatchNorm whose training-mode statistics (and running-stat update) cover only the rows
    where ``mask`` is set.  The reference runs the unrolled steps on the sub-batch of games still
    in progress (loss.py:89-93); running every step on the FULL batch with row-masked statistics
    gives the same values and gradients with fixed shapes (MIOpen compiles each convolution once
    instead of once per sub-batch size) and without a host synchronisation (no boolean gather),
    so a whole training step can be captured in one HIP graph.  ``mask``: bool [B].  Computed in
    float32 (as autocast runs BatchNorm).  A mask with no row set leaves the running statistics
    untouched (the reference skips such a step)."""
    if segments > 1 and mod.training:
        xs = x.chunk(segments)
        ms = mask.chunk(segments) if mask is not None else [None] * segments
        return torch.cat([_bn(mod, a, m) for a, m in zip(xs, ms)])
    if mask is None or not mod.training:
        return mod(x)
    if SUBBATCH_BN:  # diagnostics: the reference's own computation, native BatchNorm on the gathered live rows
        idx = mask.nonzero().squeeze(1)
        if idx.numel() == 0:
            return x * 0
        ys = mod(x.index_select(0, idx))
        return torch.zeros(x.shape, dtype=ys.dtype, device=x.device).index_copy(0, idx, ys)
    x = x.float()
    dims = [0] + list(range(2, x.dim()))
    shape = [1, -1] + [1] * (x.dim() - 2)
    w = mask.to(torch.float32).reshape([-1] + [1] * (x.dim() - 1))
    nv = mask.sum()
    n = nv.to(torch.float32) * (x[0, 0].numel())
    ns = n.clamp(min=1.0)
    mean = (x * w).sum(dim=dims) / ns                  # statistics of the valid rows only
    xc = x - mean.reshape(shape)
    var = (xc * xc * w).sum(dim=dims) / ns
    scale = torch.rsqrt(var + mod.eps) * mod.weight
    y = torch.addcmul(mod.bias.reshape(shape), xc, scale.reshape(shape))
    with torch.no_grad():  # through .data, like the native kernel: no autograd version bump (the
        m = mod.momentum      # unmasked BatchNorm calls of the same module saved these buffers)
        ok = nv > 0
        rm, rv = mod.running_mean.data, mod.running_var.data
        rm.copy_(torch.where(ok, rm * (1 - m) + m * mean.detach(), rm))
        rv.copy_(torch.where(ok, rv * (1 - m) + m * var.detach() * n / (n - 1).clamp(min=1.0), rv))
        mod.num_batches_tracked.data += ok.to(mod.num_batches_tracked.dtype)
    return y


# diagnostics only (tools/trainer_ragged_diag.py, tests): _bn runs the reference's sub-batch BatchNorm — the
# live rows gathered (h[m], loss.py:89-93) through the native module, in the activation dtype (float16
# under autocast, as the reference's AMP on CUDA) — instead of the row-masked float32 statistics
SUBBATCH_BN = False
_BN_DTYPES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
FUSED_BN = True  # device BatchNorm layers of a training-mode model run the HIP kernels (gmz_train.hip)
# the backward's dz sums of a channels-last BatchNorm whose output feeds a HIP 3x3 conv reduced in that conv's
# input-gradient epilogue (gmz_conv3x3_forward_bwdstats -> gmz_bn_backward_stats): no reduction pass of its own.
# Measured (profiles/r04_bn_bwd_fused_ab.txt): the BatchNorm backward 34.6 -> 20.8 us, but the conv's epilogue
# loads of the BN's x and y (not overlapped with its MFMAs) 35.0 -> 48.9 us, and the step 35.0-35.7 vs
# 36.3-36.8 steps/s; off (A/B switch, tested)
FUSED_BN_BWD_STATS = False
# the channels-last BatchNorm + ReLU forward also writes its ReLU's output mask (1 bit per element,
# gmz_bn_forward_m / _stats_m) and the backward reads it instead of re-reading the 16-bit output y in both of its
# passes (gmz_bn_backward_acc_m): 2 x 20 MB fewer reads per 360-board BatchNorm backward.  A/B switch
RELU_MASK = False


def _aligned16(*ts):
    return all(t is None or t.data_ptr() % 16 == 0 for t in ts)


class _BnBwdLink:
    """Hand-off from a training-mode BatchNorm (+ReLU) to the HIP conv that consumes its output y: the BN's
    input x, row mask, saved (mean, invstd) and ReLU flag (the conv saved y itself), and back from that conv's
    backward the dz partials of the gradient it produced for y, ``bwd`` = (stats, slots, that gradient)."""
    __slots__ = ("x", "mask", "save", "relu", "bwd")

    def __init__(self, x, mask, save, relu):
        self.x, self.mask, self.save, self.relu, self.bwd = x, mask, save, relu, None


def _bn_layout(x):
    """0: NCHW-contiguous, 1: channels-last (NHWC) with an even channel count, None: neither."""
    if x.is_contiguous():
        return 0
    if x.dim() == 4 and x.shape[1] % 2 == 0 and x.shape[1] <= 512 and x.is_contiguous(memory_format=torch.channels_last):
        return 1
    return None


def _like(t, layout):
    return t.contiguous(memory_format=torch.channels_last) if layout == 1 else t.contiguous()


# the optimiser step on the GPU as gmz_opt_step (unscale + clip + Adam + soft target update + zero_grad in three
# launches over the flat gradient bucket) instead of PyTorch's unscale_ / clip_grad_norm_ / fused Adam / foreach
# update (A/B: False)
FUSED_OPT = True

# data parallel: the gradient all-reduces captured inside the step's HIP graph (Trainer._capture) when every rank can
# capture a collective; False: three graphs with the all-reduces issued between their replays (A/B, fallback)
GRAPH_ALLREDUCE = True

# a training-mode BatchNorm (+ residual, ReLU) whose output is the input of a HIP 3x3 conv: its elementwise pass runs
# in that conv's board-staging prologue (gmz_conv3x3_forward_bnapply, which also writes the output for the backward)
# instead of a pass of its own: one launch and one read of the BatchNorm's input fewer per use
DEFER_BN_APPLY = True

# every packed 3x3 conv weight the step uses (_packed_conv_weight's caches on the model's and the target's parameters)
# re-packed by ONE gmz_conv3x3_pack_many launch at the top of the step instead of one gmz_conv3x3_pack per weight at
# its first use (87 launches per 15x15 step; A/B: False)
BATCH_REPACK = True


class _PendingBN:
    """A deferred BatchNorm output's recipe, attached to the (not yet written) output tensor as ``_gmz_pending``:
    its input z, residual, gamma, beta, saved (mean, invstd) and ReLU flag.  Only _conv3_apply consumes it."""
    __slots__ = ("z", "res", "gamma", "beta", "save", "relu")

    def __init__(self, z, res, gamma, beta, save, relu):
        self.z, self.res, self.gamma, self.beta, self.save, self.relu = z, res, gamma, beta, save, relu


def _conv_takes_pending(conv, z):
    """True when ``_conv3_apply(conv, y)`` of a training-mode BatchNorm output y of z's shape, dtype and layout
    runs the HIP conv that can apply the BatchNorm in its prologue (the conditions of its single-segment path)."""
    if not (DEFER_BN_APPLY and FUSED_BN and FUSED_CONV and not RELU_MASK and not FUSED_BN_BWD_STATS and z.is_cuda
            and z.dim() == 4 and z.shape[1] == 128 and z.shape[2] == z.shape[3] and z.shape[2] in (9, 15)):
        return False
    if conv.weight.shape != (128, 128, 3, 3) or conv.bias is not None:
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else z.dtype
    return dt == z.dtype and dt in _CONV_DTYPES and z.is_contiguous(memory_format=torch.channels_last)


class _FusedMaskedBN(torch.autograd.Function):
    """Row-masked training-mode BatchNorm + residual + ReLU as three HIP kernels forward and three
    backward (``gmz_bn_forward`` / ``gmz_bn_backward``, csrc/gmz_train.hip), on NCHW or channels-last
    activations.  Same statistics, running-stat update and gradients as ``_bn`` followed by
    ``+ res`` and ``relu``; the output keeps the activation dtype and memory format (float16 under
    the reference's autocast)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, mask, running_mean, running_var, num_batches, eps, momentum, relu,
                stats=None, link=None, bwd_link=False, defer=False):
        from . import _lib
        L = _lib.load()
        layout = _bn_layout(x)
        if layout is None:
            x, layout = x.contiguous(), 0
        if res is not None:
            res = _like(res, layout)
        B, C = x.shape[0], x.shape[1]
        S = x[0, 0].numel()
        y = torch.empty_like(x)
        save = torch.empty(2, C, dtype=torch.float32, device=x.device)
        rmask = None
        if (RELU_MASK and relu and layout == 1 and C % 8 == 0 and x.dtype != torch.float32 and torch.is_grad_enabled()
                and _aligned16(x, res, y) and not (FUSED_BN_BWD_STATS and bwd_link)):
            rmask = torch.empty(B * S * (C // 8), dtype=torch.uint8, device=x.device)
        if defer and layout == 1 and rmask is None and _aligned16(x, res, y):
            # DEFER_BN_APPLY: statistics and running stats now; y is written by the consuming conv's prologue
            # (gmz_conv3x3_forward_bnapply, _conv3_apply), which the caller guarantees comes next
            ws = None if stats is not None else _bn_workspace(1, B, C, S, x.device)
            _lib.check(L.gmz_bn_forward_deferred(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(mask), B, C, S, float(eps),
                                                 float(momentum), _lib.ptr(running_mean), _lib.ptr(running_var),
                                                 _lib.ptr(num_batches), _lib.ptr(save),
                                                 None if stats is None else _lib.ptr(stats[0]),
                                                 0 if stats is None else int(stats[1]),
                                                 0 if stats is None else _lib.nbytes(stats[0]), _lib.ptr(ws),
                                                 _lib.nbytes(ws), _lib.stream_ptr()))
            y._gmz_pending = _PendingBN(x, res, gamma, beta, save, relu)
        elif stats is not None and layout == 1:  # statistics reduced by the producing conv's epilogue
            if rmask is not None:
                _lib.check(L.gmz_bn_forward_stats_m(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(res), B, C, S,
                                                    _lib.ptr(gamma), _lib.ptr(beta), float(eps), float(momentum),
                                                    _lib.ptr(running_mean), _lib.ptr(running_var),
                                                    _lib.ptr(num_batches), int(relu), _lib.ptr(y), _lib.ptr(save),
                                                    _lib.ptr(stats[0]), int(stats[1]), _lib.nbytes(stats[0]),
                                                    _lib.ptr(rmask), _lib.stream_ptr()))
            else:
                _lib.check(L.gmz_bn_forward_stats(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(res), B, C, S,
                                                  _lib.ptr(gamma), _lib.ptr(beta), float(eps), float(momentum),
                                                  _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(num_batches),
                                                  int(relu), _lib.ptr(y), _lib.ptr(save), _lib.ptr(stats[0]),
                                                  int(stats[1]), _lib.nbytes(stats[0]), _lib.stream_ptr()))
        else:
            ws = _bn_workspace(layout, B, C, S, x.device)
            if rmask is not None:
                _lib.check(L.gmz_bn_forward_m(_BN_DTYPES[x.dtype], layout, _lib.ptr(x), _lib.ptr(res), _lib.ptr(mask),
                                              B, C, S, _lib.ptr(gamma), _lib.ptr(beta), float(eps), float(momentum),
                                              _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(num_batches),
                                              int(relu), _lib.ptr(y), _lib.ptr(save), _lib.ptr(ws), _lib.nbytes(ws),
                                              _lib.ptr(rmask), _lib.stream_ptr()))
            else:
                _lib.check(L.gmz_bn_forward(_BN_DTYPES[x.dtype], layout, _lib.ptr(x), _lib.ptr(res), _lib.ptr(mask), B,
                                            C, S, _lib.ptr(gamma), _lib.ptr(beta), float(eps), float(momentum),
                                            _lib.ptr(running_mean), _lib.ptr(running_var), _lib.ptr(num_batches),
                                            int(relu), _lib.ptr(y), _lib.ptr(save), _lib.ptr(ws), _lib.nbytes(ws),
                                            _lib.stream_ptr()))
        ctx.save_for_backward(x, y, mask, gamma, save)
        ctx.relu, ctx.has_res, ctx.layout = relu, res is not None, layout
        ctx.rmask = rmask
        ctx.beta = beta
        ctx.link = link
        ctx.bwd_link = None
        if bwd_link and layout == 1 and x.dtype in _CONV_DTYPES:  # a HIP conv consuming y may reduce our dz sums
            ctx.bwd_link = _BnBwdLink(x, mask, save, relu)
            y._gmz_bnsrc = ctx.bwd_link
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import _lib
        L = _lib.load()
        x, y, mask, gamma, save = ctx.saved_tensors
        layout = ctx.layout
        dy = _like(dy, layout)
        B, C = x.shape[0], x.shape[1]
        S = x[0, 0].numel()
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if ctx.has_res else None
        beta = ctx.beta
        # the parameters' f32 .grad (the trainer's flat-bucket views) take the gradients in place:
        # no gradient tensors, no AccumulateGrad adds (one per BatchNorm use and parameter)
        acc = (gamma.grad is not None and beta.grad is not None and gamma.grad.dtype == torch.float32
               and beta.grad.dtype == torch.float32 and gamma.grad.is_contiguous() and beta.grad.is_contiguous())
        if acc:
            dgamma, dbeta = gamma.grad, beta.grad
        else:
            dgamma = torch.empty(C, dtype=torch.float32, device=x.device)
            dbeta = torch.empty(C, dtype=torch.float32, device=x.device)
        ws = _bn_workspace(layout, B, C, S, x.device)
        bl = ctx.bwd_link
        pre = bl.bwd if bl is not None else None
        if bl is not None:
            bl.bwd = None
        if pre is not None and (pre[2] is dy or (pre[2].data_ptr() == dy.data_ptr() and pre[2].stride() == dy.stride()
                                                 and pre[2].dtype == dy.dtype)):
            # dz sums already reduced by the conv that produced dy (gmz_conv3x3_forward_bwdstats)
            _lib.check(L.gmz_bn_backward_stats(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(y), _lib.ptr(dy),
                                               _lib.ptr(mask), B, C, S, _lib.ptr(gamma), _lib.ptr(save), int(ctx.relu),
                                               _lib.ptr(dx), _lib.ptr(dres), _lib.ptr(dgamma), _lib.ptr(dbeta),
                                               _lib.ptr(pre[0]), int(pre[1]), _lib.nbytes(pre[0]), _lib.ptr(ws),
                                               _lib.nbytes(ws), _lib.stream_ptr(), int(acc)))
        elif ctx.rmask is not None and _aligned16(x, y, dy, dx, dres):
            _lib.check(L.gmz_bn_backward_acc_m(_BN_DTYPES[x.dtype], layout, _lib.ptr(x), _lib.ptr(y), _lib.ptr(dy),
                                               _lib.ptr(mask), B, C, S, _lib.ptr(gamma), _lib.ptr(save), int(ctx.relu),
                                               _lib.ptr(dx), _lib.ptr(dres), _lib.ptr(dgamma), _lib.ptr(dbeta),
                                               _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(ctx.rmask), _lib.stream_ptr(),
                                               int(acc)))
        else:
            _lib.check(L.gmz_bn_backward_acc(_BN_DTYPES[x.dtype], layout, _lib.ptr(x), _lib.ptr(y), _lib.ptr(dy),
                                             _lib.ptr(mask), B, C, S, _lib.ptr(gamma), _lib.ptr(save), int(ctx.relu),
                                             _lib.ptr(dx), _lib.ptr(dres), _lib.ptr(dgamma), _lib.ptr(dbeta),
                                             _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr(), int(acc)))
        ctx.rmask = None
        if ctx.link is not None and dres is not None:
            # the residual's gradient goes to the block's first conv, whose input-gradient epilogue adds it
            # (_ResLink): autograd then has one gradient for the block input, no accumulation pass
            ctx.link.dres, dres = dres, None
        if acc:
            return dx, None, None, dres, None, None, None, None, None, None, None, None, None, None, None
        return dx, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None, None


_WS_BYTES = {}


def _bn_workspace(layout, B, C, S, device):
    import ctypes
    from . import _lib
    key = (layout, B, C, S)
    if key not in _WS_BYTES:
        n = ctypes.c_size_t()
        _lib.check(_lib.load().gmz_bn_workspace_bytes(layout, B, C, S, ctypes.byref(n)))
        _WS_BYTES[key] = n.value
    return torch.empty((_WS_BYTES[key] + 7) // 8, dtype=torch.float64, device=device)


def _bn_act(mod, x, mask=None, res=None, relu=True, link=None, segments=1, consumer=None):
    """relu?(BatchNorm(x) (+ res)) with row-masked training statistics (see ``_bn``).  Training-mode
    BatchNorm on the GPU runs the fused HIP kernels; eval mode and the CPU use PyTorch ops.  ``link``:
    the block's _ResLink, used when ``res`` is the very tensor its first HIP conv consumed.  ``segments``:
    see ``_bn`` (no autograd: the batched consistency representations run under no_grad).  ``consumer``: the
    3x3 conv that consumes the output next — when it can (``_conv_takes_pending``), the output is deferred to its
    prologue (DEFER_BN_APPLY)."""
    if segments > 1 and mod.training:
        if FUSED_BN and x.is_cuda and x.dtype in _BN_DTYPES and _bn_layout(x) == 1 and not torch.is_grad_enabled():
            return _bn_seg(mod, x, mask, res, relu, segments)
        xs = x.chunk(segments)
        ms = mask.chunk(segments) if mask is not None else [None] * segments
        rs = res.chunk(segments) if res is not None else [None] * segments
        return torch.cat([_bn_act(mod, a, m, r, relu) for a, m, r in zip(xs, ms, rs)])
    if FUSED_BN and mod.training and x.is_cuda and x.dtype in _BN_DTYPES:
        if res is not None:
            res = res.to(x.dtype)
        m = None if mask is None else mask.contiguous().view(torch.uint8)
        use = link if (link is not None and res is not None and link.xin is res) else None
        want = FUSED_BN_BWD_STATS and torch.is_grad_enabled() and (x.requires_grad or mod.weight.requires_grad)
        defer = consumer is not None and _conv_takes_pending(consumer, x)
        return _FusedMaskedBN.apply(x, mod.weight, mod.bias, res, m, mod.running_mean, mod.running_var,
                                    mod.num_batches_tracked, mod.eps, mod.momentum, relu,
                                    getattr(x, "_gmz_bnstats", None), use, want, defer)
    if (FUSED_BN and not mod.training and x.is_cuda and x.dtype in _BN_DTYPES and _bn_layout(x) is not None
            and not (torch.is_grad_enabled() and (x.requires_grad or mod.weight.requires_grad))):
        return _bn_eval(mod, x, res, relu)
    y = _bn(mod, x, mask)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


def _bn_seg(mod, x, mask, res, relu, nseg):
    """Training-mode BatchNorm (+ res, ReLU) of ``nseg`` equal row segments of a channels-last activation in one
    pass (``gmz_bn_forward_seg``): segment statistics from the producing conv's per-board partials when it left
    them (``_conv3_apply`` with segments), else one reduction pass; no autograd (no_grad callers only)."""
    from . import _lib
    B, C = x.shape[0], x.shape[1]
    S = x[0, 0].numel()
    if res is not None:
        res = _like(res.to(x.dtype), 1)
    y = torch.empty_like(x)
    save = torch.empty(nseg * 2 * C, dtype=torch.float32, device=x.device)
    ws = _bn_workspace(1, B, C, S, x.device)
    st = getattr(x, "_gmz_bnstats", None)
    board = st[0] if (st is not None and st[1] == "board") else None
    m = None if mask is None else mask.contiguous().view(torch.uint8)
    _lib.check(_lib.load().gmz_bn_forward_seg(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(res), _lib.ptr(m), B, nseg, C,
                                              S, _lib.ptr(mod.weight), _lib.ptr(mod.bias), float(mod.eps),
                                              float(mod.momentum), _lib.ptr(mod.running_mean), _lib.ptr(mod.running_var),
                                              _lib.ptr(mod.num_batches_tracked), int(relu), _lib.ptr(y), _lib.ptr(save),
                                              _lib.ptr(ws), _lib.nbytes(ws), _lib.ptr(board), _lib.nbytes(board),
                                              _lib.stream_ptr()))
    return y


def _bn_eval(mod, x, res, relu):
    """Eval-mode BatchNorm (running statistics) + residual + ReLU as one HIP pass (``gmz_bn_eval``):
    the target network's fp32 forward (loss.py:54-55), no autograd."""
    from . import _lib
    layout = _bn_layout(x)
    if res is not None:
        res = _like(res.to(x.dtype), layout)
    B, C = x.shape[0], x.shape[1]
    S = x[0, 0].numel()
    y = torch.empty_like(x)
    ws = _bn_workspace(layout, B, C, S, x.device)
    _lib.check(_lib.load().gmz_bn_eval(_BN_DTYPES[x.dtype], layout, _lib.ptr(x), _lib.ptr(res), B, C, S,
                                       _lib.ptr(mod.weight), _lib.ptr(mod.bias), _lib.ptr(mod.running_mean),
                                       _lib.ptr(mod.running_var), float(mod.eps), int(relu), _lib.ptr(y),
                                       _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr()))
    return y


def _conv1x1(conv, x):
    """1x1 convolution as a batched GEMM over positions (same parameters as ``conv``).  MIOpen
    has no tuned kernels for the 1- and 2-channel head convolutions and the 1->16 action embedding
    and falls back to naive direct convolutions (tens of ms per weight gradient); as a GEMM they
    take microseconds.  A channels-last input stays channels-last (GEMM over the [n, h*w, c] view)."""
    n, c, h, w = x.shape
    wt = conv.weight.reshape(conv.weight.shape[0], c)
    wt = wt.to(x.dtype) if not torch.is_autocast_enabled() else wt
    if c > 1 and x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        y = _Conv1x1NHWC.apply(x.permute(0, 2, 3, 1).reshape(n, h * w, c), wt)   # [n, s, o]
        if conv.bias is not None:
            y = y + conv.bias.to(y.dtype)
        return y.reshape(n, h, w, -1).permute(0, 3, 1, 2)        # channels-last [n, o, h, w]
    y = _Conv1x1NCHW.apply(x.reshape(n, c, h * w), wt)
    if conv.bias is not None:
        y = y + conv.bias.reshape(1, -1, 1).to(y.dtype)
    return y.reshape(n, -1, h, w)


class _Conv1x1NCHW(torch.autograd.Function):
    """y[n] = W @ x[n] for x [n, c, s], W [o, c].  Autograd of the broadcast matmul folds the
    weight gradient into ONE GEMM with K = n*s = 81,000 and an o x c = 2 x 128 (policy), 1 x 128
    (value) or 16 x 1 (action embedding) output: hipBLASLt runs that on 1-8 workgroups, 0.55-0.63 ms
    each (7 % of a training step).  Here it is a batched GEMM over n (K = s) reduced over n in float32."""

    @staticmethod
    def forward(ctx, x, wt):
        if torch.is_autocast_enabled(x.device.type):
            dt = torch.get_autocast_dtype(x.device.type)
            x, wt = x.to(dt), wt.to(dt)
        ctx.save_for_backward(x, wt)
        return torch.matmul(wt, x)

    @staticmethod
    def backward(ctx, gy):
        x, wt = ctx.saved_tensors
        gy = gy.to(x.dtype)
        gx = torch.matmul(wt.t(), gy) if ctx.needs_input_grad[0] else None
        gw = torch.bmm(gy, x.transpose(1, 2)).sum(0, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        return gx, gw


class _Conv1x1NHWC(torch.autograd.Function):
    """y[n] = x[n] @ W^T for channels-last x [n, s, c], W [o, c]; the weight gradient as a batched
    GEMM over n reduced in float32 (see ``_Conv1x1NCHW``: one GEMM with K = n*s ran on 8 workgroups,
    0.55 ms per call)."""

    @staticmethod
    def forward(ctx, x, wt):
        if torch.is_autocast_enabled(x.device.type):
            dt = torch.get_autocast_dtype(x.device.type)
            x, wt = x.to(dt), wt.to(dt)
        ctx.save_for_backward(x, wt)
        return torch.matmul(x, wt.t())

    @staticmethod
    def backward(ctx, gy):
        x, wt = ctx.saved_tensors
        gy = gy.to(x.dtype)
        gx = torch.matmul(gy, wt) if ctx.needs_input_grad[0] else None
        gw = torch.bmm(gy.transpose(1, 2), x).sum(0, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        return gx, gw


FUSED_CONV = True  # 128->128 3x3 convs of f16/bf16 channels-last activations run gmz_conv3x3 (HIP)
_CONV_DTYPES = {torch.float16: 1, torch.bfloat16: 2}


def _packed_conv_weight(w, dtype, transpose, parent=None):
    """gmz_conv3x3_pack of ``w`` (f32 [128,128,3,3], any memory format) for ``dtype``; cached on the
    parameter per (dtype, transpose) and its version counter, so a weight used by several unroll
    steps is packed once per optimiser step (also inside a captured step: first use packs).  ``parent``: w is
    the view W[:, :128] of that larger parameter (the dynamics stem), cached on it."""
    from . import _lib
    owner = w if parent is None else parent
    key = (dtype, transpose) if parent is None else ("stem", dtype, transpose)
    cache = owner.__dict__.setdefault("_gmz_pack", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == owner._version:
        return hit[1]
    out = hit[1] if hit is not None else torch.empty(147456, dtype=torch.int16, device=w.device)
    s = w.stride()
    _lib.check(_lib.load().gmz_conv3x3_pack(_CONV_DTYPES[dtype], _lib.ptr(w.detach()), s[0], s[1], s[2], s[3],
                                            int(transpose), _lib.ptr(out), _lib.stream_ptr()))
    # (version, packed, source view, transpose, dtype): _repack_stale re-packs the entry in place from the source
    cache[key] = (owner._version, out, w.detach(), int(transpose), dtype)
    return out


_PACK_JOB = np.dtype([("w", "<u8"), ("s", "<i8", 4), ("out", "<u8"), ("transpose", "<i4"), ("pad", "<i4")])


def _repack_stale(owners, tables, prepare=False):
    """BATCH_REPACK: every _packed_conv_weight entry cached on ``owners`` whose parameter changed since it was packed
    (the optimiser step), re-packed into its own buffer by one gmz_conv3x3_pack_many launch per dtype; the entries are
    then current, so the step's forward and backward find them packed.  ``tables``: the device job tables by content
    (a captured step replays the one it was captured with; inside a capture only an existing table is used — an
    unseen set of stale weights is left to the per-use packs; ``prepare``: only build the tables, before a capture)."""
    from . import _lib
    jobs = {}
    for owner in owners:
        cache = owner.__dict__.get("_gmz_pack")
        if not cache:
            continue
        for key, hit in cache.items():
            if len(hit) == 5 and hit[0] != owner._version:
                jobs.setdefault(hit[4], []).append((owner, key, hit))
    if not jobs:
        return 0
    capturing = torch.cuda.is_current_stream_capturing()
    n = 0
    for dtype, js in jobs.items():
        sig = (dtype,) + tuple((h[2].data_ptr(), h[2].stride(), h[1].data_ptr(), h[3]) for _, _, h in js)
        table = tables.get(sig)
        if table is None:
            if capturing:
                continue
            if "job_bytes" not in tables:
                import ctypes
                nb = ctypes.c_size_t()
                _lib.check(_lib.load().gmz_conv3x3_pack_job_bytes(ctypes.byref(nb)))
                if nb.value != _PACK_JOB.itemsize:
                    raise _lib.GmzError("gmz_conv3x3_pack_job_bytes: %d, expected %d" % (nb.value, _PACK_JOB.itemsize))
                tables["job_bytes"] = nb.value
            arr = np.zeros(len(js), dtype=_PACK_JOB)
            for i, (_, _, h) in enumerate(js):
                arr[i] = (h[2].data_ptr(), h[2].stride(), h[1].data_ptr(), h[3], 0)
            table = torch.from_numpy(arr.view(np.uint8)).to(js[0][2][1].device)
            tables[sig] = table
        if prepare:
            continue
        _lib.check(_lib.load().gmz_conv3x3_pack_many(_CONV_DTYPES[dtype], _lib.ptr(table), len(js), _lib.stream_ptr()))
        for owner, key, h in js:
            owner.__dict__["_gmz_pack"][key] = (owner._version,) + tuple(h[1:])
        n += len(js)
    return n


_STATS_SLOTS = {}


def _conv3x3_hip(x, packed, mask=None, stats=None, addend=None, bnb=None, bn_y=None, pend=None):
    """``bnb``: a _BnBwdLink whose BatchNorm output ``bn_y`` fed the forward conv: the output (its dy) also
    gets that BatchNorm's backward dz sums, returned as ``bnb.bwd``.  ``pend``: x is a deferred BatchNorm output
    (_PendingBN), applied and written by this conv's prologue."""
    from . import _lib
    y = torch.empty_like(x, memory_format=torch.channels_last)
    if pend is not None:
        _lib.check(_lib.load().gmz_conv3x3_forward_bnapply(
            _CONV_DTYPES[x.dtype], x.shape[2], _lib.ptr(pend.z), _lib.ptr(pend.res), _lib.ptr(pend.gamma),
            _lib.ptr(pend.beta), _lib.ptr(pend.save), int(pend.relu), _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y),
            x.shape[0], _lib.ptr(mask), _lib.ptr(stats), _stats_slots_of(stats), _lib.stream_ptr()))
        return y
    if bnb is not None:
        if addend is not None:
            addend = addend.to(x.dtype).contiguous(memory_format=torch.channels_last)
        st, ns = _conv_stats_buffer(x.shape[0], x.device)
        _lib.check(_lib.load().gmz_conv3x3_forward_bwdstats(
            _CONV_DTYPES[x.dtype], x.shape[2], _lib.ptr(x), _lib.ptr(packed), _lib.ptr(addend), _lib.ptr(y), x.shape[0],
            _lib.ptr(bnb.mask), _lib.ptr(bnb.x), _lib.ptr(bn_y), _lib.ptr(bnb.save), int(bnb.relu), _lib.ptr(st),
            _stats_slots_of(st), _lib.stream_ptr()))
        bnb.bwd = (st, ns, y)
        return y
    if addend is not None:  # y = round(conv + addend) (the residual gradient folded into the input gradient)
        addend = addend.to(x.dtype).contiguous(memory_format=torch.channels_last)
        _lib.check(_lib.load().gmz_conv3x3_forward_add(_CONV_DTYPES[x.dtype], x.shape[2], _lib.ptr(x), _lib.ptr(packed),
                                                       _lib.ptr(addend), _lib.ptr(y), x.shape[0], _lib.stream_ptr()))
        return y
    _lib.check(_lib.load().gmz_conv3x3_forward_stats(_CONV_DTYPES[x.dtype], x.shape[2], _lib.ptr(x), _lib.ptr(packed),
                                                     _lib.ptr(y), x.shape[0], _lib.ptr(mask), _lib.ptr(stats),
                                                     _stats_slots_of(stats), _lib.stream_ptr()))
    return y


def _stats_slots_of(stats):
    """The slot capacity of an f64 [128][slots][3] statistics-partials buffer (0 for None): the library checks it
    against the slot count of the launch before writing (ABI 10)."""
    return 0 if stats is None else stats.numel() // (128 * 3)


# the residual blocks' identity-path gradient folded into conv1's input-gradient epilogue (_ResLink):
# one gradient for the block input instead of two plus an autograd accumulation pass per block
FUSED_RES_GRAD = True


class _ResLink:
    """Hand-off between one residual block's bn2 (which produces the identity path's gradient) and its
    conv1 (whose input-gradient kernel adds it): xin = the tensor conv1 consumed (the block input),
    dres = the gradient bn2's backward left for conv1's backward (always the later of the two)."""
    __slots__ = ("xin", "dres")

    def __init__(self):
        self.xin = None
        self.dres = None


# the 128->128 convs' weight gradient on gmz_conv3x3_wgrad instead of MIOpen: exact (f32 accumulation,
# tested), 47 + 9 us vs MIOpen's 55 us + the add into the f32 .grad per 360-board layer; the whole step
# 26.4-26.5 -> 26.8-27.0 steps/s (same-box A/B, tools/bench_trainer.py --hip-wgrad).  The kernel's
# per-board LDS DMA is not yet overlapped with its k-loop (~40 % MFMA busy)
HIP_WGRAD = True
# set by Trainer only while its own backward runs (its .grad tensors are views of the flat bucket that
# nothing else reads): the HIP weight gradients then add straight into .grad and return None to
# autograd.  Every other caller (torch.autograd.grad, hooks, other reducers) gets them through autograd.
_DIRECT_GRAD = [False]
_WGRAD_WS = {}


# the 3x3 weight gradients of Trainer's backward deferred to its end: one multi-segment launch per weight
# over every use of it (the dynamics trunk's convs run in all unroll steps: 5 launches and 5 partial-sum
# reductions -> 1), gmz_conv3x3_wgrad_segments
DEFER_WGRAD = True
_PENDING_WGRAD = {}


def flush_wgrads():
    """Run the deferred weight gradients (DEFER_WGRAD) into their parameters' f32 .grad."""
    import ctypes
    from . import _lib
    L = _lib.load()
    for w, uses in _PENDING_WGRAD.items():
        groups = {}
        for x, gy in uses:
            groups.setdefault((x.shape[0], x.dtype, x.shape[2]), []).append((x, gy))
        for (N, dt, H), lst in groups.items():
            for i in range(0, len(lst), 8):
                seg = lst[i:i + 8]
                n = len(seg) * N
                if n not in _WGRAD_WS:
                    nb = ctypes.c_size_t()
                    _lib.check(L.gmz_conv3x3_wgrad_workspace_bytes(n, ctypes.byref(nb)))
                    _WGRAD_WS[n] = nb.value
                ws = torch.empty(_WGRAD_WS[n] // 4, dtype=torch.float32, device=w.device)
                xs = (ctypes.c_void_p * len(seg))(*[x.data_ptr() for x, _ in seg])
                gs = (ctypes.c_void_p * len(seg))(*[g.data_ptr() for _, g in seg])
                st = w.grad.stride()
                _lib.check(L.gmz_conv3x3_wgrad_segments(_CONV_DTYPES[dt], H, ctypes.cast(xs, ctypes.c_void_p),
                                                        ctypes.cast(gs, ctypes.c_void_p), len(seg), N,
                                                        _lib.ptr(w.grad), st[0], st[1], st[2], st[3], 1, _lib.ptr(ws),
                                                        _lib.nbytes(ws), _lib.stream_ptr()))
    _PENDING_WGRAD.clear()


def _conv3x3_wgrad_hip(x, gy, grad):
    """grad (f32, any strides) += weight gradient of the 128->128 conv from channels-last x, gy."""
    import ctypes
    from . import _lib
    L = _lib.load()
    N = x.shape[0]
    if N not in _WGRAD_WS:
        n = ctypes.c_size_t()
        _lib.check(L.gmz_conv3x3_wgrad_workspace_bytes(N, ctypes.byref(n)))
        _WGRAD_WS[N] = n.value
    ws = torch.empty(_WGRAD_WS[N] // 4, dtype=torch.float32, device=x.device)
    s = grad.stride()
    _lib.check(L.gmz_conv3x3_wgrad(_CONV_DTYPES[x.dtype], x.shape[2], _lib.ptr(x), _lib.ptr(gy), N, _lib.ptr(grad),
                                   s[0], s[1], s[2], s[3], 1, _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr()))


def _conv_stats_buffer(N, device):
    """f64 [128][slots][3] partials (channel-major) for gmz_conv3x3_forward_stats -> (tensor, slots)."""
    import ctypes
    from . import _lib
    if N not in _STATS_SLOTS:
        n = ctypes.c_int()
        _lib.check(_lib.load().gmz_conv3x3_stats_slots(N, ctypes.byref(n)))
        _STATS_SLOTS[N] = n.value
    ns = _STATS_SLOTS[N]
    return torch.empty(ns * 128 * 3, dtype=torch.float64, device=device), ns


class _Conv3x3NHWC(torch.autograd.Function):
    """128 -> 128 3x3 convolution (padding 1, no bias) of channels-last f16/bf16 activations:
    forward and input gradient on the HIP implicit-GEMM kernel (csrc/gmz_conv.hip; the input
    gradient is the same kernel on the transposed, flipped weight), weight gradient by MIOpen
    (aten.convolution_backward, weight only).  The weight stays the f32 parameter: the pack kernel
    converts it (what autocast's cast would do)."""

    @staticmethod
    def forward(ctx, x, w, mask=None, stats=None, link=None, bnsrc=None, pend=None):
        ctx.save_for_backward(x, w)
        ctx.link = link
        ctx.bnsrc = bnsrc  # the _BnBwdLink of the BatchNorm whose output x is (FUSED_BN_BWD_STATS)
        return _conv3x3_hip(x, _packed_conv_weight(w, x.dtype, 0), mask, stats, pend=pend)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        add = None
        if ctx.link is not None:
            add, ctx.link.dres = ctx.link.dres, None
        gx = None
        if ctx.needs_input_grad[0]:
            bnb = ctx.bnsrc if (FUSED_BN_BWD_STATS and ctx.bnsrc is not None and ctx.bnsrc.x.dtype == x.dtype) else None
            gx = _conv3x3_hip(gy, _packed_conv_weight(w, x.dtype, 1), addend=add, bnb=bnb, bn_y=x)
        gw = None
        if ctx.needs_input_grad[1]:
            if HIP_WGRAD:
                if _DIRECT_GRAD[0] and w.grad is not None and w.grad.dtype == torch.float32:
                    # inside Trainer's backward: accumulated straight into the f32 .grad (the flat-bucket
                    # view): no f16 gradient tensor, no cast, no AccumulateGrad add.  DEFER_WGRAD: after the
                    # backward, one launch per weight over all its uses (flush_wgrads)
                    if DEFER_WGRAD:
                        _PENDING_WGRAD.setdefault(w, []).append((x, gy))
                    else:
                        _conv3x3_wgrad_hip(x, gy, w.grad)
                else:  # any other caller: the gradient goes back through autograd
                    gw = torch.zeros_like(w, dtype=torch.float32)
                    _conv3x3_wgrad_hip(x, gy, gw)
                    gw = gw.to(w.dtype)
            else:
                wd = torch.empty(w.shape, dtype=x.dtype, device=w.device, memory_format=torch.channels_last)  # shape only
                gw = torch.ops.aten.convolution_backward(gy, x, wd, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                         [False, True, False])[1]
                if _DIRECT_GRAD[0] and w.grad is not None and w.grad.dtype == torch.float32:
                    w.grad.add_(gw)  # one mixed-dtype add into the f32 .grad instead of a cast + AccumulateGrad
                    gw = None
                else:
                    gw = gw.to(w.dtype)
        return gx, gw, None, None, None, None, None


# the stamp table's dtype code for gmz_conv3x3_forward_stamp: the library takes f32 only and rejects anything else
# (or a table of the wrong size) before the launch (ABI 10); -1 = a dtype with no code
_TABLE_DTYPES = collections.defaultdict(lambda: -1, {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2})

# the dynamics trunk's first conv (144 -> 128) on the HIP conv: its 128 hidden planes as a 128 -> 128 conv, its 16
# action-embedding planes (one one-hot cell per board) as a 3x3 stamp added in the conv's epilogue
# (gmz_conv3x3_forward_stamp), instead of MIOpen's three 144-channel kernels and the concatenation (A/B switch;
# off until its GPU equivalence test is green)
DYN_STEM_HIP = False


class _StemGrad:
    """flush_wgrads' handle on the stem weight's hidden-plane gradient W.grad[:, :128] (the deferred HIP weight
    gradient of the 128 -> 128 part; one handle per parameter, so the unroll steps' uses merge into one launch)."""
    __slots__ = ("grad", "device")

    def __init__(self, device):
        self.grad, self.device = None, device


class _DynStemHIP(torch.autograd.Function):
    """y = conv3x3(cat(h, embed(a)), W) for channels-last f16/bf16 h [n, 128, H, H], W f32 [128, 144, 3, 3],
    embed = action_embed_conv (1 -> 16, no bias) of the one-hot plane of a (network.py:79-96, under autocast):
    the hidden part on gmz_conv3x3 (forward, input and weight gradients), the embedding part as the stamp table
    T[tap][o] = sum_c W16[o][128 + c][tap] * e16[c] (the 16-bit operands the 144-channel conv multiplies, f32 sums)
    added before the output's one rounding; its gradients from the 9 output cells around each board's action."""

    @staticmethod
    def forward(ctx, h, W, w_emb, a, mask, stats):
        from . import _lib
        dt = h.dtype
        n, _, H, _ = h.shape
        # the table in float32 whatever the caller's autocast state (under autocast einsum would run in f16 and
        # hand the kernel a half-size f16 buffer it reads as f32: the round-5 GPU fault)
        with torch.autocast("cuda", enabled=False):
            w2 = W.detach()[:, 128:].to(dt).float().reshape(128, 16, 9)
            e = w_emb.detach().reshape(16).to(dt).float()
            table = torch.einsum("oct,c->to", w2, e).contiguous()
        a32 = a.to(torch.int32).contiguous()
        if a32.numel() != h.shape[0]:
            raise RuntimeError("_DynStemHIP: one action per board")
        y = torch.empty_like(h, memory_format=torch.channels_last)
        _lib.check(_lib.load().gmz_conv3x3_forward_stamp(
            _CONV_DTYPES[dt], H, _lib.ptr(h), _lib.ptr(_packed_conv_weight(W[:, :128], dt, 0, parent=W)), _lib.ptr(y), n,
            _lib.ptr(mask), _lib.ptr(stats), _stats_slots_of(stats), _lib.ptr(a32), _lib.ptr(table),
            _TABLE_DTYPES[table.dtype], _lib.nbytes(table), _lib.stream_ptr()))
        ctx.save_for_backward(h, W, w_emb, a32)
        return y

    @staticmethod
    def backward(ctx, gy):
        h, W, w_emb, a32 = ctx.saved_tensors
        dt = h.dtype
        n, _, H, _ = h.shape
        A = H * H
        gy = gy.to(dt).contiguous(memory_format=torch.channels_last)
        gh = None
        if ctx.needs_input_grad[0]:
            gh = _conv3x3_hip(gy, _packed_conv_weight(W[:, :128], dt, 1, parent=W))
        gW = gemb = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # the stamp's gradient: dT[tap][o] = sum over boards of gy at the cell q = a - (tap - (1, 1))
            a = a32.long()
            ay, ax = a // H, a % H
            k = torch.arange(9, device=a.device)
            qy, qx = ay[:, None] - (k // 3 - 1), ax[:, None] - (k % 3 - 1)
            ok = ((qy >= 0) & (qy < H) & (qx >= 0) & (qx < H)).to(torch.float32)
            idx = (qy.clamp(0, H - 1) * H + qx.clamp(0, H - 1))
            g = gy.permute(0, 2, 3, 1).reshape(n, A, 128).gather(1, idx[..., None].expand(n, 9, 128)).float()
            with torch.autocast("cuda", enabled=False):
                dT = (g * ok[..., None]).sum(0)  # [9, 128]
                w2 = W.detach()[:, 128:].to(dt).float().reshape(128, 16, 9)
                e = w_emb.detach().reshape(16).to(dt).float()
                dW2 = torch.einsum("to,c->oct", dT, e).reshape(128, 16, 3, 3)
                gemb = torch.einsum("to,oct->c", dT, w2).reshape(w_emb.shape)
            if _DIRECT_GRAD[0] and W.grad is not None and W.grad.dtype == torch.float32:
                W.grad[:, 128:].add_(dW2)
                hold = W.__dict__.get("_gmz_stem_grad")
                if hold is None:
                    hold = W.__dict__.setdefault("_gmz_stem_grad", _StemGrad(W.device))
                hold.grad = W.grad[:, :128]
                if DEFER_WGRAD:
                    _PENDING_WGRAD.setdefault(hold, []).append((h, gy))
                else:
                    _conv3x3_wgrad_hip(h, gy, hold.grad)
            else:
                gW = torch.zeros(W.shape, dtype=torch.float32, device=W.device)
                _conv3x3_wgrad_hip(h, gy, gW[:, :128])
                gW[:, 128:] = dW2
                gW = gW.to(W.dtype)
            gemb = gemb.to(w_emb.dtype)
        return gh, gW, gemb, None, None, None


def _dyn_stem_hip_ok(dyn, h):
    if not (DYN_STEM_HIP and FUSED_CONV and h.is_cuda and h.dim() == 4 and h.shape[1] == 128
            and h.shape[2] == h.shape[3] and h.shape[2] in (9, 15)):
        return False
    if dyn.conv.weight.shape != (128, 128 + dyn.EMB, 3, 3) or dyn.conv.bias is not None:
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else h.dtype
    return dt in _CONV_DTYPES and h.is_contiguous(memory_format=torch.channels_last)


def _conv3(cin, cout):
    return nn.Conv2d(cin, cout, 3, padding=1, bias=False)


def _conv3_apply(conv, x, bn=None, mask=None, link=None, segments=1):
    """conv(x), on the HIP kernels when they cover the case (see ``_Conv3x3NHWC``).  ``bn``: the
    training-mode BatchNorm that consumes the output — the kernel's epilogue then also reduces its
    (row-masked) statistics, attached to the output for ``_bn_act`` (no separate reduction pass).
    ``segments`` > 1 (no_grad only): the statistics partials per board, for the segmented BatchNorm."""
    if (FUSED_CONV and x.is_cuda and x.dim() == 4 and x.shape[1] == 128 and x.shape[2] == x.shape[3]
            and x.shape[2] in (9, 15) and conv.weight.shape == (128, 128, 3, 3) and conv.bias is None):
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        if (segments > 1 and dt in _CONV_DTYPES and x.is_contiguous(memory_format=torch.channels_last)
                and not torch.is_grad_enabled()):
            from . import _lib
            xin = x.to(dt)
            N = xin.shape[0]
            y = torch.empty_like(xin, memory_format=torch.channels_last)
            packed = _packed_conv_weight(conv.weight, dt, 0)
            if bn is not None and bn.training and FUSED_BN:
                st = torch.empty(128 * N * 3, dtype=torch.float64, device=x.device)
                m = None if mask is None else mask.contiguous().view(torch.uint8)
                _lib.check(_lib.load().gmz_conv3x3_forward_board_stats(_CONV_DTYPES[dt], xin.shape[2], _lib.ptr(xin),
                                                                       _lib.ptr(packed), _lib.ptr(y), N, _lib.ptr(m),
                                                                       _lib.ptr(st), N, _lib.stream_ptr()))
                y._gmz_bnstats = (st, "board")
            else:
                _lib.check(_lib.load().gmz_conv3x3_forward(_CONV_DTYPES[dt], xin.shape[2], _lib.ptr(xin), _lib.ptr(packed),
                                                           _lib.ptr(y), N, _lib.stream_ptr()))
            return y
        if dt in _CONV_DTYPES and x.is_contiguous(memory_format=torch.channels_last):
            st = None
            if bn is not None and bn.training and FUSED_BN:
                st = _conv_stats_buffer(x.shape[0], x.device)
            m = None if mask is None else mask.contiguous().view(torch.uint8)
            xin = x.to(dt)
            bnsrc = getattr(xin, "_gmz_bnsrc", None) if xin is x else None  # x = a BatchNorm's output, as is
            pend = getattr(x, "_gmz_pending", None)
            if pend is not None:  # x is written by this conv's prologue (once: later readers see it written)
                if xin is not x:
                    raise RuntimeError("_conv3_apply: a deferred BatchNorm output needs a conv of its own dtype")
                x._gmz_pending = None
            y = _Conv3x3NHWC.apply(xin, conv.weight, m, None if st is None else st[0], link, bnsrc, pend)
            if link is not None:
                link.xin = xin
            if st is not None:
                y._gmz_bnstats = st
            return y
    if getattr(x, "_gmz_pending", None) is not None:
        raise RuntimeError("_conv3_apply: a deferred BatchNorm output reached a conv that cannot apply it")
    return conv(x)


class _Block(nn.Module):
    """Residual block (conv-BN-ReLU-conv-BN + identity, ReLU), parameter names of network.py:30-48."""

    def __init__(self, c):
        super().__init__()
        self.conv1, self.bn1 = _conv3(c, c), nn.BatchNorm2d(c, eps=1e-4)
        self.conv2, self.bn2 = _conv3(c, c), nn.BatchNorm2d(c, eps=1e-4)

    def forward(self, x, mask=None, segments=1, consumer=None):
        """``consumer``: the 3x3 conv that consumes the block's output next (the next block's conv1), which may
        then apply bn2 in its prologue (DEFER_BN_APPLY); bn1's output always goes to conv2."""
        if segments > 1:  # the batched consistency representations (no_grad): per-segment statistics
            y = _bn_act(self.bn1, _conv3_apply(self.conv1, x, self.bn1, mask, segments=segments), mask,
                        segments=segments)
            return _bn_act(self.bn2, _conv3_apply(self.conv2, y, self.bn2, mask, segments=segments), mask, res=x,
                           segments=segments)
        link = _ResLink() if (FUSED_RES_GRAD and torch.is_grad_enabled() and x.requires_grad) else None
        y = _bn_act(self.bn1, _conv3_apply(self.conv1, x, self.bn1, mask, link=link), mask, consumer=self.conv2)
        return _bn_act(self.bn2, _conv3_apply(self.conv2, y, self.bn2, mask), mask, res=x, link=link,
                       consumer=consumer)


class _Trunk(nn.Module):
    """conv3x3 + BN + ReLU followed by residual blocks (representation and dynamics trunks)."""

    def __init__(self, cin, c, blocks):
        super().__init__()
        self._build(cin, c, blocks)

    def _build(self, cin, c, blocks):
        self.conv, self.bn = _conv3(cin, c), nn.BatchNorm2d(c, eps=1e-4)
        self.resblocks = nn.Sequential(*[_Block(c) for _ in range(blocks)])

    def forward(self, x, mask=None, segments=1):
        if segments > 1:
            h = _bn_act(self.bn, self.conv(x), mask, segments=segments)
            for blk in self.resblocks:
                h = blk(h, mask, segments)
            return h
        return self._blocks(self.conv(x), mask)

    def _blocks(self, z, mask):
        """The stem's BatchNorm + ReLU of z, then the residual blocks; every BatchNorm output that a next block's
        conv1 consumes is deferred to that conv's prologue (DEFER_BN_APPLY); the trunk's output is written."""
        blocks = list(self.resblocks)
        h = _bn_act(self.bn, z, mask, consumer=blocks[0].conv1 if blocks else None)
        for i, blk in enumerate(blocks):
            h = blk(h, mask, consumer=blocks[i + 1].conv1 if i + 1 < len(blocks) else None)
        return h


# the prediction heads' two 1x1 convs (policy 128 -> 2, value 128 -> 1, same input) as one HIP pass forward and one
# backward (gmz_head_conv1x1_*: dx of both heads in one rounding, dW / db reduced in a fixed order) instead of two
# GEMMs + bias adds forward and two GEMMs + batched GEMMs + reductions + a dx add backward (False: PyTorch, A/B)
FUSED_HEADS = True


def _headconv_forward(x, w0, b0, w1, b1):
    """gmz_head_conv1x1_forward of the channels-last x: (y0, y1) channels-last [n, O, H, W] and what the backward
    needs"""
    from . import _lib
    L = _lib.load()
    n, C, H, W = x.shape
    O0, O1 = w0.shape[0], w1.shape[0]
    P = n * H * W
    wm = [_head_param(t, (O0, C)) for t in (w0, b0, w1, b1)]  # [O][C] rows / [O]: f32, contiguous views
    y0 = torch.empty((n, H, W, O0), dtype=x.dtype, device=x.device)
    y1 = torch.empty((n, H, W, O1), dtype=x.dtype, device=x.device)
    _lib.check(L.gmz_head_conv1x1_forward(_BN_DTYPES[x.dtype], _lib.ptr(x), P, C, _lib.ptr(wm[0]), _lib.ptr(wm[1]),
                                          O0, _lib.ptr(wm[2]), _lib.ptr(wm[3]), O1, _lib.ptr(y0), _lib.ptr(y1),
                                          _lib.stream_ptr()))
    return y0.permute(0, 3, 1, 2), y1.permute(0, 3, 1, 2), (wm[0], wm[2], (O0, O1))


def _headconv_backward(x, saved, params, g0, g1):
    """gmz_head_conv1x1_backward: (dx channels-last like x, the four parameter gradients — None when they went
    straight into the trainer's f32 .grad, _DIRECT_GRAD)"""
    import ctypes
    from . import _lib
    L = _lib.load()
    w0m, w1m, (O0, O1) = saved
    n, C, H, W = x.shape
    P = n * H * W
    g0 = (g0 if g0 is not None else torch.zeros((n, O0, H, W), dtype=x.dtype, device=x.device))
    g1 = (g1 if g1 is not None else torch.zeros((n, O1, H, W), dtype=x.dtype, device=x.device))
    g0 = g0.to(x.dtype).permute(0, 2, 3, 1).contiguous()  # [n, H, W, O]: positions x outputs
    g1 = g1.to(x.dtype).permute(0, 2, 3, 1).contiguous()
    dx = torch.empty_like(x)  # channels-last like x
    nb = ctypes.c_size_t()
    _lib.check(L.gmz_head_conv1x1_workspace_bytes(P, O0 + O1, ctypes.byref(nb)))
    ws = torch.empty(nb.value // 4, dtype=torch.float32, device=x.device)
    # the trainer's own backward (_DIRECT_GRAD): add into the f32 .grad views of its flat bucket
    direct = _DIRECT_GRAD[0] and all(p.grad is not None and p.grad.dtype == torch.float32
                                     and p.grad.is_contiguous() for p in params)
    outs = [p.grad if direct else torch.empty(p.shape, dtype=torch.float32, device=x.device) for p in params]
    _lib.check(L.gmz_head_conv1x1_backward(_BN_DTYPES[x.dtype], _lib.ptr(x), P, C, _lib.ptr(w0m), O0, _lib.ptr(w1m), O1,
                                           _lib.ptr(g0), _lib.ptr(g1), _lib.ptr(dx), *[_lib.ptr(t) for t in outs],
                                           int(direct), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr()))
    if direct:
        return dx, [None] * 4
    return dx, [t.to(p.dtype) for t, p in zip(outs, params)]


class _HeadConv1x1(torch.autograd.Function):
    """(policy_conv(x), value_conv(x)) for a channels-last f16/bf16 hidden state x [n, 128, H, W] under autocast:
    y0 [n, O0, H, W] and y1 [n, O1, H, W] channels-last (gmz_head_conv1x1_forward / _backward)."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1):
        y0, y1, saved = _headconv_forward(x, w0, b0, w1, b1)
        ctx.save_for_backward(x, saved[0], saved[1], w0, b0, w1, b1)
        ctx.O = saved[2]
        return y0, y1

    @staticmethod
    def backward(ctx, g0, g1):
        x, w0m, w1m, w0, b0, w1, b1 = ctx.saved_tensors
        dx, gp = _headconv_backward(x, (w0m, w1m, ctx.O), (w0, b0, w1, b1), g0, g1)
        return (dx, *gp)


def _head_param(t, shape):
    """a head conv's f32 weight [O, C, 1, 1] as its [O][C] rows (bias: as is), without a copy when it already is"""
    t = t.detach()
    t = t.reshape(t.shape[0], -1) if t.dim() > 1 else t
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    return t


def _head_convs_hip_ok(pred, h):
    if not (FUSED_HEADS and h.is_cuda and torch.is_autocast_enabled("cuda") and h.dim() == 4 and h.shape[1] == 128):
        return False
    dt = torch.get_autocast_dtype("cuda")
    return (dt in _CONV_DTYPES and h.dtype == dt and h.is_contiguous(memory_format=torch.channels_last)
            and h.data_ptr() % 16 == 0 and pred.policy_conv.bias is not None and pred.value_conv.bias is not None)


class _Prediction(nn.Module):
    def __init__(self, c, H, hd, vbins):
        super().__init__()
        A = H * H
        self.policy_conv, self.policy_bn = nn.Conv2d(c, 2, 1), nn.BatchNorm2d(2, eps=1e-4)
        self.policy_fc = nn.Linear(2 * A, A)
        self.value_conv, self.value_bn = nn.Conv2d(c, 1, 1), nn.BatchNorm2d(1, eps=1e-4)
        self.value_fc1, self.value_fc2 = nn.Linear(A, hd), nn.Linear(hd, vbins)

    def forward(self, h, mask=None):
        n = h.shape[0]
        if _head_convs_hip_ok(self, h):
            yp, yv = _HeadConv1x1.apply(h, self.policy_conv.weight, self.policy_conv.bias, self.value_conv.weight,
                                        self.value_conv.bias)
        else:
            yp, yv = _conv1x1(self.policy_conv, h), _conv1x1(self.value_conv, h)
        pol = self.policy_fc(_bn_act(self.policy_bn, yp, mask).reshape(n, -1))
        v = F.relu(self.value_fc1(_bn_act(self.value_bn, yv, mask).reshape(n, -1)))
        return pol, self.value_fc2(v)


class _Dynamics(_Trunk):
    EMB = 16  # network.py:81 action embedding planes

    def __init__(self, c, H, blocks, hd, rbins):
        nn.Module.__init__(self)
        # registration order of network.py:79-87 (action_embed_conv, conv, bn, resblocks, reward_fc):
        # parameters() order is the index order of a reference optimiser checkpoint
        self.action_embed_conv = nn.Conv2d(1, self.EMB, 1, bias=False)
        self._build(c + self.EMB, c, blocks)
        self.reward_fc = nn.Sequential(nn.Linear(c * H * H, hd), nn.ReLU(), nn.Linear(hd, rbins))

    def embed(self, a, like):
        """the action planes' embedding (network.py:88-90: one-hot plane -> 1x1 conv to 16 planes) for actions a
        [n], in like's dtype and memory format"""
        n, (H, W) = a.shape[0], like.shape[2:]
        plane = F.one_hot(a, H * W).to(like.dtype).reshape(n, 1, H, W)
        emb = _conv1x1(self.action_embed_conv, plane).to(like.dtype)
        if like.is_contiguous(memory_format=torch.channels_last) and not like.is_contiguous():
            emb = emb.contiguous(memory_format=torch.channels_last)   # cat keeps channels-last
        return emb

    def forward(self, h, a, mask=None, reward=True, emb=None):
        """(next hidden state, reward logits); ``reward`` False: the trunk only (BATCHED_HEADS takes the reward head
        of every unroll step after the unroll, in one pass).  ``emb``: this step's action embedding, already computed
        (BATCHED_HEADS embeds every step's action in one pass before the unroll)."""
        n, _, H, W = h.shape
        if _dyn_stem_hip_ok(self, h):  # DYN_STEM_HIP: the 144-channel conv as hidden-plane conv + action stamp
            dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else h.dtype
            st = _conv_stats_buffer(n, h.device) if (self.bn.training and FUSED_BN) else None
            m = None if mask is None else mask.contiguous().view(torch.uint8)
            y = _DynStemHIP.apply(h.to(dt), self.conv.weight, self.action_embed_conv.weight, a, m,
                                  None if st is None else st[0])
            if st is not None:
                y._gmz_bnstats = st
            x = self._blocks(y, mask)
            if not reward:
                return x, None
            fc0, act, fc2 = self.reward_fc
            return x, fc2(act(_linear_flat(fc0, x)))
        if emb is None:
            emb = self.embed(a, h)
        nxt = super().forward(torch.cat((h, emb.to(h.dtype)), dim=1), mask)
        if not reward:
            return nxt, None
        fc0, act, fc2 = self.reward_fc
        return nxt, fc2(act(_linear_flat(fc0, nxt)))


FLAT_NHWC = True  # channels-last flatten for the K = 28,800 Linears (False: NCHW copy per use; A/B)


def _bigk_weight(w, dt, perm):
    """w (f32 [O, K]) in the autocast dtype, cached per optimiser step (version counter, as
    _packed_conv_weight; inside a captured step the first use converts).  perm = (C, HW): the columns
    reordered from the reference's NCHW flatten (k = c*HW + p) to the channels-last one (k = p*C + c),
    so a channels-last hidden state flattens as a view instead of a transposing copy per use."""
    key = ("bigk", dt, perm)
    cache = w.__dict__.setdefault("_gmz_pack", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == w._version:
        return hit[1]
    if perm is None:
        out = w.detach().to(dt)
    else:
        C, HW = perm
        out = torch.empty(w.shape, dtype=dt, device=w.device)
        out.view(w.shape[0], HW, C).copy_(w.detach().view(w.shape[0], C, HW).transpose(1, 2))
    cache[key] = (w._version, out)
    return out


class _BigKLinear(torch.autograd.Function):
    """y = x W^T + b for the trainer's K = C*H*W = 28,800 Linears (projection fc1, reward_fc.0) under
    fp16/bf16 autocast.  hipBLASLt runs x @ W^T at B = 360 on 24 workgroups (83 us for 28800->512);
    here K is split in 16 chunks, one batched GEMM with float32 outputs summed in float32 (33 us),
    rounded once to the autocast dtype like the single GEMM's output.  Backward: dx = dy W, and
    dW = (x^T dy)^T (26 us vs 39 us for dy^T x at K = B = 360).
    perm = (C, HW): x is a channels-last hidden state flattened as (p, c) and W's columns are used in
    that order (_bigk_weight); dW goes back to the parameter's (c, p) order in the one strided pass
    that adds it into the f32 .grad."""
    SPLIT = 16

    @staticmethod
    def forward(ctx, x, w, b, dt, perm=None):
        xs, ws = x.to(dt), _bigk_weight(w, dt, perm)
        n, K = xs.shape
        S = _BigKLinear.SPLIT
        y = torch.bmm(xs.view(n, S, K // S).transpose(0, 1), ws.view(-1, S, K // S).permute(1, 2, 0),
                      out_dtype=torch.float32).sum(0)
        ctx.save_for_backward(xs, ws, w)
        ctx.perm = perm
        return (y + b).to(dt) if b is not None else y.to(dt)

    @staticmethod
    def backward(ctx, gy):
        xs, ws, w = ctx.saved_tensors
        gy = gy.to(xs.dtype)
        gx = gy @ ws if ctx.needs_input_grad[0] else None
        gw = None
        if ctx.needs_input_grad[1]:
            gwt = xs.t() @ gy  # [K, O] in x's column order
            O = w.shape[0]
            acc = (_DIRECT_GRAD[0] and w.grad is not None and w.grad.dtype == torch.float32
                   and w.grad.is_contiguous())
            if ctx.perm is None:
                gw = gwt.t().to(w.dtype)
            else:
                # W's (c, p) column order, added straight into the f32 .grad by an LDS-tiled transpose
                # (gmz_grad_add_t: 109 -> ~45 us per call vs a strided PyTorch add at 512 x 28,800)
                from . import _lib
                C, HW = ctx.perm
                dst = w.grad if acc else torch.zeros(w.shape, dtype=torch.float32, device=w.device)
                _lib.check(_lib.load().gmz_grad_add_t(_BN_DTYPES[gwt.dtype], _lib.ptr(gwt), HW, C, O, _lib.ptr(dst),
                                                     _lib.stream_ptr()))
                if not acc:
                    gw = dst
        gb = gy.sum(0, dtype=torch.float32) if ctx.needs_input_grad[2] else None
        return gx, gw, gb, None, None


def _bigk_weight_cat(w1, w2, dt, perm):
    """[w1; w2] in the autocast dtype and channels-last column order (_bigk_weight of each), cached on w1 per
    optimiser step of both (version counters; inside a captured step the first use converts)."""
    key = ("bigkcat", dt, perm, id(w2))
    cache = w1.__dict__.setdefault("_gmz_pack", {})
    hit = cache.get(key)
    if hit is not None and hit[0] == (w1._version, w2._version):
        return hit[1]
    out = torch.cat((_bigk_weight(w1, dt, perm), _bigk_weight(w2, dt, perm)))
    cache[key] = ((w1._version, w2._version), out)
    return out


def _bigk2_forward(x, w1, b1, w2, b2, dt, perm):
    """(x W1^T + b1, x W2^T + b2) as one split-K GEMM against [W1; W2] (x [n, K] in the flatten order of perm)."""
    xs, ws = x.to(dt), _bigk_weight_cat(w1, w2, dt, perm)
    n, K = xs.shape
    S = _BigKLinear.SPLIT if n <= 1024 else 4
    y = torch.bmm(xs.view(n, S, K // S).transpose(0, 1), ws.view(-1, S, K // S).permute(1, 2, 0),
                  out_dtype=torch.float32).sum(0)
    y = (y + torch.cat((b1, b2)).float()).to(dt)
    O1 = w1.shape[0]
    return y[:, :O1].contiguous(), y[:, O1:].contiguous(), xs, ws


def _bigk2_backward(xs, ws, w1, w2, perm, g1, g2, needs, gx_acc=None):
    """The backward of _bigk2_forward: gx = [g1 g2] [W1; W2] — returned, or added in place into gx_acc (a [n, K]
    view of a gradient that another consumer of x already wrote: one GEMM with beta = 1 instead of a GEMM and an
    add) — and the four parameter gradients (needs: which of w1, b1, w2, b2; the weights' go straight into their
    f32 .grad under _DIRECT_GRAD, as None)."""
    n, O1 = xs.shape[0], w1.shape[0]
    O2 = ws.shape[0] - O1
    g1 = torch.zeros((n, O1), dtype=xs.dtype, device=xs.device) if g1 is None else g1.to(xs.dtype)
    g2 = torch.zeros((n, O2), dtype=xs.dtype, device=xs.device) if g2 is None else g2.to(xs.dtype)
    gy = torch.cat((g1, g2), 1)
    gx = None
    if gx_acc is not None:
        gx_acc.addmm_(gy, ws)
    elif needs[0]:
        gx = gy @ ws
    outs = [None, None, None, None]
    if needs[1] or needs[3]:
        gwt = xs.t() @ gy  # [K, O1 + O2] in x's column order
        for i, (w, c0, O) in enumerate(((w1, 0, O1), (w2, O1, O2))):
            if not needs[1 + 2 * i]:
                continue
            acc = (_DIRECT_GRAD[0] and w.grad is not None and w.grad.dtype == torch.float32
                   and w.grad.is_contiguous())
            if perm is None:
                outs[2 * i] = gwt[:, c0:c0 + O].t().to(w.dtype)
                continue
            from . import _lib
            C, HW = perm
            dst = w.grad if acc else torch.zeros(w.shape, dtype=torch.float32, device=w.device)
            _lib.check(_lib.load().gmz_grad_add_t_cols(_BN_DTYPES[gwt.dtype], _lib.ptr(gwt), HW, C, O, O1 + O2, c0,
                                                      _lib.ptr(dst), _lib.stream_ptr()))
            if not acc:
                outs[2 * i] = dst
    if needs[2] or needs[4]:
        gb = gy.sum(0, dtype=torch.float32)
        outs[1], outs[3] = gb[:O1], gb[O1:]
    return gx, outs


class _BigKLinear2(torch.autograd.Function):
    """(x W1^T + b1, x W2^T + b2) for two K = 28,800 Linears that read the same flattened hidden state — the
    projection's fc1 (network.py:95) and the reward head's first Linear (network.py:105) of every unroll step — as
    ONE split-K GEMM against [W1; W2] (_BigKLinear's arithmetic: f32 partial sums, one rounding).  Backward: one
    dx GEMM against [W1; W2] (no add of two input gradients), one x^T dy GEMM whose two column ranges go into the
    two weights' f32 .grad (gmz_grad_add_t_cols)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dt, perm=None):
        y1, y2, xs, ws = _bigk2_forward(x, w1, b1, w2, b2, dt, perm)
        ctx.save_for_backward(xs, ws, w1, w2)
        ctx.perm = perm
        return y1, y2

    @staticmethod
    def backward(ctx, g1, g2):
        xs, ws, w1, w2 = ctx.saved_tensors
        gx, outs = _bigk2_backward(xs, ws, w1, w2, ctx.perm, g1, g2, ctx.needs_input_grad[:5])
        return (gx, *outs, None, None)


class _HeadsInput(torch.autograd.Function):
    """The first layer of every head that reads the stacked hidden states hp [(U+1)*B, 128, H, W] (BATCHED_HEADS):
    the prediction's two 1x1 convs over all U+1 steps (gmz_head_conv1x1) and the projection fc1 + reward fc0 GEMM
    over the U dynamics steps hp[B:] (_bigk2_forward) — in ONE autograd node, so hp's gradient is the convs' dx with
    the GEMM's dx added in place into its last U*B rows (addmm_, beta = 1) instead of autograd padding the slice's
    gradient to hp's shape and adding the two (a 124 MB zero fill, copy and add per step)."""

    @staticmethod
    def forward(ctx, hp, B, wp, bp, wv, bv, w1, b1, w2, b2, dt, perm):
        yp, yv, hsaved = _headconv_forward(hp, wp, bp, wv, bv)
        n, C, H, W = hp.shape
        a, r, xs, ws = _bigk2_forward(hp[B:].permute(0, 2, 3, 1).reshape(n - B, C * H * W), w1, b1, w2, b2, dt, perm)
        ctx.save_for_backward(hp, hsaved[0], hsaved[1], wp, bp, wv, bv, ws, w1, w2)
        ctx.O, ctx.B, ctx.perm = hsaved[2], B, perm
        return yp, yv, a, r

    @staticmethod
    def backward(ctx, gyp, gyv, ga, gr):
        hp, w0m, w1m, wp, bp, wv, bv, ws, w1, w2 = ctx.saved_tensors
        B = ctx.B
        dx, gh = _headconv_backward(hp, (w0m, w1m, ctx.O), (wp, bp, wv, bv), gyp, gyv)
        n, C, H, W = hp.shape
        xs = hp[B:].permute(0, 2, 3, 1).reshape(n - B, C * H * W)
        gview = dx[B:].permute(0, 2, 3, 1).view(n - B, C * H * W)  # channels-last rows: a view of dx
        needs = ctx.needs_input_grad
        _, gb = _bigk2_backward(xs, ws, w1, w2, ctx.perm, ga, gr, (False,) + tuple(needs[6:10]), gx_acc=gview)
        return (dx, None, *gh, *gb, None, None)


def _linear_flat_pair(lin1, lin2, h):
    """(lin1(flat h), lin2(flat h)) — one _BigKLinear2 GEMM on the channels-last flatten under GPU autocast."""
    n = h.shape[0]
    if (FLAT_NHWC and h.is_cuda and torch.is_autocast_enabled("cuda") and h.dim() == 4 and not h.is_contiguous()
            and h.is_contiguous(memory_format=torch.channels_last) and lin1.bias is not None and lin2.bias is not None):
        C, HW = h.shape[1], h.shape[2] * h.shape[3]
        K = C * HW
        if (K >= 4096 and K % _BigKLinear.SPLIT == 0 and lin1.weight.shape[1] == K and lin2.weight.shape[1] == K):
            return _BigKLinear2.apply(h.permute(0, 2, 3, 1).reshape(n, K), lin1.weight, lin1.bias, lin2.weight,
                                      lin2.bias, torch.get_autocast_dtype("cuda"), (C, HW))
    return _linear_flat(lin1, h), _linear_flat(lin2, h)


def _linear(lin, x):
    """lin(x), with K = 28,800 Linears under GPU autocast on ``_BigKLinear``."""
    if (x.is_cuda and torch.is_autocast_enabled("cuda") and x.dim() == 2 and x.shape[1] >= 4096
            and x.shape[1] % _BigKLinear.SPLIT == 0):
        return _BigKLinear.apply(x, lin.weight, lin.bias, torch.get_autocast_dtype("cuda"))
    return lin(x)


def _linear_flat(lin, h):
    """lin(h flattened per row in the reference's NCHW order, network.py:95,105).  A channels-last
    hidden state under GPU autocast is flattened as a view in (p, c) order and meets W's columns
    reordered the same way (_BigKLinear perm): no transposing copy of h per use."""
    n = h.shape[0]
    if (FLAT_NHWC and h.is_cuda and torch.is_autocast_enabled("cuda") and h.dim() == 4 and not h.is_contiguous()
            and h.is_contiguous(memory_format=torch.channels_last)):
        C, HW = h.shape[1], h.shape[2] * h.shape[3]
        K = C * HW
        if K >= 4096 and K % _BigKLinear.SPLIT == 0 and lin.weight.shape[1] == K:
            return _BigKLinear.apply(h.permute(0, 2, 3, 1).reshape(n, K), lin.weight, lin.bias,
                                     torch.get_autocast_dtype("cuda"), (C, HW))
    return _linear(lin, h.reshape(n, -1))


class _Projection(nn.Module):
    def __init__(self, din, hidden=512, out=512):
        super().__init__()
        self.fc1, self.bn1, self.fc2 = nn.Linear(din, hidden), nn.BatchNorm1d(hidden, eps=1e-4), nn.Linear(hidden, out)

    def forward(self, h, mask=None):
        return self.fc2(_bn_act(self.bn1, _linear_flat(self.fc1, h), mask))


class TrainNet(nn.Module):
    """GomokuNetEZ with the reference's state_dict keys (network.py:103-151).  The optional
    ``mask`` of every forward restricts training-mode BatchNorm statistics to those rows."""

    def __init__(self, cfg, reference_init=True):
        super().__init__()
        c, H, B, hd = cfg.NUM_FILTERS, cfg.BOARD_SIZE, cfg.NUM_RES_BLOCKS, cfg.HEAD_HIDDEN_DIM
        self.cfg = cfg
        self.representation_net = _Trunk(3, c, B)
        self.prediction_net = _Prediction(c, H, hd, cfg.VALUE_SUPPORT_BINS)
        self.dynamics_net = _Dynamics(c, H, B, hd, cfg.REWARD_SUPPORT_BINS)
        self.projection_net = _Projection(c * H * H)
        if reference_init:  # network.py:125-126: residual branches start switched off
            for m in self.modules():
                if isinstance(m, _Block):
                    nn.init.zeros_(m.bn2.weight)

    channels_last = False  # set by Trainer(channels_last=True): activations in NHWC memory format

    def representation(self, obs, mask=None, segments=1):
        """``segments`` > 1 (no_grad): obs holds that many equal batches (each with its own BatchNorm statistics
        and running-statistic update, in order): the five consistency representations as one pass."""
        if self.channels_last:
            obs = obs.contiguous(memory_format=torch.channels_last)
        if segments > 1:
            return self.representation_net(obs, mask, segments)
        return self.representation_net(obs, mask)

    def prediction(self, h, mask=None):
        return self.prediction_net(h, mask)

    def dynamics(self, h, a, mask=None, reward=True, emb=None):
        return self.dynamics_net(h, a, mask, reward, emb)

    def project(self, h, with_grad=True, mask=None):
        if with_grad:
            return self.projection_net(h, mask)
        with torch.no_grad():
            return self.projection_net(h, mask)

    @torch.no_grad()
    def initial_value(self, obs, f16=False):
        """initial_inference's value scalar (network.py:137-143), eval mode.  ``f16``: the representation
        trunk's convolutions with f16 operands and f32 accumulation (autocast; the residual convs on the HIP
        kernels): the 10-bit mantissa the reference's float32 target forward gets from its CUDA GPU's
        default TF32 convolutions (loss.py:54-55 runs outside autocast; torch.backends.cudnn.allow_tf32 =
        True); the prediction heads stay float32."""
        self.eval()
        with torch.autocast("cuda", dtype=torch.float16, enabled=bool(f16) and obs.is_cuda):
            h = self.representation(obs)
        _, vl = self.prediction(h.float())  # the heads' linears in float32, as matmuls on CUDA (no TF32 default)
        c = self.cfg
        return support_to_scalar(vl.float(), c.VALUE_SUPPORT_MIN, c.VALUE_SUPPORT_MAX, c.VALUE_SUPPORT_BINS)


# ------------------------------------------------------------------------------ loss
def barlow_loss(z1, z2, lam, mask=None):
    """loss.py:10-27: Barlow-twins cross-correlation loss of batch-standardised projections
    (BatchNorm1d without affine/running stats, eps 1e-5), over the rows where ``mask`` (bool [B])
    is set — the reference's sub-batch — without gathering them."""
    z1, z2 = z1.float(), z2.float()
    if mask is None:
        w = torch.ones(z1.shape[0], 1, device=z1.device)
    else:
        w = mask.to(torch.float32)[:, None]
    n = w.sum().clamp(min=1.0)

    def std(z):
        zc = z - (z * w).sum(0, keepdim=True) / n
        return zc * torch.rsqrt((zc * zc * w).sum(0, keepdim=True) / n + 1e-5) * w

    c = (std(z1).t() @ std(z2)) / n
    diag = torch.diagonal(c)
    on = (diag - 1).pow(2).sum()
    off = c.pow(2).sum() - diag.pow(2).sum()
    return on + lam * off


def barlow_loss_steps(z1, z2, lam, mask):
    """barlow_loss of U unroll steps at once: z1, z2 [U, B, D], mask bool [U, B] -> [U] (each step's
    loss over its own live rows; one batched standardisation and one bmm instead of U of each)."""
    z1, z2 = z1.float(), z2.float()
    w = mask.to(torch.float32)[..., None]
    n = w.sum(1, keepdim=True).clamp(min=1.0)  # [U, 1, 1]

    def std(z):
        zc = z - (z * w).sum(1, keepdim=True) / n
        return zc * torch.rsqrt((zc * zc * w).sum(1, keepdim=True) / n + 1e-5) * w

    c = torch.bmm(std(z1).transpose(1, 2), std(z2)) / n  # [U, D, D]
    diag = torch.diagonal(c, dim1=1, dim2=2)
    on = (diag - 1).pow(2).sum(1)
    off = c.pow(2).sum((1, 2)) - diag.pow(2).sum(1)
    return on + lam * off


def augment(obs, pi, act, k, flip):
    """loss.py:36-51: rotate the board planes k quarter turns (and mirror), the policies and the
    action indices with them.  obs [B, U+1, 3, H, W]; pi [B, U+1, A]; act [B, U] (-1 kept)."""
    B, U1, _, H, W = obs.shape
    o = torch.rot90(obs, k, dims=(3, 4))
    p = torch.rot90(pi.reshape(B, U1, H, W), k, dims=(2, 3))
    if flip:
        o, p = torch.flip(o, dims=(4,)), torch.flip(p, dims=(3,))
    r, c = act // W, act % W
    if k == 1:
        r, c = c, W - 1 - r
    elif k == 2:
        r, c = H - 1 - r, W - 1 - c
    elif k == 3:
        r, c = H - 1 - c, r
    if flip:
        c = W - 1 - c
    return o, p.reshape(B, U1, H * W), r * W + c


def value_targets(rew, mcts_val, last_value, cfg):
    """loss.py:53-65: z_i = sum_{j<n, i+j<U} g^j r_{i+j} + g^n (v_{i+n} if i+n <= U else V_target(obs_U))."""
    U, n, g = cfg.NUM_UNROLL_STEPS, cfg.N_STEPS, cfg.DISCOUNT
    # every i at once, the same operations per element in the same order as the per-i loop of the reference
    # (z_i = 0 + g^0 r_i + g^1 r_{i+1} + ..., then + g^n boot_i): bit-identical, ~13 launches instead of ~48
    z = torch.zeros_like(mcts_val)
    for j in range(min(n, U)):
        z[:, :U - j] += (g ** j) * rew[:, j:U]
    B = mcts_val.shape[0]
    if n > U:
        boot = last_value[:, None]
    else:
        boot = torch.cat((mcts_val[:, n:U + 1], last_value[:, None].expand(B, n)), 1)
    return z + (g ** n) * boot


class _HalveGrad(torch.autograd.Function):
    """Identity forward, gradient x 0.5 (loss.py:107 ``h.register_hook(lambda g: g * 0.5)``)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * 0.5


AUTOCAST_CACHE = True  # autocast's weight casts once per step (and per graph replay), not per use: +1.3 %
# the forward's two independent no-grad parts on side HIP streams (inside the captured step too): the
# target network's float32 value (loss.py:54-55) and the five consistency representations of
# obs[s+1] (loss.py:104), overlapping the unroll's dynamics chain; results are identical (same
# kernels; every BatchNorm's running statistics are updated in the same order)
CONCURRENT_FORWARD = True
# the target network's value (loss.py:54-55) with f16 operands and f32 accumulation in the representation
# trunk (TrainNet.initial_value f16=True; heads in float32).  The reference's float32 target forward runs on
# CUDA through cuDNN with TF32 allowed by default — the same 10-bit mantissa — so this is its precision, not
# less; |dv| <= 2e-3 vs float32 (test_target_value_f16_trunk_matches_float32).  C4 step: 36.3/36.8 vs
# 33.5/33.1 steps/s (profiles/r04_trainer_ab_defer_target.txt).  False: float32 on MIOpen, A/B
TARGET_F16 = True
# the unroll steps' cross-entropies and Barlow losses batched over the steps after the unroll (one call
# each over the stacked [U, B, .] head outputs) instead of per step (False: per step, for A/B)
BATCHED_LOSS = True
# the five no-grad consistency representations of obs[1..U] (loss.py:102-104) as ONE trunk pass over the U*B
# stacked boards, each step's BatchNorm statistics over its own live rows (segmented BatchNorm: per-board conv
# statistics partials, one finalisation per layer, running statistics updated step after step as the reference's
# five calls do): 16 conv launches of U*B boards instead of 80 of B, a fifth of the BatchNorm launches
BATCHED_CONSISTENCY = True
_SIDE_STREAMS = {}


def consistency_representations(model, obs, masks):
    """[representation(obs[:, s + 1], mask=masks[s]) for s < U] as one segmented pass (BATCHED_CONSISTENCY):
    the same values as the U separate calls (per-step BatchNorm statistics; running statistics in step order)."""
    U, B = len(masks), obs.shape[0]
    o = obs[:, 1:U + 1].transpose(0, 1).reshape(U * B, *obs.shape[2:])  # step-major: segment s = step s
    th = model.representation(o, mask=torch.stack(masks).reshape(U * B), segments=U)
    out = _StepList(th.split(B))
    out.stacked = th  # the batched heads take the U steps as this one tensor (no re-concatenation)
    return out


class _StepList(list):
    """per-step tensors that are consecutive row blocks of one tensor, ``stacked``"""
    stacked = None


# the heads of every unroll step taken after the unroll, each as ONE pass over the stacked steps (loss.py:70,96-106
# call prediction / reward / projection once per step): the six predictions over [(U+1)B] rows, the five reward
# heads and the five projections of the dynamics states over [UB] rows through one shared-input GEMM
# (_BigKLinear2), the five consistency targets' projections over [UB] rows.  Every BatchNorm in them normalises each
# step over ITS OWN live rows (_bn_seg_grad) and the running statistics are updated in the reference's call order
# (the projection's: dynamics step s, then target s, step after step; _bn_running_update).  The heads only feed the
# losses, so nothing in the unroll waits on them.  (False: per step, A/B)
BATCHED_HEADS = True


def _bn_seg_grad(mod, x, ms):
    """Training-mode BatchNorm of ``ms.shape[0]`` equal row segments of x [(nseg*B), C(, H, W)] (autograd allowed),
    segment s over its rows where ms[s] (bool [nseg, B]) is set — ``_bn`` of each segment, in float32 — WITHOUT the
    running-statistics update: returns (y float32 shaped like x, (mean [nseg, C], unbiased var [nseg, C], ok [nseg]))
    for ``_bn_running_update``."""
    nseg, B = ms.shape
    C = x.shape[1]
    xv = x.float().reshape(nseg, B, C, -1)  # a view for channels-last 4-D (H, W merge)
    S = xv.shape[3]
    w = ms.to(torch.float32)[:, :, None, None]
    nv = ms.sum(1)
    n = nv.to(torch.float32) * S
    ns = n.clamp(min=1.0)[:, None, None, None]
    mean = (xv * w).sum((1, 3), keepdim=True) / ns
    xc = xv - mean
    var = (xc * xc * w).sum((1, 3), keepdim=True) / ns
    y = xc * (torch.rsqrt(var + mod.eps) * mod.weight[:, None]) + mod.bias[:, None]
    y = y.reshape(x.shape)
    with torch.no_grad():
        unb = var.reshape(nseg, C) * (n / (n - 1).clamp(min=1.0))[:, None]
        st = (mean.reshape(nseg, C).detach(), unb.detach(), nv > 0)
    return y, st


# the batched heads' segmented BatchNorms on one HIP kernel each way (gmz_seg_bn_forward / _backward, running
# statistics inside the forward) instead of the PyTorch ops of _bn_seg_grad — for the BatchNorms with at least
# SEG_BN_HIP_MIN_C channels (the projection's bn1, C = 512: one workgroup per channel over 5 x 360 rows).  The 1- and
# 2-channel heads stay on PyTorch: one workgroup per channel serialises their 486 K elements (all four on HIP: 33.2 /
# 34.0 vs 40.1 / 40.6 steps/s, profiles/r05_seg_bn_ab.txt).  False: every call on PyTorch (A/B)
SEG_BN_HIP = True
SEG_BN_HIP_MIN_C = 64


# the 1- and 2-channel heads' segmented BatchNorms (C <= _SEG_BN_SMALL_C) on gmz_seg_bn_*_small: (segment, chunk)
# workgroups over every channel instead of one workgroup per channel (SEG_BN_SMALL; False: PyTorch's _bn_seg_grad)
SEG_BN_SMALL = True
_SEG_BN_SMALL_C = 8
_SBS_WS = {}


def _seg_bn_small_ws(nseg, C, device):
    import ctypes
    from . import _lib
    if nseg not in _SBS_WS:
        n = ctypes.c_size_t()
        _lib.check(_lib.load().gmz_seg_bn_small_workspace_bytes(nseg, C, ctypes.byref(n)))
        _SBS_WS[nseg] = n.value
    return torch.empty((_SBS_WS[nseg] + 7) // 8, dtype=torch.float64, device=device)


class _SegBN(torch.autograd.Function):
    """_bn_seg_grad's values and gradients for x [nseg*B, C(, H, W)] (channels-last 4-D or contiguous 2-D) on the
    GPU: y float32 like x's layout, and the stats [3*nseg*C + nseg] (mean, invstd, unbiased var, live rows)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, m, nseg, eps, update, momentum, rmean, rvar, nbt, pre):
        from . import _lib
        N, C = x.shape[0], x.shape[1]
        S = x[0, 0].numel() if x.dim() > 2 else 1
        if x.dim() == 4:
            y = torch.empty((N, x.shape[2], x.shape[3], C), dtype=torch.float32, device=x.device).permute(0, 3, 1, 2)
        else:
            y = torch.empty((N, C), dtype=torch.float32, device=x.device)
        st = torch.empty(3 * nseg * C + nseg, dtype=torch.float32, device=x.device)
        if C <= _SEG_BN_SMALL_C:  # few channels: (segment, chunk) workgroups over every channel
            ws = _seg_bn_small_ws(nseg, C, x.device)
            _lib.check(_lib.load().gmz_seg_bn_forward_small(
                _BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(m), nseg, N // nseg, S, C, _lib.ptr(gamma), _lib.ptr(beta),
                float(eps), _lib.ptr(y), _lib.ptr(st), _lib.nbytes(st), int(update), float(momentum), _lib.ptr(rmean),
                _lib.ptr(rvar), _lib.ptr(nbt), _lib.ptr(pre), _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr()))
        else:
            _lib.check(_lib.load().gmz_seg_bn_forward(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(m), nseg, N // nseg, S, C,
                                                      _lib.ptr(gamma), _lib.ptr(beta), float(eps), _lib.ptr(y),
                                                      _lib.ptr(st), _lib.nbytes(st), int(update), float(momentum),
                                                      _lib.ptr(rmean), _lib.ptr(rvar), _lib.ptr(nbt), _lib.ptr(pre),
                                                      _lib.stream_ptr()))
        ctx.save_for_backward(x, gamma, beta, st, m)
        ctx.nseg = nseg
        ctx.mark_non_differentiable(st)
        return y, st

    @staticmethod
    def backward(ctx, gy, _gst):
        from . import _lib
        x, gamma, beta, st, m = ctx.saved_tensors
        N, C = x.shape[0], x.shape[1]
        S = x[0, 0].numel() if x.dim() > 2 else 1
        dy = gy.float()
        dy = dy.permute(0, 2, 3, 1).contiguous() if x.dim() == 4 else dy.contiguous()  # [N][S][C] rows
        dx = torch.empty_like(x)
        direct = (_DIRECT_GRAD[0] and gamma.grad is not None and beta.grad is not None
                  and gamma.grad.dtype == torch.float32 and beta.grad.dtype == torch.float32
                  and gamma.grad.is_contiguous() and beta.grad.is_contiguous())
        dg = gamma.grad if direct else torch.empty(C, dtype=torch.float32, device=x.device)
        db = beta.grad if direct else torch.empty(C, dtype=torch.float32, device=x.device)
        if C <= _SEG_BN_SMALL_C:
            ws = _seg_bn_small_ws(ctx.nseg, C, x.device)
            _lib.check(_lib.load().gmz_seg_bn_backward_small(
                _BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(dy), _lib.ptr(m), ctx.nseg, N // ctx.nseg, S, C,
                _lib.ptr(gamma), _lib.ptr(st), _lib.nbytes(st), _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db), int(direct),
                _lib.ptr(ws), _lib.nbytes(ws), _lib.stream_ptr()))
        else:
            _lib.check(_lib.load().gmz_seg_bn_backward(_BN_DTYPES[x.dtype], _lib.ptr(x), _lib.ptr(dy), _lib.ptr(m),
                                                       ctx.nseg, N // ctx.nseg, S, C, _lib.ptr(gamma), _lib.ptr(st),
                                                       _lib.nbytes(st), _lib.ptr(dx), _lib.ptr(dg), _lib.ptr(db),
                                                       int(direct), _lib.stream_ptr()))
        if direct:
            return dx, None, None, None, None, None, None, None, None, None, None, None
        return dx, dg, db, None, None, None, None, None, None, None, None, None


def _bn_steps(mod, x, ms, update=True, pre=None):
    """Training-mode BatchNorm of the ms.shape[0] stacked steps of x (each over its own live rows), the running
    statistics updated (update) in step order — after ``pre``'s step by step when given (a previous call's handle:
    the projection's dynamics steps before its targets').  Returns (y float32, handle).  GPU: _SegBN (HIP); CPU
    and other layouts: _bn_seg_grad + _bn_running_update."""
    nseg = ms.shape[0]
    hip = (SEG_BN_HIP and FUSED_BN and x.is_cuda and x.dtype in _BN_DTYPES and mod.momentum is not None
           and (x.shape[1] >= SEG_BN_HIP_MIN_C or (SEG_BN_SMALL and x.shape[1] <= _SEG_BN_SMALL_C))
           and nseg <= 32 and x.shape[0] % nseg == 0
           and ((x.dim() == 2 and x.is_contiguous()) or (x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last)))
           and (pre is None or pre[0] == "hip"))
    if hip:
        m = ms.reshape(-1).contiguous().view(torch.uint8)
        y, st = _SegBN.apply(x, mod.weight, mod.bias, m, nseg, mod.eps, bool(update), mod.momentum, mod.running_mean,
                             mod.running_var, mod.num_batches_tracked, None if pre is None else pre[1])
        return y, ("hip", st)
    y, st = _bn_seg_grad(mod, x, ms)
    if update:
        if pre is None:
            _bn_running_update(mod, [st])
        else:  # interleaved: pre's step s, then this call's step s
            ps = pre[1] if pre[0] == "torch" else _seg_stats_as_torch(pre[1], nseg, x.shape[1])
            _bn_running_update(mod, [tuple(torch.stack((a, b), 1).reshape(2 * nseg, *a.shape[1:])
                                           for a, b in zip(ps, st))])
    return y, ("torch", st)


def _seg_stats_as_torch(flat, nseg, C):
    """A _SegBN handle's flat statistics [mean | invstd | unbiased var | live count] (gmz_seg_bn_forward) as the
    (mean [nseg, C], unbiased var [nseg, C], ok [nseg]) tuple of _bn_seg_grad: when the dynamics projection's call
    took the HIP kernel and the targets' call cannot, the interleaved running-statistics update still gets
    (mean, var, ok) per step."""
    f = flat.reshape(-1)
    n = nseg * C
    return f[:n].view(nseg, C), f[2 * n:3 * n].view(nseg, C), f[3 * n:3 * n + nseg] > 0


def _bn_running_update(mod, stats):
    """The running-statistics updates of a sequence of training-mode BatchNorm calls (``stats``: a list of
    _bn_seg_grad results, applied in list order, segment by segment; a segment with no live row is skipped, as the
    reference skips that step) in closed form: r <- r * prod_k f_k + sum_k m ok_k v_k prod_{j>k} f_j with
    f_k = 1 - m ok_k — the sequential r <- (1 - m) r + m v_k of each call."""
    with torch.no_grad():
        mean = torch.cat([s[0] for s in stats])
        var = torch.cat([s[1] for s in stats])
        ok = torch.cat([s[2] for s in stats]).to(torch.float32)
        m = mod.momentum
        f = 1.0 - m * ok
        suf = torch.flip(torch.cumprod(torch.flip(f, (0,)), 0), (0,))  # prod_{j >= k}
        excl = torch.cat((suf[1:], torch.ones_like(suf[:1])))        # prod_{j > k}
        a = (m * ok * excl)[:, None]
        rm, rv = mod.running_mean.data, mod.running_var.data
        rm.copy_(rm * suf[0] + (a * mean).sum(0))
        rv.copy_(rv * suf[0] + (a * var).sum(0))
        mod.num_batches_tracked.data += ok.sum().to(mod.num_batches_tracked.dtype)


def _heads_input(model, hp, B):
    """_HeadsInput (the prediction convs and the projection fc1 + reward fc0 GEMM as one autograd node) when both
    fast paths apply, else None."""
    pred, proj = model.prediction_net, model.projection_net
    fc0 = model.dynamics_net.reward_fc[0]
    if not (_head_convs_hip_ok(pred, hp) and FLAT_NHWC and fc0.bias is not None and proj.fc1.bias is not None):
        return None
    C, HW = hp.shape[1], hp.shape[2] * hp.shape[3]
    K = C * HW
    if not (K % _BigKLinear.SPLIT == 0 and proj.fc1.weight.shape[1] == K and fc0.weight.shape[1] == K):
        return None
    return _HeadsInput.apply(hp, B, pred.policy_conv.weight, pred.policy_conv.bias, pred.value_conv.weight,
                             pred.value_conv.bias, proj.fc1.weight, proj.fc1.bias, fc0.weight, fc0.bias,
                             torch.get_autocast_dtype("cuda"), (C, HW))


def _prediction_seg(pred, h, ms, convs=None):
    """prediction (network.py:67-73) of nseg stacked steps h [(nseg*B), 128, H, W], each step's BatchNorms over
    its own rows ms [nseg, B]; returns (policy logits, value logits, [policy_bn stats, value_bn stats]).
    ``convs``: the two 1x1 convs' outputs, already computed (_HeadsInput)."""
    n = h.shape[0]
    if convs is not None:
        yp, yv = convs
    elif _head_convs_hip_ok(pred, h):
        yp, yv = _HeadConv1x1.apply(h, pred.policy_conv.weight, pred.policy_conv.bias, pred.value_conv.weight,
                                    pred.value_conv.bias)
    else:
        yp, yv = _conv1x1(pred.policy_conv, h), _conv1x1(pred.value_conv, h)
    bp, _ = _bn_steps(pred.policy_bn, yp, ms)  # running statistics updated in step order
    bv, _ = _bn_steps(pred.value_bn, yv, ms)
    pol = pred.policy_fc(F.relu(bp).reshape(n, -1))
    v = F.relu(pred.value_fc1(F.relu(bv).reshape(n, -1)))
    return pol, pred.value_fc2(v)


def _reward_projection_seg(model, h, ms, first=None):
    """The reward head (network.py:105-106) and the projection (loss.py:97: project(h, with_grad=True)) of U stacked
    dynamics states h [(U*B), ...]: their first Linears in one GEMM (_linear_flat_pair), the projection's
    BatchNorm per step over ms [U, B]; returns (reward logits, projection, bn1 stats).  ``first``: the two first
    Linears' outputs, already computed (_HeadsInput)."""
    proj = model.projection_net
    fc0, act, fc2 = model.dynamics_net.reward_fc
    a, r = first if first is not None else _linear_flat_pair(proj.fc1, fc0, h)
    b, st = _bn_steps(proj.bn1, a, ms, update=False)  # its running statistics go with the targets' (interleaved)
    return fc2(act(r)), proj.fc2(F.relu(b)), st


def _projection_seg(proj, h, ms, pre):
    """projection (loss.py:104: with_grad=False) of U stacked steps, BatchNorm per step, its running statistics
    updated after ``pre``'s (the dynamics projections') step by step — the reference's order."""
    b, _ = _bn_steps(proj.bn1, _linear_flat(proj.fc1, h), ms, update=True, pre=pre)
    return proj.fc2(F.relu(b))


def _side_streams(device):
    if device not in _SIDE_STREAMS:
        _SIDE_STREAMS[device] = (torch.cuda.Stream(device), torch.cuda.Stream(device))
    return _SIDE_STREAMS[device]


def muzero_loss(model, target_model, batch, is_weights, cfg, k=None, flip=None, amp=False, amp_dtype=None,
                sync_logs=True, augmented=False):
    """loss.py:30-158.  ``batch`` = (obs [B,U+1,3,H,W], actions [B,U], rewards [B,U],
    policies [B,U+1,A], search values [B,U+1]).  ``k``/``flip``: the augmentation (default: drawn
    from numpy's global RandomState in the reference's order); ``augmented``: the batch is already
    augmented (k/flip ignored) and carries the augmented actions as a 6th member.  Returns (weighted loss tensor, (total, policy, value, reward,
    consistency) — floats, or one device tensor [5] with ``sync_logs=False`` — , |value error| at
    step 0 as a tensor).

    Fixed shapes and no host synchronisation: every unroll step runs on the full batch with the
    rows of ended games masked out of the BatchNorm statistics, the losses and the consistency
    loss, and a step with no valid row contributes nothing (the reference skips it), so the same
    kernels run every call and the step can be captured in a HIP graph."""
    obs, act, rew, pi, mval = batch[:5]
    act, rew, mval = act.long(), rew.float(), mval.float()
    if augmented:
        act_aug = batch[5]
    else:
        if k is None:
            k = np.random.randint(4)
        if flip is None:
            flip = bool(np.random.choice([True, False]))
        obs, pi, act_aug = augment(obs, pi, act, k, flip)
    model.train()
    target_model.eval()
    c, W = cfg, cfg.LOSS_WEIGHTS
    vsup = (c.VALUE_SUPPORT_MIN, c.VALUE_SUPPORT_MAX, c.VALUE_SUPPORT_BINS)
    rsup = (c.REWARD_SUPPORT_MIN, c.REWARD_SUPPORT_MAX, c.REWARD_SUPPORT_BINS)
    side = _side_streams(obs.device) if (CONCURRENT_FORWARD and obs.is_cuda) else None
    if side is not None:  # the target network's value on side stream 0, from here to its first use
        main = torch.cuda.current_stream(obs.device)
        side[0].wait_stream(main)
        with torch.cuda.stream(side[0]), torch.no_grad():
            last_v = target_model.initial_value(obs[:, -1], f16=TARGET_F16)[:, 0]
            z = value_targets(rew, mval, last_v, c)
    else:
        with torch.no_grad():
            last_v = target_model.initial_value(obs[:, -1], f16=TARGET_F16)[:, 0]
            z = value_targets(rew, mval, last_v, c)
    dev_type = obs.device.type
    zero = torch.zeros((), device=obs.device)
    with torch.autocast(dev_type, enabled=amp and dev_type == "cuda", dtype=amp_dtype or torch.float16,
                        cache_enabled=AUTOCAST_CACHE):
        h = model.representation(obs[:, 0])
        tru_h = None
        if side is not None:
            # the consistency representations of obs[1..U] (no grad) on side stream 1, in step order
            # after obs[0]'s (the representation BatchNorms' running statistics update in the
            # reference's order); their projections stay on this stream, interleaved with the dynamics'
            # projections as in the reference (the projection BatchNorm's running statistics)
            live_act = (act != -1).t().contiguous()  # [U, B]: each step's mask a contiguous row (2 launches, not U)
            masks = list(live_act)
            side[1].wait_stream(main)
            tru_h, tru_ev = [], []
            with torch.cuda.stream(side[1]), torch.no_grad():
                if BATCHED_CONSISTENCY and c.NUM_UNROLL_STEPS > 1:
                    tru_h = consistency_representations(model, obs, masks)
                    ev = torch.cuda.Event()
                    ev.record(side[1])
                    tru_ev = [ev] * c.NUM_UNROLL_STEPS
                else:
                    for s in range(c.NUM_UNROLL_STEPS):
                        tru_h.append(model.representation(obs[:, s + 1], mask=masks[s]))
                        ev = torch.cuda.Event()
                        ev.record(side[1])
                        tru_ev.append(ev)
            main.wait_stream(side[0])
            z.record_stream(main)
        elif BATCHED_CONSISTENCY and c.NUM_UNROLL_STEPS > 1:  # one stream: the batched pass right after obs[0]'s
            with torch.no_grad():
                tru_h = consistency_representations(model, obs, [act[:, s] != -1 for s in range(c.NUM_UNROLL_STEPS)])
        U = c.NUM_UNROLL_STEPS
        if BATCHED_HEADS and BATCHED_LOSS and not SUBBATCH_BN and U > 0:
            # the unroll's dynamics chain first (trunks only), then every head over the stacked steps
            zsup = scalar_to_support(z.t().contiguous(), *vsup)       # [U+1, B, bins]
            rsupt = scalar_to_support(rew.t().contiguous(), *rsup)    # [U, B, bins]
            h0, hks, mks = h, [], []
            if side is None:
                live_act = (act != -1).t().contiguous()                 # [U, B]: each step's mask a contiguous row
            a_all = torch.where(live_act, act_aug.t(), torch.zeros_like(act_aug.t())).reshape(-1)  # step-major [U*B]
            dyn_net = model.dynamics_net
            emb_all = None if _dyn_stem_hip_ok(dyn_net, h) else dyn_net.embed(a_all, h)  # every step's embedding
            B0 = h.shape[0]
            # a step with no live row counts nothing (loss.py:90-91); a count of 0/1 terms: exact in any order
            steps = live_act.any(1).to(torch.float32).sum()
            for s in range(U):
                m = live_act[s]
                hk, _ = model.dynamics(h, a_all[s * B0:(s + 1) * B0], mask=m, reward=False,
                                       emb=None if emb_all is None else emb_all[s * B0:(s + 1) * B0])
                hks.append(hk)
                mks.append(m)
                h = _HalveGrad.apply(torch.where(m[:, None, None, None], hk, h))
            ms = torch.stack(mks)                                      # [U, B]
            B = ms.shape[1]
            hp = torch.cat([h0] + hks)                                 # [(U+1)B]: step-major, step 0 = obs[0]'s
            pred = model.prediction_net
            msp = torch.cat((torch.ones_like(ms[:1]), ms))
            first = _heads_input(model, hp, B)  # the heads' first layers in one node (None: no fused path)
            pls_all, vls_all = _prediction_seg(pred, hp, msp, None if first is None else first[:2])
            rl_all, dyn_all, sdyn = _reward_projection_seg(model, hp[B:], ms, None if first is None else first[2:])
            with torch.no_grad():
                if tru_h is None:
                    tru_h = [model.representation(obs[:, s + 1], mask=mks[s]) for s in range(U)]
                elif side is not None:
                    main.wait_event(tru_ev[-1])
                th = getattr(tru_h, "stacked", None)
                if side is not None:
                    # every per-step state made on side[1] is consumed on main (by the cat, or as th itself): each
                    # is recorded on main so none returns to side[1]'s pool while main's use is still queued
                    for t in tru_h:
                        t.record_stream(main)
                if th is None:
                    th = tru_h[0] if len(tru_h) == 1 else torch.cat(tru_h)
                if side is not None:
                    th.record_stream(main)
                # the projection BatchNorm's running statistics in the reference's order: dynamics s, then target s
                tru_all = _projection_seg(model.projection_net, th, ms, sdyn)
            pl, vl = pls_all[:B], vls_all[:B]
            lp = F.cross_entropy(pl.float(), pi[:, 0], reduction="none")
            lv = F.cross_entropy(vl.float(), zsup[0], reduction="none")
            # loss.py:78 passes softmax(logits) to support_to_scalar, which applies softmax again:
            # the PER priority is computed from that doubly-softmaxed value (kept as the reference does)
            v0 = support_to_scalar(F.softmax(vl.float(), dim=1), *vsup)
            td = (v0.detach()[:, 0] - z[:, 0]).abs()
            pls, vls = pls_all[B:].view(U, B, -1), vls_all[B:].view(U, B, -1)
            rls, dyns, trus = rl_all.view(U, B, -1), dyn_all.view(U, B, -1), tru_all.view(U, B, -1)

            def ce(logits, target):
                x = logits.float().reshape(U * B, -1)
                return F.cross_entropy(x, target.reshape(U * B, -1), reduction="none").view(U, B)
            lp = lp + torch.where(ms, ce(pls, pi[:, 1:].transpose(0, 1)), zero).sum(0)
            lv = lv + torch.where(ms, ce(vls, zsup[1:]), zero).sum(0)
            lr_ = torch.where(ms, ce(rls, rsupt), zero).sum(0)
            live_s = ms.any(1).to(torch.float32)
            cons = (live_s * barlow_loss_steps(dyns, trus, c.BARLOW_LAMBDA, ms)).sum()
        else:
            pl, vl = model.prediction(h)
            lp = F.cross_entropy(pl.float(), pi[:, 0], reduction="none")
            # the support targets of every step in two calls (the per-step calls were ~10 tiny kernels each)
            # (step-major, so each step's [B, bins] block is contiguous)
            zsup = scalar_to_support(z.t().contiguous(), *vsup)       # [U+1, B, bins]
            rsupt = scalar_to_support(rew.t().contiguous(), *rsup)    # [U, B, bins]
            lv = F.cross_entropy(vl.float(), zsup[0], reduction="none")
            # loss.py:78 passes softmax(logits) to support_to_scalar, which applies softmax again:
            # the PER priority is computed from that doubly-softmaxed value (kept as the reference does)
            v0 = support_to_scalar(F.softmax(vl.float(), dim=1), *vsup)
            td = (v0.detach()[:, 0] - z[:, 0]).abs()
            lr_ = torch.zeros(obs.shape[0], device=obs.device)
            steps = zero
            cons = zero
            U = c.NUM_UNROLL_STEPS
            per_step = []  # BATCHED_LOSS: each step's head outputs, their loss terms taken after the unroll
            for s in range(U):
                m = act[:, s] != -1
                live = m.any().to(torch.float32)   # 0: the reference's `continue` (loss.py:90-91)
                steps = steps + live
                # full-batch step, row-masked BatchNorm statistics and losses (== the reference's
                # sub-batch h[m] computation, loss.py:89-107, with fixed shapes)
                hk, rl = model.dynamics(h, torch.where(m, act_aug[:, s], torch.zeros_like(act_aug[:, s])), mask=m)
                plk, vlk = model.prediction(hk, mask=m)
                if not BATCHED_LOSS:
                    lp = lp + torch.where(m, F.cross_entropy(plk.float(), pi[:, s + 1], reduction="none"), zero)
                    lv = lv + torch.where(m, F.cross_entropy(vlk.float(), zsup[s + 1],
                                                             reduction="none"), zero)
                    lr_ = lr_ + torch.where(m, F.cross_entropy(rl.float(), rsupt[s],
                                                               reduction="none"), zero)
                dyn = model.project(hk, with_grad=True, mask=m)
                with torch.no_grad():
                    if tru_h is not None and side is None:
                        tru = model.project(tru_h[s], with_grad=False, mask=m)
                    elif tru_h is not None:
                        main.wait_event(tru_ev[s])
                        tru_h[s].record_stream(main)
                        tru = model.project(tru_h[s], with_grad=False, mask=m)
                    else:
                        tru = model.project(model.representation(obs[:, s + 1], mask=m), with_grad=False, mask=m)
                if BATCHED_LOSS:
                    per_step.append((m, plk, vlk, rl, dyn, tru))
                else:
                    cons = cons + live * barlow_loss(dyn, tru, c.BARLOW_LAMBDA, m)
                h = _HalveGrad.apply(torch.where(m[:, None, None, None], hk, h))
            if BATCHED_LOSS and U > 0:
                # the U steps' cross-entropies and consistency losses as one call each over the stacked
                # [U, B, .] outputs (masked rows zeroed, summed over the steps): the same per-row values as
                # the per-step calls, ~5x fewer kernels in the forward and the backward
                ms, pls, vls, rls, dyns, trus = (torch.stack(x) for x in zip(*per_step))
                B = ms.shape[1]

                def ce(logits, target):
                    x = logits.float().reshape(U * B, -1)
                    return F.cross_entropy(x, target.reshape(U * B, -1), reduction="none").view(U, B)
                lp = lp + torch.where(ms, ce(pls, pi[:, 1:].transpose(0, 1)), zero).sum(0)
                lv = lv + torch.where(ms, ce(vls, zsup[1:]), zero).sum(0)
                lr_ = lr_ + torch.where(ms, ce(rls, rsupt), zero).sum(0)
                live_s = ms.any(1).to(torch.float32)
                cons = (live_s * barlow_loss_steps(dyns, trus, c.BARLOW_LAMBDA, ms)).sum()
    lp = lp / (steps + 1)
    lv = lv / (steps + 1)
    lr_ = lr_ / steps.clamp(min=1.0)
    cons = cons / steps.clamp(min=1.0)
    fp, fv, fr = (lp * is_weights).mean(), (lv * is_weights).mean(), (lr_ * is_weights).mean()
    total = W["policy"] * fp + W["value"] * fv + W["reward"] * fr + W["consistency"] * cons
    logs = torch.stack([x.detach().float() for x in (total, fp, fv, fr, cons)])
    if sync_logs:
        logs = tuple(float(x) for x in logs.tolist())
    return total, logs, td


# ------------------------------------------------------------------------------ replay
class ReplayBuffer:
    """Device-resident ring of TrainingSlices with the sampling of replay_buffer.py:44-106.

    Slices live in HBM as observation planes uint8 [N, U+1, 3, H, W] (0/1 planes), actions int32,
    rewards f32, policies f32 [N, U+1, A], values f32; priorities f32 [N].  Sampling: uniform
    without replacement (ENABLE_PER off, the reference default) or stratified proportional PER
    (segment i of the total priority, one uniform draw each; prefix sums + binary search give the
    same leaf as the reference's sum-tree descent), IS weights (count * p / total)^-beta / max."""

    def __init__(self, cfg, capacity=None, device="cuda"):
        c = cfg
        self.cfg, self.N = c, int(capacity or c.TRAIN_BUFFER_SIZE)
        U, H, A = c.NUM_UNROLL_STEPS, c.BOARD_SIZE, c.BOARD_SIZE * c.BOARD_SIZE
        d = torch.device(device)
        self.obs = torch.zeros(self.N, U + 1, 3, H, H, dtype=torch.uint8, device=d)
        self.act = torch.zeros(self.N, U, dtype=torch.int32, device=d)
        self.rew = torch.zeros(self.N, U, dtype=torch.float32, device=d)
        self.pol = torch.zeros(self.N, U + 1, A, dtype=torch.float32, device=d)
        self.val = torch.zeros(self.N, U + 1, dtype=torch.float32, device=d)
        self.prio = torch.zeros(self.N, dtype=torch.float32, device=d)
        self.ptr, self.count, self.max_priority, self.device = 0, 0, 1.0, d

    def __len__(self):
        return self.count

    def add(self, slices):
        """Append TrainingSlice-like objects (observation, action_history, reward_history,
        policy_history, value_history)."""
        n = len(slices)
        if n == 0:
            return
        idx = (torch.arange(n) + self.ptr) % self.N
        st = lambda f, dt: torch.from_numpy(np.stack([np.asarray(getattr(s, f)) for s in slices]).astype(dt))  # noqa: E731
        self.obs[idx] = st("observation", np.uint8).to(self.device)
        self.act[idx] = st("action_history", np.int32).to(self.device)
        self.rew[idx] = st("reward_history", np.float32).to(self.device)
        self.pol[idx] = st("policy_history", np.float32).to(self.device)
        self.val[idx] = st("value_history", np.float32).to(self.device)
        if self.cfg.ENABLE_PER:
            self.prio[idx.to(self.device)] = torch.as_tensor(self.max_priority, dtype=torch.float32, device=self.device)
        else:
            self.prio[idx.to(self.device)] = 1.0
        self.ptr = (self.ptr + n) % self.N
        self.count = min(self.N, self.count + n)

    def add_arrays(self, obs, act, rew, pol, val):
        """Append n slices given as stacked arrays/tensors (obs [n,U+1,3,H,W] 0/1, act [n,U] int,
        rew [n,U], pol [n,U+1,A], val [n,U+1]); same ring semantics as :meth:`add`."""
        n = int(obs.shape[0])
        if n == 0:
            return
        if n > self.N:  # only the newest N survive the ring
            obs, act, rew, pol, val = obs[-self.N:], act[-self.N:], rew[-self.N:], pol[-self.N:], val[-self.N:]
            n = self.N
        idx = ((torch.arange(n) + self.ptr) % self.N).to(self.device)
        def dv(x, dt):
            if isinstance(x, np.ndarray) and not x.flags.writeable:
                x = np.array(x)  # torch.as_tensor warns on (and would alias) a read-only numpy array
            return torch.as_tensor(x).to(self.device, dt)
        self.obs[idx] = dv(obs, torch.uint8)
        self.act[idx] = dv(act, torch.int32)
        self.rew[idx] = dv(rew, torch.float32)
        self.pol[idx] = dv(pol, torch.float32)
        self.val[idx] = dv(val, torch.float32)
        if self.cfg.ENABLE_PER:
            self.prio[idx] = torch.as_tensor(self.max_priority, dtype=torch.float32, device=self.device)
        else:
            self.prio[idx] = 1.0
        self.ptr = (self.ptr + n) % self.N
        self.count = min(self.N, self.count + n)

    def sample(self, B, rng=np.random, dist=None):
        """replay_buffer.py:58-94.  ``dist``: torch.distributed when this buffer is one rank's shard of
        a data-parallel trainer (sharded PER): each rank samples its B slices from its
        own shard (rank chosen uniformly, then proportional within the shard, so a slice's sampling
        probability is p_i / (N * T_rank)); the IS weights use the GLOBAL slice count (one all-reduce
        SUM) and are normalised by the max over the global batch (one all-reduce MAX).  With one rank
        this is exactly the reference's (count * p_i / T)^-beta / max."""
        if self.count < B:
            return None
        if self.cfg.ENABLE_PER:
            # no host synchronisation: the reference's per-segment draws uniform(seg*i, seg*(i+1))
            # = seg * (i + random_sample()) take B host uniforms; the total stays on the device
            p = self.prio[: self.count].double()
            cum = torch.cumsum(p, 0)
            total = cum[-1]
            r = torch.from_numpy(rng.random_sample(B)).to(self.device, non_blocking=True)
            u = (torch.arange(B, device=self.device, dtype=torch.float64) + r) * (total / B)
            idx = torch.searchsorted(cum, u).clamp_max(self.count - 1)
            prob = p[idx] / total
            count = float(self.count)
            if dist is not None and dist.get_world_size() > 1:
                count = _allreduce(torch.tensor([count], dtype=torch.float64, device=self.device), dist)
                prob = prob / dist.get_world_size()
            w = (count * prob) ** (-self.cfg.PER_BETA)
            wmax = w.max()
            if dist is not None and dist.get_world_size() > 1:
                wmax = _allreduce(wmax.reshape(1), dist, max_op=True)[0]
            w = (w / wmax).float()
        else:
            idx = torch.from_numpy(rng.choice(self.count, B, replace=False)).to(self.device)
            w = torch.ones(B, device=self.device)
        batch = (self.obs[idx].float(), self.act[idx], self.rew[idx], self.pol[idx], self.val[idx])
        return batch, idx, w

    def update_priorities(self, idx, td, dist=None):
        """replay_buffer.py:96-101; with ``dist`` the running max priority (the priority of newly added
        slices) is kept global by an all-reduce MAX, so every shard admits new slices alike."""
        if not self.cfg.ENABLE_PER:
            return
        p = td.abs().to(self.device).float() + self.cfg.PER_EPSILON
        m = torch.maximum(torch.as_tensor(self.max_priority, device=self.device, dtype=torch.float32), p.max())
        if dist is not None and dist.get_world_size() > 1:
            m = _allreduce(m.reshape(1), dist, max_op=True)[0]
        self.max_priority = m  # device scalar
        self.prio[idx] = p


def _allreduce(t, dist, max_op=False):
    """All-reduce a small tensor (SUM or MAX) on any backend: RCCL takes device tensors, gloo host
    tensors.  Returns the reduced tensor on ``t``'s device."""
    op = dist.ReduceOp.MAX if max_op else dist.ReduceOp.SUM
    if dist.get_backend() == "gloo" and t.is_cuda:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        out = h.to(t.device)
    else:
        dist.all_reduce(t, op=op)
        out = t
    return out


# ------------------------------------------------------------------------------ trainer
class Trainer:
    """training_worker's step (workers.py:452-463, 556-584) without the queues: Adam with weight
    decay, LinearLR warm-up (1000 updates) then cosine annealing to 1e-7 over 200k updates, AMP
    grad scaler, gradient clipping, soft target update after every optimiser step.  Under an
    initialised torch.distributed every rank trains on its own batch and the gradients are averaged
    with one all-reduce of a flat bucket (RCCL) before the update.

    MI355X execution: every parameter's gradient is a view of ONE flat buffer (the all-reduce
    bucket, no gather/scatter copies); on the GPU the optimiser is the fused multi-tensor Adam with
    the learning rate as a device tensor and the AMP inf-check handed to it on the device; with
    ``graph=True`` (default on cuda, GRADIENT_ACCUMULATION_STEPS == 1) the whole step — target-net
    bootstrap, loss, backward, unscale, clip, Adam, scale update, soft target update — is captured
    once into a HIP graph and replayed (distributed: with the RCCL all-reduces inside it).  The
    batch is augmented eagerly into static input buffers before each replay.  The first ``graph_warmup`` steps run eagerly (they are real steps)."""

    def __init__(self, cfg=None, device="cuda", state_dict=None, amp=None, amp_dtype=None, channels_last=None,
                 graph=None, graph_warmup=3):
        c = cfg if isinstance(cfg, TrainConfig) else TrainConfig.from_any(cfg)
        self.cfg, self.device = c, torch.device(device)
        self.model = TrainNet(c).to(self.device)
        if state_dict is not None:
            self.model.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}, strict=False)
        self.target = TrainNet(c).to(self.device)
        self.target.load_state_dict(self.model.state_dict())
        self.amp = (self.device.type == "cuda") if amp is None else amp
        self.amp_dtype = amp_dtype  # None: float16 as the reference's torch.amp.autocast('cuda')
        # default on the GPU: channels-last (18.8 vs 13.8 steps/s at config C4 with the same kernels)
        channels_last = (self.device.type == "cuda") if channels_last is None else channels_last
        self.channels_last = channels_last
        if channels_last:  # NHWC activations: MIOpen's NHWC convolutions without layout transposes
            self.model = self.model.to(memory_format=torch.channels_last)
            self.model.channels_last = True
            # the target network's value (loss.py:54-55) runs in float32 like the reference's, outside
            # autocast.  With MIOpen Find (torch.backends.cudnn.benchmark) its NHWC fp32 implicit GEMM
            # takes 0.19 ms per 360-board conv (128 TFLOP/s, fp32 MFMA), so the target goes channels-last
            # too; without Find MIOpen's immediate-mode NHWC fp32 pick takes 0.51 ms and its NCHW fp32
            # Winograd 0.26 ms, so the target stays NCHW
            if torch.backends.cudnn.benchmark or TARGET_F16:  # (f16: the HIP residual convs need NHWC)
                self.target = self.target.to(memory_format=torch.channels_last)
                self.target.channels_last = True
        import torch.distributed as dist
        self.dist = dist if (dist.is_available() and dist.is_initialized()) else None
        if self.dist is not None:  # every rank starts from rank 0's weights
            for t in list(self.model.parameters()) + list(self.model.buffers()):
                self.dist.broadcast(t.data, 0)
            self.target.load_state_dict(self.model.state_dict())
        # gradients as views of one flat buffer, the all-reduce operand, in two buckets: [A | B], B = the residual
        # blocks' 3x3 conv weights, whose gradients the deferred weight-gradient pass (flush_wgrads, DEFER_WGRAD)
        # writes after the backward, A = everything else, final when the backward ends.  Data parallel: A's
        # all-reduce runs while B's weight gradients are computed (workers.py:565-583).  The optimiser
        # keeps the reference's parameter order (its state_dict indices); only the gradient views are reordered.
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        late = {id(m.conv1.weight) for m in self.model.modules() if isinstance(m, _Block)}
        late |= {id(m.conv2.weight) for m in self.model.modules() if isinstance(m, _Block)}
        late |= {id(m.conv.weight) for m in self.model.modules() if isinstance(m, _Dynamics)}  # DYN_STEM_HIP
        layout = [p for p in self.params if id(p) not in late] + [p for p in self.params if id(p) in late]
        self.flat_grad = torch.zeros(sum(p.numel() for p in self.params), dtype=torch.float32, device=self.device)
        self._bucket_a = sum(p.numel() for p in layout if id(p) not in late)
        off = 0
        for p in layout:
            p.grad = self.flat_grad[off:off + p.numel()].as_strided(p.shape, p.stride())  # same layout as p
            off += p.numel()
        # the communication clock of the data-parallel step (gmz_comm_stamp, int64 [5]: captured into the step's graph
        # with the all-reduces, where host events cannot time): bucket A issued, B's weight gradients done, both averaged
        self._comm_clock = (torch.zeros(5, dtype=torch.int64, device=self.device)
                            if self.dist is not None and self.device.type == "cuda" else None)
        cuda = self.device.type == "cuda"
        lr = torch.tensor(c.LEARNING_RATE, device=self.device) if cuda else c.LEARNING_RATE
        self.opt = torch.optim.Adam(self.params, lr=lr, weight_decay=c.WEIGHT_DECAY,
                                    **(dict(fused=True, capturable=True) if cuda else {}))
        acc = max(1, c.GRADIENT_ACCUMULATION_STEPS)
        warm, total = 1000 // acc, 200000 // acc
        self.sched = torch.optim.lr_scheduler.SequentialLR(self.opt, [
            torch.optim.lr_scheduler.LinearLR(self.opt, start_factor=0.01, total_iters=warm),
            torch.optim.lr_scheduler.CosineAnnealingLR(self.opt, T_max=total - warm, eta_min=1e-7)], milestones=[warm])
        self.scaler = torch.amp.GradScaler(self.device.type, enabled=self.amp and amp_dtype in (None, torch.float16))
        self.step_count = 0
        self.graph = (cuda and acc == 1) if graph is None else (bool(graph) and cuda and acc == 1)
        self.graph_warmup = max(1, int(graph_warmup))  # eager steps first: lazy AMP/optimiser state
        self._graphs = None  # the captured step: a CUDAGraph, or (step, flush, update) graphs (see _capture)
        self._fopt = None  # FUSED_OPT's buffers (built at the first update)
        self.graph_allreduce = False  # True once the captured step holds the RCCL all-reduces
        self._static = None
        self._pack_tables = {}  # BATCH_REPACK's job tables

    # ------------------------------------------------------------------ step pieces
    def _forward_backward(self, batch, is_weights, acc=1, k=None, flip=None, augmented=False, flush=True):
        """Loss and backward; ``flush`` = False leaves the deferred 3x3 weight gradients queued (bucket B) for
        ``flush_wgrads`` after bucket A's all-reduce has been issued."""
        if BATCH_REPACK and self.device.type == "cuda":
            _repack_stale(list(self.model.parameters()) + list(self.target.parameters()), self._pack_tables)
        loss, logs, td = muzero_loss(self.model, self.target, batch, is_weights, self.cfg, k=k, flip=flip,
                                     amp=self.amp, amp_dtype=self.amp_dtype, sync_logs=False, augmented=augmented)
        _DIRECT_GRAD[0] = True
        ok = False
        try:
            self.scaler.scale(loss / acc).backward()
            if flush:
                flush_wgrads()
            ok = True
        finally:
            _DIRECT_GRAD[0] = False
            if flush or not ok:
                _PENDING_WGRAD.clear()
        return logs, td

    def _flush(self):
        try:
            flush_wgrads()
        finally:
            _PENDING_WGRAD.clear()

    def _stamp(self, phase):
        if self._comm_clock is not None:
            from . import _lib
            _lib.check(_lib.load().gmz_comm_stamp(_lib.ptr(self._comm_clock), phase, _lib.stream_ptr()))

    def _allreduce_start(self):
        """Bucket A's all-reduce, issued asynchronously (RCCL on its own stream, after the backward's kernels)."""
        if self.dist is None:
            return None
        self._stamp(0)
        return self.dist.all_reduce(self.flat_grad[:self._bucket_a], async_op=True)

    def _mark_flushed(self):
        """Bucket B's weight gradients are enqueued (the compute stream's work between A's issue and B's)."""
        self._stamp(1)

    def _allreduce_finish(self, work):
        """Bucket B's all-reduce (its gradients are final once flush_wgrads ran), then both buckets averaged."""
        if self.dist is None:
            return
        if self._bucket_a < self.flat_grad.numel():
            self.dist.all_reduce(self.flat_grad[self._bucket_a:])
        work.wait()
        self.flat_grad.div_(self.dist.get_world_size())
        self._stamp(2)

    def _allreduce(self):
        if self.dist is not None:  # data parallel: the two buckets' all-reduces (RCCL), A's issued first
            work = self._allreduce_start()
            self._mark_flushed()
            self._allreduce_finish(work)

    def allreduce_times(self):
        """Mean per-step times (ms) on the compute stream since construction or ``reset_allreduce_times`` (GPU with a
        process group; None otherwise or before any step): ``flush_ms`` from bucket A's all-reduce issue (the backward
        done) to bucket B's weight gradients done — the work A's communication overlaps; ``wait_ms`` from there to
        both buckets averaged — bucket B's all-reduce and whatever of A's did not hide under the flush: the exposed
        communication; ``window_ms`` the sum.  Read from the device clock gmz_comm_stamp keeps (one host sync)."""
        if self._comm_clock is None:
            return None
        t0, t1, flush, wait, n = self._comm_clock.tolist()
        if n == 0:
            return None
        flush, wait = flush / n / 1e5, wait / n / 1e5  # 100 MHz ticks -> ms
        return {"flush_ms": flush, "wait_ms": wait, "window_ms": flush + wait, "steps": n}

    def reset_allreduce_times(self):
        if self._comm_clock is not None:
            self._comm_clock.zero_()

    def allreduce_ms(self):
        """The exposed communication per step (``allreduce_times()['wait_ms']``), None without a process group."""
        t = self.allreduce_times()
        return None if t is None else t["wait_ms"]

    def _fused_opt_ok(self):
        g = self.opt.param_groups[0]
        return (FUSED_OPT and self.device.type == "cuda" and len(self.opt.param_groups) == 1
                and torch.is_tensor(g["lr"]) and not g.get("amsgrad") and not g.get("maximize")
                and all(p.dtype == torch.float32 for p in self.params))

    def _fused_opt_setup(self):
        """gmz_opt_step's work items over the gradient bucket, the Adam moments as bucket-shaped buffers (torch's
        optimiser state becomes views of them, so state_dict / load_state_dict keep the reference's format) and the
        target twins (a parameter whose twin has other strides gets its soft update from PyTorch)."""
        import ctypes
        from . import _lib
        L = _lib.load()
        ib, ch, wsb = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_size_t()
        _lib.check(L.gmz_opt_layout(ctypes.byref(ib), ctypes.byref(ch), ctypes.byref(wsb)))
        dt = np.dtype([("p", "<u8"), ("t", "<u8"), ("off", "<i8"), ("n", "<i4"), ("pi", "<i4")])
        if ib.value != dt.itemsize:
            raise _lib.GmzError("gmz_opt_layout: item of %d bytes, expected %d" % (ib.value, dt.itemsize))
        twin = {id(p): t for t, p in zip(self.target.parameters(), self.model.parameters())}
        m, v = torch.zeros_like(self.flat_grad), torch.zeros_like(self.flat_grad)
        step = torch.zeros((), dtype=torch.float32, device=self.device)
        base, items, fallback = self.flat_grad.data_ptr(), [], []
        for p in self.params:
            n = p.numel()
            off = (p.grad.data_ptr() - base) // 4
            dense = p.is_contiguous() or p.is_contiguous(memory_format=torch.channels_last)
            if not (dense and p.grad.stride() == p.stride() and 0 <= off and off + n <= self.flat_grad.numel()):
                raise RuntimeError("Trainer: a parameter's gradient is not its bucket range in its own layout")
            t = twin.get(id(p))
            t_ok = t is not None and t.is_cuda and t.dtype == torch.float32 and t.stride() == p.stride()
            if t is not None and not t_ok:
                fallback.append((t, p))
            for i0 in range(0, n, ch.value):
                items.append((p.data_ptr(), t.data_ptr() if t_ok else 0, off + i0, min(ch.value, n - i0), i0))
            mv = m[off:off + n].as_strided(p.shape, p.stride())
            vv = v[off:off + n].as_strided(p.shape, p.stride())
            st = self.opt.state.get(p)
            if st:  # resumed or earlier PyTorch steps: the moments and the step carry over
                mv.copy_(st["exp_avg"])
                vv.copy_(st["exp_avg_sq"])
                step.copy_(torch.as_tensor(st["step"], dtype=torch.float32))
            self.opt.state[p] = {"step": step, "exp_avg": mv, "exp_avg_sq": vv}
        arr = np.array(items, dtype=dt)
        versioned = list(self.params) + [twin[id(p)] for p in self.params if id(p) in twin]
        self._fopt = {"items": torch.from_numpy(arr.view(np.uint8)).to(self.device), "n_items": len(items),
                      "m": m, "v": v, "step": step, "coef": torch.zeros(2, dtype=torch.float32, device=self.device),
                      "ws": torch.zeros((wsb.value + 7) // 8, dtype=torch.float64, device=self.device),
                      "fallback": fallback, "versioned": versioned}

    def _update(self):
        c = self.cfg
        if self._fused_opt_ok():  # FUSED_OPT: unscale + clip + Adam + soft update + zero_grad in three launches
            from . import _lib
            if self._fopt is None:
                self._fused_opt_setup()
            f, g = self._fopt, self.opt.param_groups[0]
            amp = self.scaler.is_enabled()
            scale = self.scaler._scale if amp else None
            b1, b2 = g["betas"]
            _lib.check(_lib.load().gmz_opt_step(
                _lib.ptr(f["items"]), f["n_items"], _lib.ptr(self.flat_grad), _lib.ptr(f["m"]), _lib.ptr(f["v"]),
                self.flat_grad.numel(), _lib.ptr(scale), int(amp), float(c.GRAD_CLIP_NORM), _lib.ptr(g["lr"]),
                float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), float(c.TARGET_MODEL_TAU),
                _lib.ptr(f["step"]), _lib.ptr(f["coef"]), _lib.ptr(f["ws"]), _lib.nbytes(f["ws"]), _lib.stream_ptr()))
            if amp:  # GradScaler.update with the step's found_inf
                torch._amp_update_scale_(self.scaler._scale, self.scaler._growth_tracker, f["coef"][:1],
                                         self.scaler._growth_factor, self.scaler._backoff_factor,
                                         self.scaler._growth_interval)
            # the kernel wrote the parameters through raw pointers: advance their version counters as PyTorch's
            # in-place update would, so the packed-weight caches keyed on them (_packed_conv_weight, _bigk_weight)
            # re-pack — and a graph capture after this step records the packs
            from torch.autograd.graph import increment_version
            increment_version(f["versioned"])
            self.opt._opt_called = True  # what Optimizer.step records for the LR scheduler's call-order check
            if f["fallback"]:
                with torch.no_grad():
                    tp, sp = [t for t, _ in f["fallback"]], [p for _, p in f["fallback"]]
                    torch._foreach_mul_(tp, 1.0 - c.TARGET_MODEL_TAU)
                    torch._foreach_add_(tp, sp, alpha=c.TARGET_MODEL_TAU)
            return
        if self._fopt is not None:  # back on PyTorch's optimiser after fused steps: one step tensor per parameter again
            for p in self.params:
                st = self.opt.state[p]
                st["step"] = st["step"].clone()
            self._fopt = None
        self.scaler.unscale_(self.opt)
        torch.nn.utils.clip_grad_norm_(self.params, c.GRAD_CLIP_NORM, foreach=self.device.type == "cuda")
        self.scaler.step(self.opt)
        self.scaler.update()
        self.flat_grad.zero_()
        with torch.no_grad():  # utils.py:28-31 soft update (parameters only): tau * s + (1 - tau) * t
            pairs = list(zip(self.target.parameters(), self.model.parameters()))
            for same in (True, False):  # fused foreach kernels need equal strides (NCHW target, NHWC model)
                tp = [t for t, p in pairs if (t.stride() == p.stride()) == same]
                sp = [p for t, p in pairs if (t.stride() == p.stride()) == same]
                if tp:
                    torch._foreach_mul_(tp, 1.0 - c.TARGET_MODEL_TAU)
                    torch._foreach_add_(tp, sp, alpha=c.TARGET_MODEL_TAU)

    def _augment_into_static(self, batch, is_weights, k, flip):
        obs, act, rew, pi, mval = batch
        if k is None:
            k = np.random.randint(4)
        if flip is None:
            flip = bool(np.random.choice([True, False]))
        o, p, a = augment(obs, pi, act.long(), k, flip)
        src = (o, act.long(), rew.float(), p, mval.float(), a, is_weights.float())
        if self._static is None:
            self._static = tuple(torch.empty_like(t).contiguous() for t in src)
        for dst, t in zip(self._static, src):
            dst.copy_(t)

    def _capture(self):
        """The whole step as ONE HIP graph.  Data parallel (workers.py:571-580): the graph holds
        the RCCL all-reduces too — bucket A's issued on the process group's stream right after the backward (a fork
        in the graph), bucket B's weight gradients computed beside it on the capture stream, then B's all-reduce,
        the join, the average and the update — so no host call sits between the backward and the update.  If any
        rank cannot capture a collective (``_graph_collectives_ok``), every rank falls back to three graphs with the
        all-reduces issued eagerly between their replays (the round-5 form)."""
        st = self._static
        # with a process group, RCCL's watchdog thread queries its work events at any time; in the default global
        # capture mode such a query from another thread during the capture fails the process ("operation not
        # permitted when stream is capturing"), so the capture only restricts this thread
        import torch.distributed as tdist
        pg = self.dist is not None or (tdist.is_available() and tdist.is_initialized())
        mode = "thread_local" if pg else "global"
        dp = self.dist is not None
        in_graph = dp and GRAPH_ALLREDUCE and self._graph_collectives_ok(mode)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                self._out = self._forward_backward(st[:6], st[6], augmented=True, flush=not dp)
                if in_graph:  # bucket A's all-reduce beside bucket B's weight gradients, inside the graph
                    work = self._allreduce_start()
                    self._flush()
                    self._mark_flushed()
                    self._allreduce_finish(work)
                if not dp or in_graph:
                    self._update()
            if dp and not in_graph:  # bucket B's weight gradients and the update as graphs of their own
                gf, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gf, stream=s, pool=g.pool(), capture_error_mode=mode):
                    self._flush()
                with torch.cuda.graph(g2, stream=s, pool=g.pool(), capture_error_mode=mode):
                    self._update()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self._graphs = (g, gf, g2) if (dp and not in_graph) else g
        self.graph_allreduce = in_graph

    def _graph_collectives_ok(self, mode):
        """Whether every rank can capture an RCCL all-reduce into a HIP graph and replay it correctly: each rank
        captures a small one, the ranks agree (an eager MIN all-reduce) BEFORE any replays it — a rank replaying a
        collective its peers never captured would wait forever — then replay and check the sum, and agree again."""
        dist = self.dist
        if dist.get_backend() != "nccl":  # gloo stages device tensors through the host: never capturable (all ranks)
            return False
        n, r = dist.get_world_size(), dist.get_rank()
        t = torch.full((64,), float(r + 1), device=self.device)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        ok = 1
        try:
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                    dist.all_reduce(t)
        except Exception:  # noqa: BLE001 - any capture failure means: not in the graph
            ok = 0
        torch.cuda.current_stream(self.device).wait_stream(s)
        flag = torch.tensor([ok], dtype=torch.int32, device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            return False
        t.fill_(float(r + 1))
        g.replay()
        flag.fill_(int(bool((t == n * (n + 1) / 2).all())))
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    def step(self, batch, is_weights, k=None, flip=None, sync=True):
        """One training step -> ((total, policy, value, reward, consistency) floats, td errors [B]).
        ``sync=False``: the five losses stay a device tensor [5] (no host synchronisation, so the host
        can prepare the next step while this one runs; read them with ``.tolist()`` later)."""
        c = self.cfg
        acc = max(1, c.GRADIENT_ACCUMULATION_STEPS)
        if self.graph and self.step_count >= self.graph_warmup:
            self._augment_into_static(batch, is_weights, k, flip)
            if self._graphs is None:
                if BATCH_REPACK:  # the job table the captured step will replay, built before the capture
                    _repack_stale(list(self.model.parameters()) + list(self.target.parameters()), self._pack_tables,
                                  prepare=True)
                self._capture()
            if isinstance(self._graphs, tuple):  # collectives not capturable: the all-reduces between replays
                g1, gf, g2 = self._graphs
                g1.replay()
                work = self._allreduce_start()
                gf.replay()
                self._mark_flushed()
                self._allreduce_finish(work)
                g2.replay()
            else:
                self._graphs.replay()
            logs, td = self._out
            td = td.clone()
            self.sched.step()
        else:
            last = (self.step_count + 1) % acc == 0
            overlap = self.dist is not None and last
            logs, td = self._forward_backward(batch, is_weights, acc, k=k, flip=flip, flush=not overlap)
            if overlap:  # bucket A's all-reduce beside bucket B's weight gradients
                work = self._allreduce_start()
                self._flush()
                self._mark_flushed()
                self._allreduce_finish(work)
            if last:
                self._update()
                self.sched.step()
        self.step_count += 1
        if not sync:
            return logs.detach().clone(), td
        return tuple(float(x) for x in logs.tolist()), td

    def load_trainer_state(self, state):
        """Resume from the reference's trainer checkpoint (workers.py:469-475; the dict
        formats.RecordStore.load_trainer_state decodes): model, optimiser moments and step counts,
        scheduler position, train_step_count.  The target network restarts as a copy of the model
        (workers.py:491).  Execution flags stay this trainer's (fused, capturable, device lr)."""
        self.model.load_state_dict(state["model_state_dict"])
        self.target.load_state_dict(self.model.state_dict())
        self.opt.load_state_dict(state["optimizer_state_dict"])
        cuda = self.device.type == "cuda"
        for g in self.opt.param_groups:
            lr = float(g["lr"])
            g["lr"] = torch.tensor(lr, device=self.device) if cuda else lr
            g["fused"], g["capturable"], g["foreach"] = (True, True, None) if cuda else (None, False, None)
        for st in self.opt.state.values():
            if "step" in st:
                st["step"] = torch.as_tensor(float(st["step"]), dtype=torch.float32,
                                             device=self.device if cuda else "cpu")
        self.sched.load_state_dict(state["scheduler_state_dict"])
        self.step_count = int(state.get("train_step_count", 0))
        self.games_completed = int(state.get("games_completed_count", 0))
        self._graphs, self._static = None, None  # re-captured on the next step
        self._fopt = None  # FUSED_OPT adopts the loaded moments and step at the next update

    def trainer_state(self, games_completed_count=None):
        """The reference's checkpoint dict (workers.py:594-597), CPU tensors, optimiser state in the
        reference's form (float lr, CPU step counts, no fused/capturable flags) so either side can
        resume from it; store with formats.RecordStore.save_trainer_state."""
        opt = self.opt.state_dict()
        opt = {"state": {i: {k: (v.detach().cpu().reshape(()) if k == "step" else v.detach().cpu())
                             for k, v in st.items()} for i, st in opt["state"].items()},
               "param_groups": [dict(g, lr=float(g["lr"]), fused=None, capturable=False, foreach=None)
                                for g in opt["param_groups"]]}
        sch = self.sched.state_dict()
        return {"model_state_dict": self.state_dict_cpu(), "optimizer_state_dict": opt, "scheduler_state_dict": sch,
                "train_step_count": self.step_count,
                "games_completed_count": getattr(self, "games_completed", 0) if games_completed_count is None
                else int(games_completed_count)}

    def state_dict_cpu(self):
        """ModelWeightsUpdate payload (workers.py:587-593) for the self-play engines."""
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
