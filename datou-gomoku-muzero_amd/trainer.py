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
The convolutions run in PyTorch's kernels in this round; the fused HIP kernels cover inference.
"""
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
    """network.py:15-25: two-hot projection of a clamped scalar onto the support grid."""
    x = x.clamp(vmin, vmax)
    pos = (x - vmin) * ((bins - 1) / (vmax - vmin))
    lo, hi = torch.floor(pos).long(), torch.ceil(pos).long()
    w_hi = pos - lo.float()
    out = torch.zeros(x.shape[0], bins, device=x.device)
    out.scatter_add_(1, lo[:, None], (1 - w_hi)[:, None])
    out.scatter_add_(1, hi[:, None], w_hi[:, None])
    return out


# ------------------------------------------------------------------------------ network
def _conv3(cin, cout):
    return nn.Conv2d(cin, cout, 3, padding=1, bias=False)


def _bn(mod, x, mask=None):
    """BatchNorm whose training-mode statistics (and running-stat update) cover only the rows
    where ``mask`` is set.  The reference runs the unrolled steps on the sub-batch of games still
    in progress (loss.py:89-93); running every step on the FULL batch with row-masked statistics
    gives the same values and gradients with fixed shapes, so MIOpen compiles each convolution
    once instead of once per sub-batch size.  Computed in float32 (as autocast runs BatchNorm)."""
    if mask is None or not mod.training:
        return mod(x)
    x = x.float()
    dims = [0] + list(range(2, x.dim()))
    shape = [1, -1] + [1] * (x.dim() - 2)
    var, mean = torch.var_mean(x[mask], dim=dims, correction=0)  # statistics of the valid rows
    n = mask.sum().to(torch.float32) * (x[0, 0].numel())
    scale = torch.rsqrt(var + mod.eps) * mod.weight
    y = torch.addcmul((mod.bias - mean * scale).reshape(shape), x, scale.reshape(shape))  # one pass
    with torch.no_grad():  # through .data, like the native kernel: no autograd version bump (the
        m = mod.momentum      # unmasked BatchNorm calls of the same module saved these buffers)
        mod.running_mean.data.mul_(1 - m).add_(m * mean.detach())
        mod.running_var.data.mul_(1 - m).add_(m * var.detach() * n / (n - 1))
        mod.num_batches_tracked.data += 1
    return y


def _conv1x1(conv, x):
    """1x1 convolution as a batched GEMM over positions (same parameters as ``conv``).  MIOpen
    has no tuned kernels for the 1- and 2-channel head convolutions and the 1->16 action embedding
    and falls back to naive direct convolutions (tens of ms per weight gradient); as a GEMM they
    take microseconds."""
    n, c, h, w = x.shape
    wt = conv.weight.reshape(conv.weight.shape[0], c)
    y = torch.matmul(wt.to(x.dtype) if not torch.is_autocast_enabled() else wt, x.reshape(n, c, h * w))
    if conv.bias is not None:
        y = y + conv.bias.reshape(1, -1, 1).to(y.dtype)
    return y.reshape(n, -1, h, w)


class _Block(nn.Module):
    """Residual block (conv-BN-ReLU-conv-BN + identity, ReLU), parameter names of network.py:30-48."""

    def __init__(self, c):
        super().__init__()
        self.conv1, self.bn1 = _conv3(c, c), nn.BatchNorm2d(c, eps=1e-4)
        self.conv2, self.bn2 = _conv3(c, c), nn.BatchNorm2d(c, eps=1e-4)

    def forward(self, x, mask=None):
        y = F.relu(_bn(self.bn1, self.conv1(x), mask))
        return F.relu(_bn(self.bn2, self.conv2(y), mask) + x)


class _Trunk(nn.Module):
    """conv3x3 + BN + ReLU followed by residual blocks (representation and dynamics trunks)."""

    def __init__(self, cin, c, blocks):
        super().__init__()
        self.conv, self.bn = _conv3(cin, c), nn.BatchNorm2d(c, eps=1e-4)
        self.resblocks = nn.Sequential(*[_Block(c) for _ in range(blocks)])

    def forward(self, x, mask=None):
        h = F.relu(_bn(self.bn, self.conv(x), mask))
        for blk in self.resblocks:
            h = blk(h, mask)
        return h


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
        pol = self.policy_fc(F.relu(_bn(self.policy_bn, _conv1x1(self.policy_conv, h), mask)).reshape(n, -1))
        v = F.relu(self.value_fc1(F.relu(_bn(self.value_bn, _conv1x1(self.value_conv, h), mask)).reshape(n, -1)))
        return pol, self.value_fc2(v)


class _Dynamics(_Trunk):
    EMB = 16  # network.py:81 action embedding planes

    def __init__(self, c, H, blocks, hd, rbins):
        super().__init__(c + self.EMB, c, blocks)
        self.action_embed_conv = nn.Conv2d(1, self.EMB, 1, bias=False)
        self.reward_fc = nn.Sequential(nn.Linear(c * H * H, hd), nn.ReLU(), nn.Linear(hd, rbins))

    def forward(self, h, a, mask=None):
        n, _, H, W = h.shape
        plane = F.one_hot(a, H * W).to(h.dtype).reshape(n, 1, H, W)
        nxt = super().forward(torch.cat((h, _conv1x1(self.action_embed_conv, plane).to(h.dtype)), dim=1), mask)
        return nxt, self.reward_fc(nxt.reshape(n, -1))


class _Projection(nn.Module):
    def __init__(self, din, hidden=512, out=512):
        super().__init__()
        self.fc1, self.bn1, self.fc2 = nn.Linear(din, hidden), nn.BatchNorm1d(hidden, eps=1e-4), nn.Linear(hidden, out)

    def forward(self, h, mask=None):
        return self.fc2(F.relu(_bn(self.bn1, self.fc1(h.reshape(h.shape[0], -1)), mask)))


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

    def representation(self, obs, mask=None):
        return self.representation_net(obs, mask)

    def prediction(self, h, mask=None):
        return self.prediction_net(h, mask)

    def dynamics(self, h, a, mask=None):
        return self.dynamics_net(h, a, mask)

    def project(self, h, with_grad=True, mask=None):
        if with_grad:
            return self.projection_net(h, mask)
        with torch.no_grad():
            return self.projection_net(h, mask)

    @torch.no_grad()
    def initial_value(self, obs):
        """initial_inference's value scalar (network.py:137-143), eval mode."""
        self.eval()
        _, vl = self.prediction(self.representation(obs))
        c = self.cfg
        return support_to_scalar(vl, c.VALUE_SUPPORT_MIN, c.VALUE_SUPPORT_MAX, c.VALUE_SUPPORT_BINS)


# ------------------------------------------------------------------------------ loss
def barlow_loss(z1, z2, lam):
    """loss.py:10-27: Barlow-twins cross-correlation loss of batch-standardised projections
    (BatchNorm1d without affine/running stats, eps 1e-5, written out so any row count runs the
    same elementwise kernels)."""
    z1, z2 = z1.float(), z2.float()
    n = z1.shape[0]

    def std(z):
        zc = z - z.mean(0, keepdim=True)
        return zc * torch.rsqrt((zc * zc).mean(0, keepdim=True) + 1e-5)

    c = (std(z1).t() @ std(z2)) / n
    diag = torch.diagonal(c)
    on = (diag - 1).pow(2).sum()
    off = c.pow(2).sum() - diag.pow(2).sum()
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
    out = torch.zeros_like(mcts_val)
    for i in range(U + 1):
        z = 0.0
        for j in range(n):
            if i + j >= U:
                break
            z = z + (g ** j) * rew[:, i + j]
        boot = mcts_val[:, i + n] if i + n <= U else last_value
        out[:, i] = z + (g ** n) * boot
    return out


def muzero_loss(model, target_model, batch, is_weights, cfg, k=None, flip=None, amp=False, amp_dtype=None):
    """loss.py:30-158.  ``batch`` = (obs [B,U+1,3,H,W], actions [B,U], rewards [B,U],
    policies [B,U+1,A], search values [B,U+1]).  ``k``/``flip``: the augmentation (default: drawn
    from numpy's global RandomState in the reference's order).  Returns (weighted loss tensor,
    (total, policy, value, reward, consistency) floats, |value error| at step 0 as a tensor)."""
    if k is None:
        k = np.random.randint(4)
    if flip is None:
        flip = bool(np.random.choice([True, False]))
    model.train()
    target_model.eval()
    obs, act, rew, pi, mval = batch
    act, rew, mval = act.long(), rew.float(), mval.float()
    obs, pi, act_aug = augment(obs, pi, act, k, flip)
    c, W = cfg, cfg.LOSS_WEIGHTS
    vsup = (c.VALUE_SUPPORT_MIN, c.VALUE_SUPPORT_MAX, c.VALUE_SUPPORT_BINS)
    rsup = (c.REWARD_SUPPORT_MIN, c.REWARD_SUPPORT_MAX, c.REWARD_SUPPORT_BINS)
    with torch.no_grad():
        last_v = target_model.initial_value(obs[:, -1])[:, 0]
        z = value_targets(rew, mval, last_v, c)
    dev_type = obs.device.type
    with torch.autocast(dev_type, enabled=amp and dev_type == "cuda", dtype=amp_dtype or torch.float16):
        h = model.representation(obs[:, 0])
        pl, vl = model.prediction(h)
        lp = F.cross_entropy(pl.float(), pi[:, 0], reduction="none")
        lv = F.cross_entropy(vl.float(), scalar_to_support(z[:, 0], *vsup), reduction="none")
        # loss.py:78 passes softmax(logits) to support_to_scalar, which applies softmax again:
        # the PER priority is computed from that doubly-softmaxed value (kept as the reference does)
        v0 = support_to_scalar(F.softmax(vl.float(), dim=1), *vsup)
        td = (v0.detach()[:, 0] - z[:, 0]).abs()
        lr_ = torch.zeros(obs.shape[0], device=obs.device)
        proj_pairs = []
        steps = 0
        for s in range(c.NUM_UNROLL_STEPS):
            m = act[:, s] != -1
            if not bool(m.any()):
                continue
            steps += 1
            mf = m.to(torch.float32)
            # full-batch step, row-masked BatchNorm statistics and losses (== the reference's
            # sub-batch h[m] computation, loss.py:89-107, with fixed shapes)
            hk, rl = model.dynamics(h, torch.where(m, act_aug[:, s], torch.zeros_like(act_aug[:, s])), mask=m)
            plk, vlk = model.prediction(hk, mask=m)
            lp = lp + mf * F.cross_entropy(plk.float(), pi[:, s + 1], reduction="none")
            lv = lv + mf * F.cross_entropy(vlk.float(), scalar_to_support(z[:, s + 1], *vsup), reduction="none")
            lr_ = lr_ + mf * F.cross_entropy(rl.float(), scalar_to_support(rew[:, s], *rsup), reduction="none")
            dyn = model.project(hk, with_grad=True, mask=m)
            with torch.no_grad():
                tru = model.project(model.representation(obs[:, s + 1], mask=m), with_grad=False, mask=m)
            proj_pairs.append((dyn[m], tru[m]))
            nh = torch.where(m[:, None, None, None], hk, h)
            nh.register_hook(lambda g: g * 0.5)
            h = nh
    lp = lp / (steps + 1)
    lv = lv / (steps + 1)
    lr_ = lr_ / steps if steps else torch.zeros_like(lr_)
    cons = (sum(barlow_loss(a, b, c.BARLOW_LAMBDA) for a, b in proj_pairs) / steps if steps
            else torch.zeros((), device=obs.device))
    fp, fv, fr = (lp * is_weights).mean(), (lv * is_weights).mean(), (lr_ * is_weights).mean()
    total = W["policy"] * fp + W["value"] * fv + W["reward"] * fr + W["consistency"] * cons
    logs = tuple(float(x.detach()) for x in (total, fp, fv, fr, cons))
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
        self.prio[idx.to(self.device)] = self.max_priority if self.cfg.ENABLE_PER else 1.0
        self.ptr = (self.ptr + n) % self.N
        self.count = min(self.N, self.count + n)

    def sample(self, B, rng=np.random):
        if self.count < B:
            return None
        if self.cfg.ENABLE_PER:
            p = self.prio[: self.count].double()
            cum = torch.cumsum(p, 0)
            total = float(cum[-1])
            seg = total / B
            u = torch.from_numpy(np.array([rng.uniform(seg * i, seg * (i + 1)) for i in range(B)])).to(self.device)
            idx = torch.searchsorted(cum, u).clamp_max(self.count - 1)
            w = (self.count * (p[idx] / total)) ** (-self.cfg.PER_BETA)
            w = (w / w.max()).float()
        else:
            idx = torch.from_numpy(rng.choice(self.count, B, replace=False)).to(self.device)
            w = torch.ones(B, device=self.device)
        batch = (self.obs[idx].float(), self.act[idx], self.rew[idx], self.pol[idx], self.val[idx])
        return batch, idx, w

    def update_priorities(self, idx, td):
        if not self.cfg.ENABLE_PER:
            return
        p = td.abs().to(self.device).float() + self.cfg.PER_EPSILON
        self.max_priority = max(self.max_priority, float(p.max()))
        self.prio[idx] = p


# ------------------------------------------------------------------------------ trainer
class Trainer:
    """training_worker's step (workers.py:452-463, 556-584) without the queues: Adam with weight
    decay, LinearLR warm-up (1000 updates) then cosine annealing to 1e-7 over 200k updates, AMP
    grad scaler, gradient clipping, soft target update after every optimiser step.  Under an
    initialised torch.distributed every rank trains on its own batch and the gradients are averaged
    with one all-reduce of a flat bucket (RCCL) before the update."""

    def __init__(self, cfg=None, device="cuda", state_dict=None, amp=None, amp_dtype=None, channels_last=False):
        c = cfg if isinstance(cfg, TrainConfig) else TrainConfig.from_any(cfg)
        self.cfg, self.device = c, torch.device(device)
        self.model = TrainNet(c).to(self.device)
        if state_dict is not None:
            self.model.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}, strict=False)
        self.target = TrainNet(c).to(self.device)
        self.target.load_state_dict(self.model.state_dict())
        self.amp = (self.device.type == "cuda") if amp is None else amp
        self.amp_dtype = amp_dtype  # None: float16 as the reference's torch.amp.autocast('cuda')
        self.channels_last = channels_last
        if channels_last:
            self.model = self.model.to(memory_format=torch.channels_last)
            self.target = self.target.to(memory_format=torch.channels_last)
        import torch.distributed as dist
        self.dist = dist if (dist.is_available() and dist.is_initialized()) else None
        if self.dist is not None:  # every rank starts from rank 0's weights
            for t in list(self.model.parameters()) + list(self.model.buffers()):
                self.dist.broadcast(t.data, 0)
            self.target.load_state_dict(self.model.state_dict())
        self.opt = torch.optim.Adam(self.model.parameters(), lr=c.LEARNING_RATE, weight_decay=c.WEIGHT_DECAY)
        acc = max(1, c.GRADIENT_ACCUMULATION_STEPS)
        warm, total = 1000 // acc, 200000 // acc
        self.sched = torch.optim.lr_scheduler.SequentialLR(self.opt, [
            torch.optim.lr_scheduler.LinearLR(self.opt, start_factor=0.01, total_iters=warm),
            torch.optim.lr_scheduler.CosineAnnealingLR(self.opt, T_max=total - warm, eta_min=1e-7)], milestones=[warm])
        self.scaler = torch.amp.GradScaler(self.device.type, enabled=self.amp and amp_dtype in (None, torch.float16))
        self.step_count = 0

    def step(self, batch, is_weights, k=None, flip=None):
        c = self.cfg
        acc = max(1, c.GRADIENT_ACCUMULATION_STEPS)
        if self.channels_last:
            batch = (batch[0].contiguous(memory_format=torch.channels_last) if batch[0].dim() == 4 else batch[0],) + tuple(batch[1:])
        loss, logs, td = muzero_loss(self.model, self.target, batch, is_weights, c, k=k, flip=flip, amp=self.amp,
                                     amp_dtype=self.amp_dtype)
        self.scaler.scale(loss / acc).backward()
        if self.dist is not None:  # data parallel: ONE all-reduce of a flat gradient bucket (RCCL)
            ps = [p for p in self.model.parameters() if p.grad is not None]
            flat = torch.cat([p.grad.reshape(-1) for p in ps])
            self.dist.all_reduce(flat)
            flat.div_(self.dist.get_world_size())
            off = 0
            for p in ps:
                n = p.grad.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        if (self.step_count + 1) % acc == 0:
            self.scaler.unscale_(self.opt)
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), c.GRAD_CLIP_NORM)
            self.scaler.step(self.opt)
            self.scaler.update()
            self.sched.step()
            self.opt.zero_grad(set_to_none=True)
            with torch.no_grad():  # utils.py:28-31 soft update (parameters only)
                for t, s in zip(self.target.parameters(), self.model.parameters()):
                    t.copy_(c.TARGET_MODEL_TAU * s + (1.0 - c.TARGET_MODEL_TAU) * t)
        self.step_count += 1
        return logs, td

    def state_dict_cpu(self):
        """ModelWeightsUpdate payload (workers.py:587-593) for the self-play engines."""
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}
