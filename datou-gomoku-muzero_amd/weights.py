"""GomokuNetEZ weights: reference ``state_dict`` key layout and a portable seeded generator.

Key names and shapes follow /root/reference/network.py:27-135 exactly, so a reference checkpoint
(``ModelWeightsUpdate.weights``, ipc_messages.py:74-82) loads unchanged and a synthetic dict made
here loads into the reference ``GomokuNetEZ`` with ``load_state_dict``.

The synthetic generator uses ``numpy.random.RandomState`` (portable across torch versions,
SURVEY.md §7.1).  Deliberately NOT the reference init (network.py:125-126 zeroes every ResBlock
``bn2.weight``, which makes every residual branch vanish): bn2 gets a small non-zero gamma so
every conv is exercised, and BN running statistics are non-trivial so BN folding is tested.
"""
from collections import OrderedDict

import numpy as np


def _bn(prefix, c):
    return [(prefix + ".weight", (c,)), (prefix + ".bias", (c,)), (prefix + ".running_mean", (c,)),
            (prefix + ".running_var", (c,)), (prefix + ".num_batches_tracked", ())]


def reference_param_shapes(cfg, with_projection=True):
    """Ordered (key, shape) list of GomokuNetEZ(cfg).state_dict() (network.py:109-123)."""
    C, H = cfg.NUM_FILTERS, cfg.BOARD_SIZE
    A, hd, B = H * H, cfg.HEAD_HIDDEN_DIM, cfg.NUM_RES_BLOCKS
    out = [("representation_net.conv.weight", (C, 3, 3, 3))]
    out += _bn("representation_net.bn", C)
    for i in range(B):
        p = "representation_net.resblocks.%d." % i
        out += [(p + "conv1.weight", (C, C, 3, 3))] + _bn(p + "bn1", C)
        out += [(p + "conv2.weight", (C, C, 3, 3))] + _bn(p + "bn2", C)
    out += [("prediction_net.policy_conv.weight", (2, C, 1, 1)), ("prediction_net.policy_conv.bias", (2,))]
    out += _bn("prediction_net.policy_bn", 2)
    out += [("prediction_net.policy_fc.weight", (A, 2 * A)), ("prediction_net.policy_fc.bias", (A,))]
    out += [("prediction_net.value_conv.weight", (1, C, 1, 1)), ("prediction_net.value_conv.bias", (1,))]
    out += _bn("prediction_net.value_bn", 1)
    out += [("prediction_net.value_fc1.weight", (hd, A)), ("prediction_net.value_fc1.bias", (hd,)),
            ("prediction_net.value_fc2.weight", (cfg.VALUE_SUPPORT_BINS, hd)),
            ("prediction_net.value_fc2.bias", (cfg.VALUE_SUPPORT_BINS,))]
    out += [("dynamics_net.action_embed_conv.weight", (16, 1, 1, 1)),
            ("dynamics_net.conv.weight", (C, C + 16, 3, 3))]
    out += _bn("dynamics_net.bn", C)
    for i in range(B):  # network.py:83 reads the *global* config.NUM_RES_BLOCKS; callers keep them equal
        p = "dynamics_net.resblocks.%d." % i
        out += [(p + "conv1.weight", (C, C, 3, 3))] + _bn(p + "bn1", C)
        out += [(p + "conv2.weight", (C, C, 3, 3))] + _bn(p + "bn2", C)
    out += [("dynamics_net.reward_fc.0.weight", (hd, C * A)), ("dynamics_net.reward_fc.0.bias", (hd,)),
            ("dynamics_net.reward_fc.2.weight", (cfg.REWARD_SUPPORT_BINS, hd)),
            ("dynamics_net.reward_fc.2.bias", (cfg.REWARD_SUPPORT_BINS,))]
    if with_projection:
        out += [("projection_net.fc1.weight", (512, C * A)), ("projection_net.fc1.bias", (512,))]
        out += _bn("projection_net.bn1", 512)
        out += [("projection_net.fc2.weight", (512, 512)), ("projection_net.fc2.bias", (512,))]
    return out


def synthetic_state_dict(cfg, seed=0, with_projection=True):
    """Numpy-seeded synthetic weights (float32 numpy arrays; num_batches_tracked int64 scalars).

    Convs: He-normal (std sqrt(2/fan_in)); Linear: U(+-1/sqrt(fan_in)) (torch's default bound);
    BN: gamma ~ U(0.8, 1.2) (bn2 of every ResBlock ~ U(0.15, 0.35) to keep the residual stream
    bounded over 8-16 blocks), beta ~ N(0, 0.05), running_mean ~ N(0, 0.05), running_var ~ U(0.7, 1.3).
    """
    rs = np.random.RandomState(seed)
    sd = OrderedDict()
    for key, shape in reference_param_shapes(cfg, with_projection):
        leaf = key.rsplit(".", 1)[-1]
        if leaf == "num_batches_tracked":
            sd[key] = np.array(0, dtype=np.int64)
            continue
        is_bn = any(t in key for t in ("bn.", "bn1.", "bn2.", "_bn."))
        if is_bn:
            n = shape[0]
            if leaf == "weight":
                lo, hi = (0.15, 0.35) if ".bn2." in key else (0.8, 1.2)
                v = rs.uniform(lo, hi, n)
            elif leaf == "bias":
                v = rs.normal(0.0, 0.05, n)
            elif leaf == "running_mean":
                v = rs.normal(0.0, 0.05, n)
            else:
                v = rs.uniform(0.7, 1.3, n)
        elif len(shape) == 4:  # conv weight
            fan_in = shape[1] * shape[2] * shape[3]
            v = rs.normal(0.0, np.sqrt(2.0 / fan_in), shape)
        elif len(shape) == 2:  # linear weight
            bound = 1.0 / np.sqrt(shape[1])
            v = rs.uniform(-bound, bound, shape)
        else:  # 1-D bias of a conv or linear layer
            fan_in = _fan_in_of_bias(key, sd)
            bound = 1.0 / np.sqrt(fan_in)
            v = rs.uniform(-bound, bound, shape)
        sd[key] = np.asarray(v, dtype=np.float32)
    return sd


def _fan_in_of_bias(key, sd):
    w = sd[key[: -len("bias")] + "weight"]
    return int(np.prod(w.shape[1:]))


def to_torch(sd):
    import torch
    return OrderedDict((k, torch.from_numpy(np.array(v))) for k, v in sd.items())


def from_torch(sd):
    """Accept a torch state_dict (e.g. ModelWeightsUpdate.weights) → numpy float32 dict."""
    out = OrderedDict()
    for k, v in sd.items():
        a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
        out[k] = a if a.dtype == np.int64 else a.astype(np.float32)
    return out


def synthetic_slices(n, size, unroll, rs):
    """n TrainingSlice-shaped arrays (replay_buffer.py payload) of random content: sparse 0/1 planes,
    actions with a random game end (-1 after it), rewards in {-1,0,1}, normalised random policies,
    values in [-1, 1]."""
    A = size * size
    obs = (rs.rand(n, unroll + 1, 3, size, size) < 0.2).astype(np.uint8)
    act = rs.randint(0, A, (n, unroll)).astype(np.int32)
    ends = rs.randint(1, unroll + 1, n)
    act[np.arange(unroll)[None, :] >= ends[:, None]] = -1
    rew = rs.choice(np.array([-1.0, 0.0, 1.0], np.float32), (n, unroll))
    pol = rs.exponential(1.0, (n, unroll + 1, A)).astype(np.float32)
    pol /= pol.sum(-1, keepdims=True)
    val = rs.uniform(-1, 1, (n, unroll + 1)).astype(np.float32)
    return obs, act, rew, pol, val
