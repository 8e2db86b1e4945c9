"""Float32 numpy restatement of GomokuNetEZ inference (TEST INFRASTRUCTURE / oracle).

ORACLE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker for the HIP network (csrc/gmz_net.hip).  Restates /root/reference/network.py:
  support_to_scalar      network.py:9-13
  EvarResBlock           network.py:30-47   (eval-mode BatchNorm, eps 1e-4)
  RepresentationNetwork  network.py:49-56
  PredictionNetwork      network.py:58-74
  DynamicsNetwork        network.py:76-96   (one-hot action plane -> 1x1 embed -> concat -> conv)
  initial_inference      network.py:137-143
  recurrent_inference    network.py:145-152
Parity: PINNED against tests/golden/net_small.npz and net_c15.npz (reference forward on the same
numpy-seeded weights, tests/test_netref.py).
"""
import numpy as np

EPS = 1e-4


def _conv(x, w, b=None, pad=1):
    """NCHW conv, stride 1, zero padding; im2col + matmul in float32."""
    B, C, H, W = x.shape
    O, _, kh, kw = w.shape
    if pad:
        xp = np.zeros((B, C, H + 2 * pad, W + 2 * pad), np.float32)
        xp[:, :, pad:pad + H, pad:pad + W] = x
    else:
        xp = x
    cols = np.empty((B, C, kh, kw, H, W), np.float32)
    for dy in range(kh):
        for dx in range(kw):
            cols[:, :, dy, dx] = xp[:, :, dy:dy + H, dx:dx + W]
    cols = cols.reshape(B, C * kh * kw, H * W)
    out = np.einsum("ok,bkp->bop", w.reshape(O, -1).astype(np.float32), cols, optimize=True)
    if b is not None:
        out += b.reshape(1, O, 1)
    return out.reshape(B, O, H, W).astype(np.float32)


def _bn(x, sd, p):
    g, b, m, v = (sd[p + k] for k in (".weight", ".bias", ".running_mean", ".running_var"))
    s = (g / np.sqrt(v + EPS)).astype(np.float32)
    return (x - m.reshape(1, -1, 1, 1)) * s.reshape(1, -1, 1, 1) + b.reshape(1, -1, 1, 1)


def _relu(x):
    return np.maximum(x, 0, dtype=np.float32)


def _tower(x, sd, prefix, blocks):
    for i in range(blocks):
        p = "%s.resblocks.%d." % (prefix, i)
        y = _relu(_bn(_conv(x, sd[p + "conv1.weight"]), sd, p + "bn1"))
        y = _bn(_conv(y, sd[p + "conv2.weight"]), sd, p + "bn2")
        x = _relu(y + x)
    return x


def _softmax(z):
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


def support_to_scalar(logits, lo=-1, hi=1, bins=3):
    support = np.linspace(lo, hi, bins, dtype=np.float32)
    return (support * _softmax(logits.astype(np.float32))).sum(axis=1, keepdims=True).astype(np.float32)


def _num_blocks(sd, prefix):
    return len({k.split(".")[2] for k in sd if k.startswith(prefix + ".resblocks.")})


def representation(sd, obs):
    x = _relu(_bn(_conv(obs.astype(np.float32), sd["representation_net.conv.weight"]), sd, "representation_net.bn"))
    return _tower(x, sd, "representation_net", _num_blocks(sd, "representation_net"))


def prediction(sd, h):
    B = h.shape[0]
    p = _relu(_bn(_conv(h, sd["prediction_net.policy_conv.weight"], sd["prediction_net.policy_conv.bias"], pad=0),
                  sd, "prediction_net.policy_bn")).reshape(B, -1)
    logits = p @ sd["prediction_net.policy_fc.weight"].T + sd["prediction_net.policy_fc.bias"]
    v = _relu(_bn(_conv(h, sd["prediction_net.value_conv.weight"], sd["prediction_net.value_conv.bias"], pad=0),
                  sd, "prediction_net.value_bn")).reshape(B, -1)
    v = _relu(v @ sd["prediction_net.value_fc1.weight"].T + sd["prediction_net.value_fc1.bias"])
    vl = v @ sd["prediction_net.value_fc2.weight"].T + sd["prediction_net.value_fc2.bias"]
    return logits.astype(np.float32), vl.astype(np.float32)


def dynamics(sd, h, action):
    B, C, H, W = h.shape
    plane = np.zeros((B, 1, H, W), np.float32)
    plane.reshape(B, -1)[np.arange(B), np.asarray(action, np.int64)] = 1.0
    emb = _conv(plane, sd["dynamics_net.action_embed_conv.weight"], pad=0)
    x = np.concatenate([h, emb], axis=1)
    x = _relu(_bn(_conv(x, sd["dynamics_net.conv.weight"]), sd, "dynamics_net.bn"))
    nxt = _tower(x, sd, "dynamics_net", _num_blocks(sd, "dynamics_net"))
    r = _relu(nxt.reshape(B, -1) @ sd["dynamics_net.reward_fc.0.weight"].T + sd["dynamics_net.reward_fc.0.bias"])
    rl = r @ sd["dynamics_net.reward_fc.2.weight"].T + sd["dynamics_net.reward_fc.2.bias"]
    return nxt, rl.astype(np.float32)


def initial_inference(sd, obs):
    h = representation(sd, obs)
    logits, vl = prediction(sd, h)
    return logits, support_to_scalar(vl), h


def recurrent_inference(sd, h, action):
    nxt, rl = dynamics(sd, h, action)
    logits, vl = prediction(sd, nxt)
    return logits, support_to_scalar(vl), nxt, support_to_scalar(rl)
