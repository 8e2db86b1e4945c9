"""GomokuNetEZ inference on MI355X: weight packing + the device backend used by the engine.

``pack_weights`` turns a reference ``state_dict`` (network.py:109-123 key names, e.g. the
``ModelWeightsUpdate.weights`` the trainer sends, workers.py:332-335) into the kernel layouts of
csrc/gmz_net.hip:
  * eval-mode BatchNorm (eps 1e-4, network.py:34,37,53,62,65,82) folded into conv weight/bias;
  * 3x3 conv weights as f16 (default) or bf16 in v_mfma_f32_16x16x32_{f16,bf16} A-operand fragment order
    [tap][k-step][n-tile][lane][8] (rows = output channels), so a 16 KB weight stage is a
    linear copy and every fragment read is one conflict-free ds_read_b128;
  * the dynamics action embedding (one-hot plane -> 1x1 conv, network.py:90-92) folded into a
    [9][C] per-tap additive term of the dynamics conv (exact algebra: the plane has one 1);
  * reward_fc.0 permuted from NCHW-flatten to the NHWC hidden-state order, B-fragment order.

``precision``: "fp16" (default; 10-bit mantissa, the type of the reference trainer's own autocast)
or "bf16" (7-bit mantissa) — the 16-bit type of the packed weights, the activations and the
hidden-state pool; MFMA accumulation is float32 either way and gfx950 runs both at the same rate.

``GomokuNetHip`` owns the 16-bit hidden-state slot pool (HBM) and launches the kernels through the
C ABI (include/gmz.h gmz_net_*).  It is the ``net`` backend of engine.BatchedSelfPlayEngine.
"""
import contextlib
import copy
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import P, I, SZ, check, ptr
from .config import from_any

EPS = 1e-4
C = 128


class NetWeights(ctypes.Structure):
    _fields_ = [("board_size", ctypes.c_int32), ("channels", ctypes.c_int32), ("blocks", ctypes.c_int32),
                ("head_hidden", ctypes.c_int32)] + [(n, ctypes.c_void_p) for n in (
                    "repr_stem_w", "repr_stem_b", "repr_convs", "repr_bias", "dyn_convs", "dyn_bias", "dyn_action",
                    "head_conv_w", "head_conv_b", "policy_fc_w", "policy_fc_b", "value_fc1_w", "value_fc1_b",
                    "value_fc2_w", "value_fc2_b", "reward_fc1_w", "reward_fc1_b", "reward_fc2_w", "reward_fc2_b")] + [
                    ("dtype", ctypes.c_int32), ("max_grid", ctypes.c_int32)]


PRECISIONS = {"fp16": 0, "bf16": 1}  # include/gmz.h GMZ_NET_F16 / GMZ_NET_BF16
_TORCH16 = {"fp16": torch.float16, "bf16": torch.bfloat16}


_lib.register({
    "gmz_net_workspace_bytes": ([ctypes.POINTER(NetWeights), I, ctypes.POINTER(ctypes.c_size_t)], I),
    "gmz_net_initial": ([ctypes.POINTER(NetWeights), P, I, P, P, P, P, P, SZ, P], I),
    "gmz_net_initial_tower": ([ctypes.POINTER(NetWeights), P, I, P, P, P, SZ, P], I),
    "gmz_net_initial_heads": ([ctypes.POINTER(NetWeights), P, P, I, P, P, P, SZ, P], I),
    "gmz_net_recurrent": ([ctypes.POINTER(NetWeights), P, P, P, P, I, P, P, P, P, SZ, P], I),
    "gmz_net_recurrent_tower": ([ctypes.POINTER(NetWeights), P, P, P, P, I, P, SZ, P], I),
    "gmz_net_recurrent_heads": ([ctypes.POINTER(NetWeights), P, P, I, P, P, P, P, SZ, P], I),
})


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def fold_bn(sd, prefix):
    g, b, m, v = (_f32(sd[prefix + k]) for k in (".weight", ".bias", ".running_mean", ".running_var"))
    s = g / np.sqrt(v + np.float32(EPS))
    return s.astype(np.float32), (b - m * s).astype(np.float32)


def _e16_bits(x, precision="fp16"):
    """float32 array -> uint16 bit patterns of the 16-bit type (round to nearest even; f16 saturates
    at +-65504 instead of overflowing to inf)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    if precision == "fp16":
        x = np.clip(x, -65504.0, 65504.0)
    t = torch.from_numpy(x).to(_TORCH16[precision])
    return t.view(torch.int16).numpy().view(np.uint16)


CHUNK_OF_GROUP = np.array([0, 8, 1, 9])  # lane group g of k-step s reads channel chunk 2s + CHUNK_OF_GROUP[g]


def conv_input_channel(ks, l, j):
    """Input channel fed to MFMA k-slot 8*(l>>4)+j of k-step ks (see the LDS layout note in gmz_net.hip)."""
    return (2 * ks + CHUNK_OF_GROUP[l >> 4]) * 8 + j


def output_channel(nt, m):
    """Output channel of MFMA row m (0..15) of n-tile nt in the tower kernels (k_tower3's chan0):
    n-tiles pair up so that a lane's accumulators of tiles 2u and 2u+1 are 8 consecutive channels,
    stored as one 16-byte chunk."""
    return (nt >> 1) * 32 + 8 * (m >> 2) + 4 * (nt & 1) + (m & 3)


def pack_conv3x3(wf, precision="fp16"):
    """[128(n), 128(c), 3, 3] f32 -> 16-bit [9][4][8][64][8]: frag(t, ks, nt, l, j) =
    W[n = output_channel(nt, l&15)][c = conv_input_channel(ks, l, j)][t // 3][t % 3]."""
    Wt = wf.transpose(2, 3, 0, 1).reshape(9, C, C)  # [t][n][c]
    ks, nt, l, j = np.meshgrid(np.arange(4), np.arange(8), np.arange(64), np.arange(8), indexing="ij")
    n = output_channel(nt, l & 15)
    c = conv_input_channel(ks, l, j)
    out = Wt[:, n, c]  # [9][4][8][64][8]
    return _e16_bits(out, precision)


def pack_stem(wf, precision="fp16"):
    """conv 3->128 [128, 3, 3, 3] -> 16-bit [8][64][8] with k = tap*3 + c (27, zero-padded to 32), rows
    in output_channel order."""
    Wk = np.zeros((C, 32), np.float32)
    for dy in range(3):
        for dx in range(3):
            for c in range(3):
                Wk[:, (dy * 3 + dx) * 3 + c] = wf[:, c, dy, dx]
    nt, l, j = np.meshgrid(np.arange(8), np.arange(64), np.arange(8), indexing="ij")
    return _e16_bits(Wk[output_channel(nt, l & 15), 8 * (l >> 4) + j], precision)


def r16(x):
    return (x + 15) // 16 * 16


def pad_fc(w, rows, cols):
    """torch Linear weight [out, in] -> f32 [rows][cols], zero padded (output-major, k contiguous:
    the f32-MFMA head GEMMs read one 16-float k-chunk per lane group)."""
    out = np.zeros((rows, cols), np.float32)
    out[:w.shape[0], :w.shape[1]] = w
    return out


def pack_reward_fc1(w, A, precision="fp16"):
    """reward_fc.0.weight [hd, C*A] (NCHW-flatten input) -> 16-bit B fragments [K/32][hd/16][64][8]
    over the NHWC hidden order k = p*C + c."""
    hd = w.shape[0]
    Wn = w.reshape(hd, C, A).transpose(2, 1, 0).reshape(A * C, hd)  # [k = p*C + c][n]
    kk, nt, l, j = np.meshgrid(np.arange(A * C // 32), np.arange(hd // 16), np.arange(64), np.arange(8), indexing="ij")
    return _e16_bits(Wn[kk * 32 + 8 * (l >> 4) + j, nt * 16 + (l & 15)], precision)


def pack_weights(sd, cfg, precision="fp16"):
    """Reference state_dict (numpy or torch tensors) -> dict of packed numpy arrays."""
    sd = {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)) for k, v in sd.items()}
    H = cfg.BOARD_SIZE
    A = H * H
    nb = cfg.NUM_RES_BLOCKS
    out = {}
    s, b = fold_bn(sd, "representation_net.bn")
    out["repr_stem_w"] = pack_stem(_f32(sd["representation_net.conv.weight"]) * s[:, None, None, None], precision)
    out["repr_stem_b"] = b

    def tower(prefix):
        convs, biases = [], []
        for i in range(nb):
            for k in (1, 2):
                p = "%s.resblocks.%d." % (prefix, i)
                s, b = fold_bn(sd, p + "bn%d" % k)
                convs.append(pack_conv3x3(_f32(sd[p + "conv%d.weight" % k]) * s[:, None, None, None], precision))
                biases.append(b)
        return convs, biases

    convs, biases = tower("representation_net")
    out["repr_convs"] = np.stack(convs)
    out["repr_bias"] = np.stack(biases)
    s, b = fold_bn(sd, "dynamics_net.bn")
    wd = _f32(sd["dynamics_net.conv.weight"]) * s[:, None, None, None]  # [C, C+16, 3, 3]
    emb = _f32(sd["dynamics_net.action_embed_conv.weight"]).reshape(16)
    act = np.einsum("ncyx,c->yxn", wd[:, C:], emb).reshape(9, C)
    convs, biases = tower("dynamics_net")
    out["dyn_convs"] = np.stack([pack_conv3x3(wd[:, :C], precision)] + convs)
    out["dyn_bias"] = np.stack([b] + biases)
    out["dyn_action"] = act.astype(np.float32)
    sp, bp = fold_bn(sd, "prediction_net.policy_bn")
    sv, bv = fold_bn(sd, "prediction_net.value_bn")
    hw = np.concatenate([_f32(sd["prediction_net.policy_conv.weight"]).reshape(2, C) * sp[:, None],
                         _f32(sd["prediction_net.value_conv.weight"]).reshape(1, C) * sv[:, None]])
    hb = np.concatenate([_f32(sd["prediction_net.policy_conv.bias"]) * sp + bp,
                         _f32(sd["prediction_net.value_conv.bias"]) * sv + bv])
    out["head_conv_w"], out["head_conv_b"] = hw.astype(np.float32), hb.astype(np.float32)
    out["policy_fc_w"] = pad_fc(_f32(sd["prediction_net.policy_fc.weight"]), r16(A), r16(2 * A))
    out["policy_fc_b"] = _f32(sd["prediction_net.policy_fc.bias"])
    out["value_fc1_w"] = pad_fc(_f32(sd["prediction_net.value_fc1.weight"]), 64, r16(A))
    out["value_fc1_b"] = _f32(sd["prediction_net.value_fc1.bias"])
    out["value_fc2_w"] = np.ascontiguousarray(_f32(sd["prediction_net.value_fc2.weight"]).T)
    out["value_fc2_b"] = _f32(sd["prediction_net.value_fc2.bias"])
    out["reward_fc1_w"] = pack_reward_fc1(_f32(sd["dynamics_net.reward_fc.0.weight"]), A, precision)
    out["reward_fc1_b"] = _f32(sd["dynamics_net.reward_fc.0.bias"])
    out["reward_fc2_w"] = np.ascontiguousarray(_f32(sd["dynamics_net.reward_fc.2.weight"]).T)
    out["reward_fc2_b"] = _f32(sd["dynamics_net.reward_fc.2.bias"])
    return out


class KernelTimer:
    """HIP-event pairs recorded on the launch stream around one kernel; read after a sync."""

    def __init__(self, stream=None):
        self.stream = stream if stream is not None else torch.cuda.current_stream()
        self.pairs = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        self.pairs.append([e, None, 0])

    def stop(self, units):
        e = torch.cuda.Event(enable_timing=True)
        e.record(self.stream)
        self.pairs[-1][1] = e
        self.pairs[-1][2] = units

    def reset(self):
        self.pairs = []

    def summary(self):
        """(launches, mean ms per launch, mean units per launch)."""
        if not self.pairs:
            return 0, 0.0, 0.0
        ms = [a.elapsed_time(b) for a, b, _ in self.pairs]
        return len(ms), sum(ms) / len(ms), sum(u for _, _, u in self.pairs) / len(ms)


class GomokuNetHip:
    """GomokuNetEZ initial/recurrent inference on the device (engine ``net`` backend).

    ``num_slots`` hidden-state slots of 16-bit [A][128] (``precision``: "fp16" default, or "bf16")
    live in ``self.pool`` (HBM); the engine addresses node u of game g as slot hbase[g] + u, the per-game
    bases packed by the legal-move count of each search (engine.BatchedSelfPlayEngine._place_hidden;
    ``engine.hidden_slots(cfg, G)`` is the steady-state size, the pool grows when a search needs more).
    """

    def __init__(self, state_dict, cfg=None, num_slots=1, max_rows=1, device="cuda", precision="fp16", **overrides):
        if precision not in PRECISIONS:
            raise ValueError("GomokuNetHip: precision must be 'fp16' or 'bf16'")
        self.precision = precision
        self.cfg = from_any(cfg, **overrides)
        c = self.cfg
        if c.NUM_FILTERS != C or c.HEAD_HIDDEN_DIM != 64 or c.BOARD_SIZE not in (6, 9, 15, 19):
            raise ValueError("GomokuNetHip: kernels support NUM_FILTERS=128, HEAD_HIDDEN_DIM=64, BOARD_SIZE 6/9/15/19")
        self.device = torch.device(device)
        self.A = c.ACTION_SPACE_SIZE
        self.lib = _lib.load()
        self.max_rows = int(max_rows)
        self.pool = torch.empty(int(num_slots) * self.A * C, dtype=torch.int16, device=self.device)
        self.workspace = None
        self.tower_timer = None  # optional KernelTimer around the dynamics tower launches (bench.py)
        self.repr_timer = None   # optional KernelTimer around the representation tower launches
        self.load_state_dict(state_dict)

    def load_state_dict(self, state_dict):
        """Hot-swap weights (ModelWeightsUpdate, workers.py:332-335)."""
        packed = pack_weights(state_dict, self.cfg, self.precision)
        self._tensors = {k: torch.from_numpy(np.ascontiguousarray(v)).to(self.device) for k, v in packed.items()}
        c = self.cfg
        w = NetWeights(c.BOARD_SIZE, C, c.NUM_RES_BLOCKS, c.HEAD_HIDDEN_DIM)
        w.dtype = PRECISIONS[self.precision]
        for k, t in self._tensors.items():
            setattr(w, k, t.data_ptr())
        self.w = w
        # the workspace (head scratch + the tower's scheduling counters, zero between launches) does not
        # depend on the weights: a hot swap keeps it, so no zero-fill is ever queued on another stream
        # behind launches that already use it
        if getattr(self, "workspace", None) is None:
            nbytes = ctypes.c_size_t()
            check(self.lib.gmz_net_workspace_bytes(ctypes.byref(w), self.max_rows, ctypes.byref(nbytes)))
            self.workspace = torch.zeros(nbytes.value, dtype=torch.uint8, device=self.device)
        for q in getattr(self, "_children", []):  # split() views follow the hot swap
            keep = q.w.max_grid
            q.w = NetWeights.from_buffer_copy(w)
            q.w.max_grid = keep
            q._tensors = self._tensors

    def ensure_slots(self, n, stream=None):
        """At least ``n`` hidden-state slots in ``self.pool`` (engine._place_hidden, between moves: the
        contents are not kept).  A split() view that outgrows its slice gets a pool of its own.  ``stream``:
        the (torch) stream whose launches use the pool (default: the current one); the old pool's memory is
        recorded on it, so the caching allocator reuses it only after that stream's queued launches, and no
        other stream (the other engine half, a concurrent trainer) is waited for."""
        per = self.A * C
        if n * per > self.pool.numel():
            self.pool.record_stream(stream if stream is not None else torch.cuda.current_stream(self.device))
            self.pool = torch.empty(int(n * 1.25 + 1) * per, dtype=torch.int16, device=self.device)

    def split(self, parts, max_grid=0):
        """``parts`` backends over disjoint, equal slices of this hidden-state pool that share the
        packed weights, each with its own workspace (engine.SplitSelfPlayEngine: one per HIP stream,
        so their launches may run concurrently).  ``max_grid`` caps their persistent tower grid."""
        n = self.pool.numel() // parts
        out = []
        for i in range(parts):
            q = copy.copy(self)
            q.pool = self.pool[i * n:(i + 1) * n]
            q.max_rows = max(1, self.max_rows // parts)
            q.w = NetWeights.from_buffer_copy(self.w)  # the same weight pointers
            q.w.max_grid = int(max_grid)
            nbytes = ctypes.c_size_t()
            check(self.lib.gmz_net_workspace_bytes(ctypes.byref(q.w), q.max_rows, ctypes.byref(nbytes)))
            q.workspace = torch.zeros(nbytes.value, dtype=torch.uint8, device=self.device)
            q.tower_timer = q.repr_timer = None
            q._children = []
            out.append(q)
        self._children = getattr(self, "_children", []) + out
        return out

    def _ws(self, rows, stream=None):
        if rows > self.max_rows:  # grow the scratch (k_heads / reward split-K partials)
            self.max_rows = rows
            nbytes = ctypes.c_size_t()
            check(self.lib.gmz_net_workspace_bytes(ctypes.byref(self.w), rows, ctypes.byref(nbytes)))
            # zero-filled on the launch stream, so the fill is ordered before this launch's tower reads
            # its ticket word (the caller's current stream may be another one)
            raw = stream.value if isinstance(stream, ctypes.c_void_p) else stream
            st = (torch.cuda.ExternalStream(raw, device=self.device) if raw else
                  torch.cuda.default_stream(self.device) if stream is not None else None)
            with torch.cuda.stream(st) if st is not None else contextlib.nullcontext():
                self.workspace = torch.zeros(nbytes.value, dtype=torch.uint8, device=self.device)
        return ptr(self.workspace)

    # ---- engine backend interface
    def initial(self, obs, out_slot, logits, value, stream):
        rows = obs.shape[0]
        ws = self._ws(rows, stream)
        t = self.repr_timer
        if t is not None:
            t.start()
        wsb = self.workspace.numel()
        check(self.lib.gmz_net_initial_tower(ctypes.byref(self.w), ptr(obs), rows, ptr(out_slot), ptr(self.pool), ws,
                                             wsb, stream))
        if t is not None:
            t.stop(rows)
        check(self.lib.gmz_net_initial_heads(ctypes.byref(self.w), ptr(self.pool), ptr(out_slot), rows, ptr(logits),
                                             ptr(value), ws, wsb, stream))

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        rows = in_slot.shape[0]
        ws = self._ws(rows, stream)
        t = self.tower_timer
        if t is not None:
            t.start()
        wsb = self.workspace.numel()
        check(self.lib.gmz_net_recurrent_tower(ctypes.byref(self.w), ptr(self.pool), ptr(in_slot), ptr(action),
                                               ptr(out_slot), rows, ws, wsb, stream))
        if t is not None:
            t.stop(rows)
        check(self.lib.gmz_net_recurrent_heads(ctypes.byref(self.w), ptr(self.pool), ptr(out_slot), rows,
                                               ptr(logits), ptr(value), ptr(reward), ws, wsb, stream))

    # ---- convenience (tests / single-game adapters): slots 0..rows-1 are used as scratch
    def hidden(self, slots):
        """The hidden states of the given slots as float32 [n, C, H, W] (NCHW, like the reference)."""
        H = self.cfg.BOARD_SIZE
        idx = torch.as_tensor(np.asarray(slots, dtype=np.int64), device=self.device)
        hv = self.pool.view(-1, self.A, C)[idx]  # [n][A][C] 16-bit patterns
        f = hv.view(_TORCH16[self.precision]).float()
        return f.permute(0, 2, 1).reshape(len(slots), C, H, H)

    def initial_inference(self, obs, slots=None):
        obs = torch.as_tensor(obs, dtype=torch.float32).to(self.device).contiguous()
        n = obs.shape[0]
        slots = torch.arange(n, dtype=torch.int32, device=self.device) if slots is None else \
            torch.as_tensor(slots, dtype=torch.int32).to(self.device)
        lg = torch.empty(n, self.A, dtype=torch.float32, device=self.device)
        v = torch.empty(n, dtype=torch.float32, device=self.device)
        self.initial(obs, slots, lg, v, _lib.stream_ptr())
        return lg, v, slots

    def recurrent_inference(self, in_slots, actions, out_slots):
        dev = self.device
        i_s = torch.as_tensor(in_slots, dtype=torch.int32).to(dev)
        a = torch.as_tensor(actions, dtype=torch.int32).to(dev)
        o_s = torch.as_tensor(out_slots, dtype=torch.int32).to(dev)
        n = i_s.shape[0]
        lg = torch.empty(n, self.A, dtype=torch.float32, device=dev)
        v = torch.empty(n, dtype=torch.float32, device=dev)
        r = torch.empty(n, dtype=torch.float32, device=dev)
        self.recurrent(i_s, a, o_s, lg, v, r, _lib.stream_ptr())
        return lg, v, r
