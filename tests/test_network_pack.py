"""CPU checks of the HIP network's weight packing (network.py): fragment layouts invert exactly,
and a float32 emulation of the kernels' algebra on the packed (BN-folded, f16 or bf16) weights matches
the oracle forward (oracle/netref.py) within the 16-bit weight-rounding tolerance."""
import numpy as np
import pytest

import netref
from datou_gomoku_muzero_amd import network as N
from datou_gomoku_muzero_amd import weights as W
from datou_gomoku_muzero_amd.config import GmzConfig


PREC = "fp16"  # set by the `small` fixture


def bf(u16, prec=None):
    """16-bit patterns of the packing precision -> float32."""
    u = np.asarray(u16, np.uint16)
    if (prec or PREC) == "fp16":
        return u.view(np.float16).astype(np.float32)
    return (u.astype(np.uint32) << 16).view(np.float32)


def unpack_conv(pk):  # [9][4][8][64][8] -> [9][n][c]
    out = np.zeros((9, 128, 128), np.float32)
    ks, nt, l, j = np.meshgrid(np.arange(4), np.arange(8), np.arange(64), np.arange(8), indexing="ij")
    out[:, N.output_channel(nt, l & 15), N.conv_input_channel(ks, l, j)] = bf(pk)
    return out


def conv_from_taps(x, Wt, bias):  # x [B, C, H, W], Wt [9][n][c]
    B, Cc, H, _ = x.shape
    xp = np.zeros((B, Cc, H + 2, H + 2), np.float32)
    xp[:, :, 1:-1, 1:-1] = x
    out = np.zeros((B, Wt.shape[1], H, H), np.float32)
    for t in range(9):
        dy, dx = t // 3, t % 3
        out += np.einsum("nc,bchw->bnhw", Wt[t], xp[:, :, dy:dy + H, dx:dx + H], optimize=True)
    return out + bias.reshape(1, -1, 1, 1)


@pytest.fixture(scope="module", params=["fp16", "bf16"])
def small(request):
    global PREC
    PREC = request.param
    cfg = GmzConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=2)
    sd = W.synthetic_state_dict(cfg, seed=9, with_projection=False)
    return cfg, sd, N.pack_weights(sd, cfg, request.param)


def test_output_channel_is_a_permutation_in_16_byte_chunks():
    nt, m = np.meshgrid(np.arange(8), np.arange(16), indexing="ij")
    ch = N.output_channel(nt, m)
    assert sorted(ch.ravel()) == list(range(128))
    # lane group g (rows 4g..4g+3) of tiles 2u, 2u+1: channels 32u + 8g + 0..7 (one 16-B chunk)
    for u in range(4):
        for g in range(4):
            got = np.concatenate([ch[2 * u, 4 * g:4 * g + 4], ch[2 * u + 1, 4 * g:4 * g + 4]])
            assert list(got) == list(range(32 * u + 8 * g, 32 * u + 8 * g + 8))


def test_conv_pack_inverts(small):
    cfg, sd, pk = small
    s, _ = N.fold_bn(sd, "representation_net.resblocks.0.bn1")
    wf = sd["representation_net.resblocks.0.conv1.weight"] * s[:, None, None, None]
    got = unpack_conv(pk["repr_convs"][0])
    want = bf(N._e16_bits(wf.transpose(2, 3, 0, 1).reshape(9, 128, 128), PREC))
    assert (got == want).all()


def emulate(pk, cfg, obs=None, h=None, action=None):
    """float32 emulation of csrc/gmz_net.hip on packed weights (activations kept in f32)."""
    H = cfg.BOARD_SIZE
    A = H * H
    nb = cfg.NUM_RES_BLOCKS
    if obs is not None:
        Wk = np.zeros((128, 32), np.float32)
        nt, l, j = np.meshgrid(np.arange(8), np.arange(64), np.arange(8), indexing="ij")
        Wk[N.output_channel(nt, l & 15), 8 * (l >> 4) + j] = bf(pk["repr_stem_w"])
        Wt = np.zeros((9, 128, 3), np.float32)
        for t in range(9):
            Wt[t] = Wk[:, t * 3:t * 3 + 3]
        x = np.maximum(conv_from_taps(obs, Wt, pk["repr_stem_b"]), 0)
        convs, bias = pk["repr_convs"], pk["repr_bias"]
        L0 = 0
    else:
        B = h.shape[0]
        x = conv_from_taps(h, unpack_conv(pk["dyn_convs"][0]), pk["dyn_bias"][0])
        for b in range(B):
            ay, ax = divmod(int(action[b]), H)
            for t in range(9):
                y, xx = ay - (t // 3 - 1), ax - (t % 3 - 1)
                if 0 <= y < H and 0 <= xx < H:
                    x[b, :, y, xx] += pk["dyn_action"][t]
        x = np.maximum(x, 0)
        convs, bias = pk["dyn_convs"], pk["dyn_bias"]
        L0 = 1
    for i in range(nb):
        t1 = np.maximum(conv_from_taps(x, unpack_conv(convs[L0 + 2 * i]), bias[L0 + 2 * i]), 0)
        x = np.maximum(conv_from_taps(t1, unpack_conv(convs[L0 + 2 * i + 1]), bias[L0 + 2 * i + 1]) + x, 0)
    B = x.shape[0]
    feat = np.maximum(np.einsum("oc,bchw->bohw", pk["head_conv_w"], x) + pk["head_conv_b"].reshape(1, 3, 1, 1), 0)
    feat = feat.reshape(B, 3 * A)
    logits = feat[:, :2 * A] @ pk["policy_fc_w"][:A, :2 * A].T + pk["policy_fc_b"]
    hv = np.maximum(feat[:, 2 * A:] @ pk["value_fc1_w"][:, :A].T + pk["value_fc1_b"], 0)
    value = netref.support_to_scalar(hv @ pk["value_fc2_w"] + pk["value_fc2_b"])
    reward = None
    if obs is None:
        Wn = np.zeros((A * 128, 64), np.float32)
        kk, nt, l, j = np.meshgrid(np.arange(A * 128 // 32), np.arange(4), np.arange(64), np.arange(8), indexing="ij")
        Wn[kk * 32 + 8 * (l >> 4) + j, nt * 16 + (l & 15)] = bf(pk["reward_fc1_w"])
        hn = x.transpose(0, 2, 3, 1).reshape(B, -1)  # NHWC flatten
        hr = np.maximum(hn @ Wn + pk["reward_fc1_b"], 0)
        reward = netref.support_to_scalar(hr @ pk["reward_fc2_w"] + pk["reward_fc2_b"])
    return logits, value, x, reward


def test_packed_emulation_matches_oracle(small):
    cfg, sd, pk = small
    rs = np.random.RandomState(0)
    obs = (rs.rand(3, 3, 6, 6) < 0.3).astype(np.float32)
    p, v, h = netref.initial_inference(sd, obs)
    ep, ev, eh, _ = emulate(pk, cfg, obs=obs)
    scale = np.abs(p).max()
    tol = 0.003 if PREC == "fp16" else 0.02  # weight rounding only: 2^-11 vs 2^-8 relative
    assert np.abs(ep - p).max() <= tol * scale + 1e-3
    assert np.abs(ev - v).max() <= tol
    acts = np.array([0, 17, 35])
    p2, v2, h2, r2 = netref.recurrent_inference(sd, h, acts)
    ep2, ev2, eh2, er2 = emulate(pk, cfg, h=h, action=acts)
    assert np.abs(ep2 - p2).max() <= tol * np.abs(p2).max() + 1e-3
    assert np.abs(ev2 - v2).max() <= tol and np.abs(er2 - r2).max() <= tol
    assert np.abs(eh2 - h2).max() <= tol * np.abs(h2).max()
