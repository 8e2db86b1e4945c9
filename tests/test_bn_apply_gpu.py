"""The training-mode BatchNorm applied in the consuming 3x3 conv's prologue (trainer.DEFER_BN_APPLY,
gmz_bn_forward_deferred + gmz_conv3x3_forward_bnapply; VERDICT r5 next #4, the residual blocks of network.py:30-48
trained by loss.py:70-111).  The prologue computes the same float32 expression as the BatchNorm's own elementwise
pass (k_bnl_apply) and rounds once, so everything is BIT-identical to the two-pass path: the normalised activation
it writes, the conv output and its statistics partials, the running statistics, and a whole training step."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from datou_gomoku_muzero_amd import trainer
    return trainer


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _bits(t):
    """t's bit pattern (so that bit-identical means bit-identical, -0 and NaN included)"""
    t = t.contiguous()
    return t.view({2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()]) if t.is_floating_point() else t


@pytest.mark.parametrize("H,N,dt,res,relu", [(15, 37, torch.float16, True, True), (15, 360, torch.float16, False, True),
                                             (9, 24, torch.float16, True, True), (9, 5, torch.bfloat16, True, False),
                                             (15, 3, torch.bfloat16, False, True)])
def test_bnapply_conv_equals_bn_then_conv(T, H, N, dt, res, relu):
    from datou_gomoku_muzero_amd import _lib
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(H * 1000 + N)
    z = _cl(torch.randn(N, 128, H, H, device="cuda", generator=g).to(dt))
    r = _cl(torch.randn(N, 128, H, H, device="cuda", generator=g).to(dt)) if res else None
    gamma = torch.rand(128, device="cuda", generator=g) + 0.5
    beta = torch.randn(128, device="cuda", generator=g) * 0.1
    w = torch.randn(128, 128, 3, 3, device="cuda", generator=g) / 34
    dcode = T._CONV_DTYPES[dt]
    packed = T._packed_conv_weight(w, dt, 0)
    mask = (torch.rand(N, device="cuda", generator=g) > 0.3).view(torch.uint8)
    # statistics of z from a stats conv of its own (the producer), shared by both paths
    st, ns = T._conv_stats_buffer(N, z.device)
    zin = _cl(torch.randn(N, 128, H, H, device="cuda", generator=g).to(dt))
    _lib.check(L.gmz_conv3x3_forward_stats(dcode, H, _lib.ptr(zin), _lib.ptr(packed), _lib.ptr(z), N, _lib.ptr(mask),
                                           _lib.ptr(st), ns, _lib.stream_ptr()))
    outs = []
    for deferred in (False, True):
        rm, rv = torch.zeros(128, device="cuda"), torch.ones(128, device="cuda")
        nb = torch.zeros(1, dtype=torch.int64, device="cuda")
        save = torch.empty(2, 128, device="cuda")
        y = torch.full_like(z, 3.0)
        out = torch.empty_like(z)
        st2, ns2 = T._conv_stats_buffer(N, z.device)
        if deferred:
            _lib.check(L.gmz_bn_forward_deferred(dcode, _lib.ptr(z), _lib.ptr(mask), N, 128, H * H, 1e-4, 0.1,
                                                 _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nb), _lib.ptr(save), _lib.ptr(st), ns,
                                                 _lib.nbytes(st), None, 0, _lib.stream_ptr()))
            _lib.check(L.gmz_conv3x3_forward_bnapply(dcode, H, _lib.ptr(z), _lib.ptr(r), _lib.ptr(gamma), _lib.ptr(beta),
                                                     _lib.ptr(save), int(relu), _lib.ptr(y), _lib.ptr(packed),
                                                     _lib.ptr(out), N, _lib.ptr(mask), _lib.ptr(st2), ns2,
                                                     _lib.stream_ptr()))
        else:
            _lib.check(L.gmz_bn_forward_stats(dcode, _lib.ptr(z), _lib.ptr(r), N, 128, H * H, _lib.ptr(gamma),
                                              _lib.ptr(beta), 1e-4, 0.1, _lib.ptr(rm), _lib.ptr(rv), _lib.ptr(nb),
                                              int(relu), _lib.ptr(y), _lib.ptr(save), _lib.ptr(st), ns, _lib.nbytes(st),
                                              _lib.stream_ptr()))
            _lib.check(L.gmz_conv3x3_forward_stats(dcode, H, _lib.ptr(y), _lib.ptr(packed), _lib.ptr(out), N,
                                                   _lib.ptr(mask), _lib.ptr(st2), ns2, _lib.stream_ptr()))
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (y, out, st2, rm, rv, nb, save)])
    for a, b in zip(*outs):
        assert torch.equal(_bits(a), _bits(b))
    # and the normalisation itself against float32 torch (the saved statistics)
    y = outs[1][0].float()
    ref = (z.float() - outs[1][6][0].view(1, -1, 1, 1)) * (gamma * outs[1][6][1]).view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)
    if res:
        ref = ref + r.float()
    if relu:
        ref = ref.clamp_min(0)
    assert float((y - ref).abs().max()) <= 1e-2 * float(ref.abs().max())


def test_bnapply_capacity_and_alias_checks(T):
    from datou_gomoku_muzero_amd import _lib
    L = _lib.load()
    N, H = 8, 9
    z = _cl(torch.randn(N, 128, H, H, device="cuda").half())
    y, out = torch.empty_like(z), torch.empty_like(z)
    gamma, beta, save = torch.ones(128, device="cuda"), torch.zeros(128, device="cuda"), torch.zeros(2, 128, device="cuda")
    packed = T._packed_conv_weight(torch.randn(128, 128, 3, 3, device="cuda"), torch.float16, 0)
    st, ns = T._conv_stats_buffer(N, z.device)
    with pytest.raises(_lib.GmzError, match="slots"):
        _lib.check(L.gmz_conv3x3_forward_bnapply(1, H, _lib.ptr(z), None, _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(save),
                                                 1, _lib.ptr(y), _lib.ptr(packed), _lib.ptr(out), N, None, _lib.ptr(st),
                                                 ns - 1, _lib.stream_ptr()))
    with pytest.raises(_lib.GmzError, match="alias"):
        _lib.check(L.gmz_conv3x3_forward_bnapply(1, H, _lib.ptr(z), None, _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(save),
                                                 1, _lib.ptr(z), _lib.ptr(packed), _lib.ptr(out), N, None, None, 0,
                                                 _lib.stream_ptr()))
    with pytest.raises(_lib.GmzError, match="statistics partials"):
        _lib.check(L.gmz_bn_forward_deferred(1, _lib.ptr(z), None, N, 128, H * H, 1e-4, 0.1, None, None, None,
                                             _lib.ptr(save), _lib.ptr(st), ns, _lib.nbytes(st) - 8, None, 0,
                                             _lib.stream_ptr()))


@pytest.mark.parametrize("H,blocks,B", [(15, 3, 24), (9, 2, 40)])
def test_trunk_with_deferred_bn_is_bit_identical(T, monkeypatch, H, blocks, B):
    """A representation trunk (MIOpen stem + residual blocks) forward and backward under fp16 autocast, with and
    without DEFER_BN_APPLY: output, input gradient, every parameter gradient and running statistic bit-identical
    (MIOpen's stem conv in deterministic mode: its own algorithm choice must not differ between the runs)."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(7)
    trunk = T._Trunk(4, 128, blocks).cuda().to(memory_format=torch.channels_last).train()
    for m in trunk.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.normal_(0, 0.1)
    x0 = _cl(torch.randn(B, 4, H, H, device="cuda"))
    dy = torch.randn(B, 128, H, H, device="cuda")
    mask = torch.ones(B, dtype=torch.bool, device="cuda")
    mask[B // 3:B // 2] = False
    init = {k: v.clone() for k, v in trunk.state_dict().items()}
    outs = []
    for defer in (False, True):
        monkeypatch.setattr(T, "DEFER_BN_APPLY", defer)
        trunk.load_state_dict(init)
        trunk.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.float16):
            y = trunk(x, mask)
        y.float().backward(dy)
        torch.cuda.synchronize()
        outs.append([y.detach().clone(), x.grad.clone()] + [p.grad.clone() for p in trunk.parameters()]
                    + [b.clone() for b in trunk.buffers()])
    names = ["y", "x.grad"] + ["grad " + n for n, _ in trunk.named_parameters()] + [n for n, _ in trunk.named_buffers()]
    bad = [n for n, a, b in zip(names, *outs) if not torch.equal(_bits(a), _bits(b))]
    assert not bad, bad


def test_training_step_with_deferred_bn_is_bit_identical(T, monkeypatch):
    """The graph-captured production step (9x9, 2 blocks, B = 32): losses and weights after 4 steps bit-identical
    with and without DEFER_BN_APPLY."""
    from datou_gomoku_muzero_amd import weights as W
    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)
    batches = []
    for i in range(2):
        obs, act, rew, pol, val = W.synthetic_slices(32, 9, cfg.NUM_UNROLL_STEPS, np.random.RandomState(5 + i))
        bt = [torch.as_tensor(v).cuda() for v in (obs, act, rew, pol, val)]
        bt[0] = bt[0].float()
        batches.append(bt)
    w = torch.rand(32, device="cuda") + 0.5
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    runs = []
    for defer in (False, True):
        monkeypatch.setattr(T, "DEFER_BN_APPLY", defer)
        torch.manual_seed(0)
        tr = T.Trainer(cfg, device="cuda", graph_warmup=2)
        logs = [tr.step(batches[i % 2], w, k=i % 4, flip=bool(i % 2))[0] for i in range(4)]
        runs.append((np.array(logs), torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu()))
    assert np.array_equal(runs[0][0], runs[1][0]), runs
    assert torch.equal(_bits(runs[0][1]), _bits(runs[1][1]))
