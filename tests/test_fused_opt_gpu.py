"""The trainer's optimiser step on the GPU (trainer.FUSED_OPT, gmz_opt_step): GradScaler.unscale_ + clip_grad_norm_ +
torch.optim.Adam (L2 weight decay) + GradScaler.update + the soft target update of utils.py:28-31 + zero_grad, in
three launches over the flat gradient bucket (workers.py:565-583).  Against PyTorch's own path (FUSED_OPT = False):
the same steps within float32 rounding of the gradient norm and the Adam moments; a non-finite gradient skips Adam
exactly as GradScaler.step does; the optimiser state keeps the reference's state_dict format and resumes exactly."""
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


def _batches(T, cfg, n, B=32):
    from datou_gomoku_muzero_amd import weights as W
    out = []
    for i in range(n):
        obs, act, rew, pol, val = W.synthetic_slices(B, cfg.BOARD_SIZE, cfg.NUM_UNROLL_STEPS, np.random.RandomState(70 + i))
        bt = [torch.as_tensor(x).cuda() for x in (obs, act, rew, pol, val)]
        bt[0] = bt[0].float()
        out.append(bt)
    return out


def _cfg(T):
    return T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)


def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def test_fused_optimiser_matches_pytorch_adam(T, monkeypatch):
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg = _cfg(T)
    bs = _batches(T, cfg, 3)
    w = torch.rand(32, device="cuda") + 0.5
    runs = []
    for fused in (False, True):
        monkeypatch.setattr(T, "FUSED_OPT", fused)
        torch.manual_seed(0)
        tr = T.Trainer(cfg, device="cuda", graph_warmup=2)
        # this synthetic batch's gradient norm is ~2e5: the GradScaler's default 65,536 overflows f16 for ~16 steps
        tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
        logs = [tr.step(bs[i % 3], w, k=i % 4, flip=bool(i % 2))[0] for i in range(6)]
        torch.cuda.synchronize()
        ost = tr.opt.state_dict()["state"]
        runs.append((np.array(logs), _flat(tr.model), _flat(tr.target),
                     torch.cat([ost[i]["exp_avg"].reshape(-1) for i in range(len(tr.params))]),
                     float(ost[0]["step"]), float(tr.scaler.get_scale())))
        assert (tr._fopt is not None) == fused
        assert float(tr.flat_grad.abs().max()) == 0.0  # zeroed for the next step
    (l0, p0, t0, m0, s0, sc0), (l1, p1, t1, m1, s1, sc1) = runs
    assert np.array_equal(l0[0], l1[0])  # the first forward precedes any update
    # later steps: training dynamics from different float32 roundings (this 32-game batch's BatchNorm statistics
    # amplify them: the small loss components move by up to ~1.5 % within 6 steps)
    assert np.allclose(l0, l1, rtol=3e-2, atol=1e-3), (l0, l1)
    lr, steps = cfg.LEARNING_RATE, 6
    d = (p0 - p1).abs()
    # six steps of training dynamics from different float32 roundings (the gradient norm's summation order): Adam
    # divides each update by the gradient's own scale, so a parameter with a near-zero gradient turns them into
    # lr-scale steps; nearly every element agrees to a tenth of one step (the kernel's arithmetic itself is pinned
    # by the one-step test below)
    assert float(d.max()) <= 2 * lr * steps, float(d.max())
    assert float((d > 0.1 * lr).float().mean()) < 0.01, float((d > 0.1 * lr).float().mean())
    assert float((t0 - t1).abs().max()) <= 2 * lr * steps
    assert s0 == s1 == 6.0 and sc0 == sc1  # every step taken on both paths (no overflow at this scale)


def test_one_fused_step_equals_pytorchs_from_the_same_gradient(T, monkeypatch):
    """One optimiser step from identical weights, moments and gradient: parameters, moments, target and the
    GradScaler's scale within float32 rounding of PyTorch's unscale_ / clip_grad_norm_ / fused Adam / soft update
    (the gradient norm is summed in f64 in another order: clip coefficient rounding only)."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg = _cfg(T)
    bs = _batches(T, cfg, 2)
    w = torch.rand(32, device="cuda") + 0.5
    trs = []
    for fused in (False, True):
        monkeypatch.setattr(T, "FUSED_OPT", fused)
        torch.manual_seed(3)
        tr = T.Trainer(cfg, device="cuda", graph=False)
        tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
        tr.step(bs[0], w, k=0, flip=False)  # one step on each path: non-zero moments to start from
        trs.append(tr)
    a, b = trs
    with torch.no_grad():  # identical starting state
        for pa, pb in zip(list(a.model.parameters()) + list(a.target.parameters()),
                          list(b.model.parameters()) + list(b.target.parameters())):
            pb.copy_(pa)
        for pa, pb in zip(a.params, b.params):
            sa, sb = a.opt.state[pa], b.opt.state[pb]
            sb["exp_avg"].copy_(sa["exp_avg"])
            sb["exp_avg_sq"].copy_(sa["exp_avg_sq"])
        b.scaler._scale.copy_(a.scaler._scale)
    a._forward_backward(bs[1], w, k=1, flip=True)
    monkeypatch.setattr(T, "FUSED_OPT", True)
    b.flat_grad.copy_(a.flat_grad)
    b._update()
    monkeypatch.setattr(T, "FUSED_OPT", False)
    a._update()
    torch.cuda.synchronize()
    pa, pb = _flat(a.model), _flat(b.model)
    step = a.opt.param_groups[0]["lr"]
    assert float((pa - pb).abs().max()) <= 1e-6 + 1e-3 * float(step), float((pa - pb).abs().max())
    assert float((_flat(a.target) - _flat(b.target)).abs().max()) <= 1e-6
    for key in ("exp_avg", "exp_avg_sq"):
        ma = torch.cat([a.opt.state[p][key].reshape(-1) for p in a.params])
        mb = torch.cat([b.opt.state[p][key].reshape(-1) for p in b.params])
        assert float((ma - mb).abs().max()) <= 1e-5 * float(ma.abs().max()) + 1e-12, key
    assert float(a.scaler.get_scale()) == float(b.scaler.get_scale())


def test_non_finite_gradient_skips_adam_but_not_the_target_update(T):
    cfg = _cfg(T)
    bs = _batches(T, cfg, 1)
    w = torch.ones(32, device="cuda")
    torch.manual_seed(1)
    tr = T.Trainer(cfg, device="cuda", graph=False)
    tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)  # a scale this batch's gradients fit in f16
    tr.step(bs[0], w, k=0, flip=False)
    tr.step(bs[0], w, k=2, flip=False)
    torch.cuda.synchronize()
    assert tr._fopt is not None and float(tr._fopt["step"]) == 2.0
    p_before, t_before = _flat(tr.model).clone(), _flat(tr.target).clone()
    step_before, scale_before = float(tr._fopt["step"]), float(tr.scaler.get_scale())
    m_before = tr._fopt["m"].clone()
    tr.flat_grad.fill_(1.0)
    tr.flat_grad[123] = float("inf")
    tr._update()
    torch.cuda.synchronize()
    assert torch.equal(_flat(tr.model), p_before)  # Adam skipped
    assert torch.equal(tr._fopt["m"], m_before) and float(tr._fopt["step"]) == step_before
    assert float(tr.scaler.get_scale()) == scale_before * 0.5  # GradScaler backoff
    tau = cfg.TARGET_MODEL_TAU
    want = t_before * (1.0 - tau) + p_before * tau  # the soft update still ran
    assert float((_flat(tr.target) - want).abs().max()) <= 1e-6
    assert float(tr.flat_grad.abs().max()) == 0.0
    # and a finite step afterwards advances the step counter again
    tr.step(bs[0], w, k=1, flip=True)
    torch.cuda.synchronize()
    assert float(tr._fopt["step"]) == step_before + 1


def test_fused_step_advances_the_packed_weight_caches(T):
    """The fused kernel writes the parameters through raw pointers; their version counters must still advance, or the
    packed conv weights (cached per version) of the next eager step — and of a graph captured after it — are stale."""
    cfg = _cfg(T)
    bs = _batches(T, cfg, 1)
    w = torch.ones(32, device="cuda")
    tr = T.Trainer(cfg, device="cuda", graph=False)
    tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
    conv = tr.model.representation_net.resblocks[0].conv1.weight
    tconv = tr.target.representation_net.resblocks[0].conv1.weight
    v0, t0 = conv._version, tconv._version
    tr.step(bs[0], w, k=0, flip=False)
    assert conv._version > v0 and tconv._version > t0
    packed = T._packed_conv_weight(conv, torch.float16, 0)
    fresh = torch.empty_like(packed)
    from datou_gomoku_muzero_amd import _lib
    s = conv.stride()
    _lib.check(_lib.load().gmz_conv3x3_pack(1, _lib.ptr(conv.detach()), s[0], s[1], s[2], s[3], 0, _lib.ptr(fresh),
                                            _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(packed, fresh)  # the cache re-packed the updated weight


def test_fused_optimiser_state_resumes_exactly(T, monkeypatch):
    """trainer_state() after fused steps is the reference's optimiser dict; a second trainer resumed from it takes
    the next step bit-identically to the first."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg = _cfg(T)
    bs = _batches(T, cfg, 2)
    w = torch.rand(32, device="cuda") + 0.5
    torch.manual_seed(2)
    a = T.Trainer(cfg, device="cuda", graph=False)
    a.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
    for i in range(3):
        a.step(bs[i % 2], w, k=i, flip=False)
    state = a.trainer_state()
    ost = state["optimizer_state_dict"]["state"]
    assert set(ost) == set(range(len(a.params)))
    assert all(float(ost[i]["step"]) == 3.0 and ost[i]["exp_avg"].device.type == "cpu" for i in ost)
    b = T.Trainer(cfg, device="cuda", graph=False)
    b.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
    b.load_trainer_state(state)
    b.target.load_state_dict(a.target.state_dict())  # the reference restarts its target from the model; align them
    b.scaler.load_state_dict(a.scaler.state_dict())
    la = a.step(bs[0], w, k=0, flip=True)[0]
    lb = b.step(bs[0], w, k=0, flip=True)[0]
    torch.cuda.synchronize()
    assert la == lb
    assert torch.equal(_flat(a.model), _flat(b.model))
    assert torch.equal(a._fopt["m"], b._fopt["m"]) and torch.equal(a._fopt["v"], b._fopt["v"])
