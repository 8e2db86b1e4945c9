"""The batched conv-weight re-pack (trainer.BATCH_REPACK, gmz_conv3x3_pack_many): every packed 3x3 weight of the
step re-packed by one launch at the top of the step instead of one gmz_conv3x3_pack at each weight's first use.
The packing is a pure re-layout, so everything is BIT-identical: each job's output equals gmz_conv3x3_pack of the
same weight (contiguous, channels-last, the dynamics stem's [:, :128] view, transposed), and whole training steps —
eager and graph-captured, with a weight changed from outside between replays — equal the per-use path."""
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


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_pack_many_equals_one_pack_per_weight(T, dt):
    from datou_gomoku_muzero_amd import _lib
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    ws = [torch.randn(128, 128, 3, 3, device="cuda", generator=g),
          torch.randn(128, 128, 3, 3, device="cuda", generator=g).contiguous(memory_format=torch.channels_last),
          torch.randn(128, 130, 3, 3, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)[:, :128],
          torch.randn(128, 128, 3, 3, device="cuda", generator=g)]
    trans = [0, 1, 0, 1]
    outs = [torch.full((147456,), -1, dtype=torch.int16, device="cuda") for _ in ws]
    arr = np.zeros(len(ws), dtype=T._PACK_JOB)
    for i, (w, t, o) in enumerate(zip(ws, trans, outs)):
        arr[i] = (w.data_ptr(), w.stride(), o.data_ptr(), t, 0)
    table = torch.from_numpy(arr.view(np.uint8)).cuda()
    _lib.check(L.gmz_conv3x3_pack_many(T._CONV_DTYPES[dt], _lib.ptr(table), len(ws), _lib.stream_ptr()))
    for w, t, o in zip(ws, trans, outs):
        ref = torch.empty_like(o)
        s = w.stride()
        _lib.check(L.gmz_conv3x3_pack(T._CONV_DTYPES[dt], _lib.ptr(w), s[0], s[1], s[2], s[3], t, _lib.ptr(ref),
                                      _lib.stream_ptr()))
        torch.cuda.synchronize()
        assert torch.equal(o, ref)
    with pytest.raises(_lib.GmzError, match="n_jobs"):
        _lib.check(L.gmz_conv3x3_pack_many(1, _lib.ptr(table), 0, _lib.stream_ptr()))
    with pytest.raises(_lib.GmzError, match="dtype"):
        _lib.check(L.gmz_conv3x3_pack_many(3, _lib.ptr(table), 1, _lib.stream_ptr()))


def _batches(cfg, n, B=32):
    from datou_gomoku_muzero_amd import weights as W
    out = []
    for i in range(n):
        obs, act, rew, pol, val = W.synthetic_slices(B, cfg.BOARD_SIZE, cfg.NUM_UNROLL_STEPS, np.random.RandomState(40 + i))
        bt = [torch.as_tensor(x).cuda() for x in (obs, act, rew, pol, val)]
        bt[0] = bt[0].float()
        out.append(bt)
    return out


@pytest.mark.parametrize("graph", [False, True])
def test_training_steps_with_batched_repack_are_bit_identical(T, monkeypatch, graph):
    """6 steps (9x9, 2 blocks, B = 32), graph-captured after 2 eager ones or all eager; before step 4 a conv weight
    is changed in place from outside (as a weight load would): losses, weights and the packed caches bit-identical
    with and without BATCH_REPACK, and with it every cached pack is current after each step."""
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)
    bs = _batches(cfg, 2)
    w = torch.rand(32, device="cuda") + 0.5
    runs = []
    for batched in (False, True):
        monkeypatch.setattr(T, "BATCH_REPACK", batched)
        torch.manual_seed(0)
        tr = T.Trainer(cfg, device="cuda", graph=graph, graph_warmup=2)
        tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
        conv = tr.model.representation_net.resblocks[0].conv1.weight
        logs = []
        for i in range(6):
            if i == 3:
                with torch.no_grad():
                    conv.mul_(0.5)
            logs.append(tr.step(bs[i % 2], w, k=i % 4, flip=bool(i % 2))[0])
        torch.cuda.synchronize()
        if batched:
            assert tr._pack_tables, "no batched re-pack ran"
        params = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()])
        runs.append((np.array(logs), params.cpu()))
    assert np.array_equal(runs[0][0], runs[1][0]), runs
    assert torch.equal(runs[0][1].view(torch.int32), runs[1][1].view(torch.int32))


def test_batched_repack_leaves_every_pack_current(T, monkeypatch):
    """After the top-of-step re-pack, each cached entry is the pack of its parameter's current value."""
    from datou_gomoku_muzero_amd import _lib
    monkeypatch.setattr(T, "BATCH_REPACK", True)
    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)
    bs = _batches(cfg, 1)
    w = torch.ones(32, device="cuda")
    tr = T.Trainer(cfg, device="cuda", graph=False)
    tr.scaler = torch.amp.GradScaler("cuda", init_scale=1.0 / 16)
    for i in range(2):
        tr.step(bs[0], w, k=i, flip=False)
    owners = list(tr.model.parameters()) + list(tr.target.parameters())
    assert T._repack_stale(owners, tr._pack_tables) > 0  # the update made them stale; one launch re-packed them
    assert T._repack_stale(owners, tr._pack_tables) == 0
    torch.cuda.synchronize()
    n = 0
    for p in owners:
        for key, hit in p.__dict__.get("_gmz_pack", {}).items():
            if len(hit) != 5:
                continue
            assert hit[0] == p._version
            ref = torch.empty_like(hit[1])
            s = hit[2].stride()
            _lib.check(_lib.load().gmz_conv3x3_pack(T._CONV_DTYPES[hit[4]], _lib.ptr(hit[2]), s[0], s[1], s[2], s[3],
                                                    hit[3], _lib.ptr(ref), _lib.stream_ptr()))
            torch.cuda.synchronize()
            assert torch.equal(ref, hit[1]), key
            n += 1
    assert n >= 8
