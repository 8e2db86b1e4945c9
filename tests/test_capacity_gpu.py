"""ABI 10 capacity arguments on the GPU: an undersized caller buffer fails cleanly — a
gmz_last_error() message, nothing launched, the output and partials buffers untouched — and the same call with the
right size runs.  The fault classes of round 5 were a statistics-partials buffer sized for another launch variant
(k_conv3db) and an f16 stamp table read as f32 [9][128]; tests/test_abi.py checks every capacity argument on the CPU,
this one checks that a refused call leaves device memory as it was."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def _setup(N=40, H=9):
    import torch
    from datou_gomoku_muzero_amd import _lib
    L = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(N, H * H, 128, device="cuda", generator=g).half()
    w = torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.05
    packed = torch.empty(294912 // 2, dtype=torch.int16, device="cuda")
    _lib.check(L.gmz_conv3x3_pack(1, _lib.ptr(w), *w.stride(), 0, _lib.ptr(packed), _lib.stream_ptr()))
    ns = ctypes.c_int()
    _lib.check(L.gmz_conv3x3_stats_slots(N, ctypes.byref(ns)))
    return torch, _lib, L, x, packed, ns.value


def test_short_statistics_buffer_is_refused_and_untouched():
    torch, _lib, L, x, packed, ns = _setup()
    N, H = x.shape[0], 9
    y = torch.full_like(x, 7.0)
    st = torch.full((128 * (ns - 1) * 3,), float("nan"), dtype=torch.float64, device="cuda")
    with pytest.raises(_lib.GmzError, match="slots"):
        _lib.check(L.gmz_conv3x3_forward_stats(1, H, _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y), N, None, _lib.ptr(st),
                                               ns - 1, _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert bool((y == 7.0).all()) and bool(st.isnan().all())  # no launch: nothing written
    st = torch.full((128 * ns * 3,), float("nan"), dtype=torch.float64, device="cuda")
    _lib.check(L.gmz_conv3x3_forward_stats(1, H, _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y), N, None, _lib.ptr(st), ns,
                                           _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert not bool(st.isnan().any()) and not bool((y == 7.0).all())
    # the statistics sums equal the output's (f64 vs the kernel's f32-per-lane partials)
    ref = y.double().sum((0, 1))
    got = st.view(128, ns, 3)[:, :, 0].sum(1)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-2)


def test_stamp_table_of_the_wrong_dtype_is_refused():
    torch, _lib, L, x, packed, ns = _setup()
    N, H = x.shape[0], 9
    y = torch.full_like(x, 7.0)
    act = torch.randint(0, H * H, (N,), dtype=torch.int32, device="cuda")
    t16 = torch.randn(9, 128, device="cuda").half()  # the round-5 fault: an f16 table (2,304 bytes)
    with pytest.raises(_lib.GmzError, match="table"):
        _lib.check(L.gmz_conv3x3_forward_stamp(1, H, _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y), N, None, None, 0,
                                               _lib.ptr(act), _lib.ptr(t16), 1, _lib.nbytes(t16), _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert bool((y == 7.0).all())
    t32 = t16.float()
    _lib.check(L.gmz_conv3x3_forward_stamp(1, H, _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y), N, None, None, 0,
                                           _lib.ptr(act), _lib.ptr(t32), 0, _lib.nbytes(t32), _lib.stream_ptr()))
    y0 = torch.empty_like(x)
    _lib.check(L.gmz_conv3x3_forward(1, H, _lib.ptr(x), _lib.ptr(packed), _lib.ptr(y0), N, _lib.stream_ptr()))
    torch.cuda.synchronize()
    # the stamp adds table[tap] at the 3x3 window around each board's action cell, nothing elsewhere
    d = (y.float() - y0.float()).view(N, H, H, 128)
    a = act.long().cpu()
    far = torch.ones(N, H, H, dtype=torch.bool)
    for n in range(N):
        ay, ax = int(a[n]) // H, int(a[n]) % H
        far[n, max(0, ay - 1):ay + 2, max(0, ax - 1):ax + 2] = False
    assert float(d[far.cuda()].abs().max()) == 0.0


def test_short_workspaces_are_refused():
    torch, _lib, L, x, packed, ns = _setup()
    N, H = x.shape[0], 9
    need = ctypes.c_size_t()
    _lib.check(L.gmz_conv3x3_wgrad_workspace_bytes(N, ctypes.byref(need)))
    ws = torch.full((need.value // 4,), 3.0, device="cuda")
    dw = torch.zeros(128, 128, 3, 3, device="cuda")
    with pytest.raises(_lib.GmzError, match="workspace"):
        _lib.check(L.gmz_conv3x3_wgrad(1, H, _lib.ptr(x), _lib.ptr(x), N, _lib.ptr(dw), *dw.stride(), 1, _lib.ptr(ws),
                                       need.value - 4, _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert bool((ws == 3.0).all()) and bool((dw == 0).all())
    _lib.check(L.gmz_bn_workspace_bytes(1, N, 128, H * H, ctypes.byref(need)))
    ws = torch.full((need.value // 8,), 3.0, dtype=torch.float64, device="cuda")
    gamma, beta = torch.ones(128, device="cuda"), torch.zeros(128, device="cuda")
    y = torch.full_like(x, 7.0)
    save = torch.zeros(2, 128, device="cuda")
    with pytest.raises(_lib.GmzError, match="workspace"):
        _lib.check(L.gmz_bn_forward(1, 1, _lib.ptr(x), None, None, N, 128, H * H, _lib.ptr(gamma), _lib.ptr(beta), 1e-4,
                                    0.1, None, None, None, 1, _lib.ptr(y), _lib.ptr(save), _lib.ptr(ws), need.value - 8,
                                    _lib.stream_ptr()))
    torch.cuda.synchronize()
    assert bool((ws == 3.0).all()) and bool((y == 7.0).all())
    _lib.check(L.gmz_bn_forward(1, 1, _lib.ptr(x), None, None, N, 128, H * H, _lib.ptr(gamma), _lib.ptr(beta), 1e-4, 0.1,
                                None, None, None, 1, _lib.ptr(y), _lib.ptr(save), _lib.ptr(ws), need.value,
                                _lib.stream_ptr()))
    torch.cuda.synchronize()
    ref = torch.relu(torch.nn.functional.batch_norm(x.float().permute(0, 2, 1), None, None, training=True, eps=1e-4))
    assert float((y.float().permute(0, 2, 1) - ref).abs().max()) < 2e-2
