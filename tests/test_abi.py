"""The C ABI library loads (no GPU needed) and exports every symbol include/gmz.h declares."""
import os
import re

from conftest import REPO


def test_library_exports_every_header_symbol():
    import datou_gomoku_muzero_amd._lib as L
    import datou_gomoku_muzero_amd.network  # noqa: F401  (registers the gmz_net_* signatures)
    lib = L.load()
    hdr = open(os.path.join(REPO, "include", "gmz.h")).read()
    names = re.findall(r"^\s*(?:int|const char \*)\s*(gmz_\w+)\(", hdr, re.M)
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.gmz_abi_version() == 10


def test_product_package_never_imports_oracle():
    """Only tests/, smoke() and bench.py's cpu_baseline may touch oracle/ (the checker)."""
    pkg = os.path.join(REPO, "datou-gomoku-muzero_amd")
    bad = re.compile(r"\bimport oracle\b|from oracle\b|gmz_oracle|\bnetref\b|\bimport hashnet\b")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                assert not bad.search(open(os.path.join(root, f)).read()), f


def test_capacity_arguments_fail_before_any_launch():
    """ABI 10: an entry point handed a buffer shorter than what it would write (or read) fails with
    gmz_last_error() and launches nothing.  The pointers are never dereferenced on these paths (they are fake, and
    there is no GPU here): each call must stop at its capacity check."""
    import ctypes
    import datou_gomoku_muzero_amd._lib as L
    from datou_gomoku_muzero_amd import network
    lib = L.load()
    fake = ctypes.c_void_p(1 << 20)
    err = lambda: lib.gmz_last_error().decode()  # noqa: E731
    ns = ctypes.c_int()
    assert lib.gmz_conv3x3_stats_slots(360, ctypes.byref(ns)) == 0 and ns.value > 0
    # conv statistics partials: the slot count is the partials' row stride, so it must match the launch exactly
    for bad in (ns.value - 1, ns.value + 1):
        assert lib.gmz_conv3x3_forward_stats(1, 15, fake, fake, fake, 360, None, fake, bad, None) < 0
        assert "slots" in err()
        assert lib.gmz_conv3x3_forward_bwdstats(1, 15, fake, fake, None, fake, 360, None, fake, fake, fake, 1, fake, bad,
                                                None) < 0
        assert "slots" in err()
    assert lib.gmz_conv3x3_forward_board_stats(1, 15, fake, fake, fake, 360, None, fake, 359, None) < 0
    assert "one per board" in err()
    # the dynamics stem's stamp table: f32 [9][128] only (the round-5 faults: an f16 table of 2,304 bytes)
    assert lib.gmz_conv3x3_forward_stamp(1, 15, fake, fake, fake, 8, None, None, 0, fake, fake, 1, 9 * 128 * 2, None) < 0
    assert "table_dtype" in err()
    assert lib.gmz_conv3x3_forward_stamp(1, 15, fake, fake, fake, 8, None, None, 0, fake, fake, 0, 9 * 128 * 2, None) < 0
    assert "4608" in err()
    # weight-gradient partials
    need = ctypes.c_size_t()
    assert lib.gmz_conv3x3_wgrad_workspace_bytes(360, ctypes.byref(need)) == 0
    assert lib.gmz_conv3x3_wgrad(1, 15, fake, fake, 360, fake, 1, 1, 1, 1, 1, fake, need.value - 4, None) < 0
    assert "workspace" in err()
    # BatchNorm workspaces and statistics partials
    assert lib.gmz_bn_workspace_bytes(1, 360, 128, 225, ctypes.byref(need)) == 0
    assert lib.gmz_bn_forward(1, 1, fake, None, None, 360, 128, 225, fake, fake, 1e-4, 0.1, None, None, None, 1, fake,
                              fake, fake, need.value - 8, None) < 0
    assert "workspace" in err()
    assert lib.gmz_bn_forward_stats(1, fake, None, 360, 128, 225, fake, fake, 1e-4, 0.1, None, None, None, 1, fake, fake,
                                    fake, ns.value, 128 * ns.value * 24 - 8, None) < 0
    assert "partials" in err()
    assert lib.gmz_bn_backward_stats(1, fake, fake, fake, None, 360, 128, 225, fake, fake, 1, fake, None, fake, fake,
                                     fake, ns.value, 128 * ns.value * 24, fake, need.value - 8, None, 0) < 0
    assert "workspace" in err()
    assert lib.gmz_head_conv1x1_workspace_bytes(360 * 225, 3, ctypes.byref(need)) == 0
    assert lib.gmz_head_conv1x1_backward(1, fake, 360 * 225, 128, fake, 2, fake, 1, fake, fake, fake, None, None, None,
                                         None, 0, fake, need.value - 4, None) < 0
    assert "workspace" in err()
    assert lib.gmz_seg_bn_forward(1, fake, None, 5, 360, 1, 512, fake, fake, 1e-4, fake, fake, 4 * (3 * 5 * 512 + 5) - 4,
                                  0, 0.1, None, None, None, None, None) < 0
    assert "stats" in err()
    # the network's scratch (reward split-K partials, head features)
    w = network.NetWeights()
    w.board_size, w.channels, w.blocks, w.head_hidden, w.dtype = 15, 128, 8, 64, 0
    assert lib.gmz_net_workspace_bytes(ctypes.byref(w), 512, ctypes.byref(need)) == 0
    assert lib.gmz_net_recurrent_tower(ctypes.byref(w), fake, fake, fake, fake, 512, fake, need.value - 1, None) < 0
    assert "gmz_net_workspace_bytes" in err()
    assert lib.gmz_net_initial_heads(ctypes.byref(w), fake, fake, 512, fake, fake, fake, need.value - 1, None) < 0
    assert "workspace" in err()


def test_round6_entry_points_check_before_launching():
    """The round-6 additions keep the same contract: the fused optimiser's workspace and gradient alignment, the
    deferred BatchNorm's statistics partials, the BatchNorm-apply conv's slots and aliasing — all refused before
    any launch (fake pointers, no GPU)."""
    import ctypes
    import datou_gomoku_muzero_amd._lib as L
    lib = L.load()
    fake = ctypes.c_void_p(1 << 20)
    err = lambda: lib.gmz_last_error().decode()  # noqa: E731
    ib, ch, wsb = ctypes.c_size_t(), ctypes.c_int(), ctypes.c_size_t()
    assert lib.gmz_opt_layout(ctypes.byref(ib), ctypes.byref(ch), ctypes.byref(wsb)) == 0
    assert ib.value == 32 and ch.value > 0 and wsb.value > 0
    assert lib.gmz_opt_step(fake, 4, fake, fake, fake, 1000, None, 1, 5.0, fake, 0.9, 0.999, 1e-8, 1e-5, 0.995, fake,
                            fake, fake, wsb.value - 1, None) < 0
    assert "workspace" in err()
    assert lib.gmz_opt_step(fake, 4, ctypes.c_void_p((1 << 20) + 4), fake, fake, 1000, None, 1, 5.0, fake, 0.9, 0.999,
                            1e-8, 1e-5, 0.995, fake, fake, fake, wsb.value, None) < 0
    assert "aligned" in err()
    ns = ctypes.c_int()
    assert lib.gmz_conv3x3_stats_slots(360, ctypes.byref(ns)) == 0
    assert lib.gmz_bn_forward_deferred(1, fake, None, 360, 128, 225, 1e-4, 0.1, None, None, None, fake, fake, ns.value,
                                       128 * ns.value * 24 - 8, None, 0, None) < 0
    assert "partials" in err()
    assert lib.gmz_bn_forward_deferred(1, fake, None, 360, 128, 225, 1e-4, 0.1, None, None, None, fake, None, 0, 0, fake,
                                       8, None) < 0
    assert "workspace" in err()
    assert lib.gmz_conv3x3_forward_bnapply(1, 15, fake, None, fake, fake, fake, 1, fake, fake, fake, 360, None, fake,
                                           ns.value - 1, None) < 0
    assert "slots" in err()
    assert lib.gmz_conv3x3_forward_bnapply(1, 15, fake, None, fake, fake, fake, 1, fake, fake,
                                           ctypes.c_void_p((1 << 20) + 4096), 360, None, None, 0, None) < 0
    assert "alias" in err()
    assert lib.gmz_comm_stamp(fake, 3, None) < 0 and "phase" in err()
    # the batched conv-weight re-pack: its job record is the trainer's numpy layout; empty tables and bad dtypes refused
    jb = ctypes.c_size_t()
    assert lib.gmz_conv3x3_pack_job_bytes(ctypes.byref(jb)) == 0 and jb.value == 56
    assert lib.gmz_conv3x3_pack_many(1, fake, 0, None) < 0 and "n_jobs" in err()
    assert lib.gmz_conv3x3_pack_many(3, fake, 2, None) < 0 and "dtype" in err()
