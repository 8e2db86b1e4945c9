"""Loader for libgmz.so (the HIP kernels + C ABI of include/gmz.h).

The product path has NO fallback: if the shared library is missing or was built for another
ABI, importing this module raises.  ``torch`` is imported first so that libgmz.so binds to the
same HIP runtime (soname libamdhip64.so.7) that torch's allocator and streams use.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GMZ_LIB") or os.path.join(PKG_DIR, "libgmz.so")  # GMZ_LIB: A/B builds (tools)
ABI_VERSION = 10

P = ctypes.c_void_p
I = ctypes.c_int
L = ctypes.c_long
U64 = ctypes.c_uint64
SZ = ctypes.c_size_t  # capacity arguments (ABI 10): a buffer's size in bytes


class EngineCfg(ctypes.Structure):
    _fields_ = [("num_games", ctypes.c_int32), ("board_size", ctypes.c_int32), ("n_in_row", ctypes.c_int32),
                ("num_simulations", ctypes.c_int32), ("num_top_actions", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("c_visit", ctypes.c_int32), ("flags", ctypes.c_int32), ("c_scale", ctypes.c_double),
                ("minmax_delta", ctypes.c_double), ("discount", ctypes.c_double), ("game_offset", ctypes.c_int32)]


_SIGS = {
    "gmz_last_error": ([], ctypes.c_char_p),
    "gmz_abi_version": ([], I),
    "gmz_device_synchronize": ([], I),
    "gmz_game_check_win": ([P, I, I, I, P, P, P], I),
    "gmz_game_board_state": ([P, I, I, P, P, P, P], I),
    "gmz_game_play": ([P, I, I, I, P, P, P, P, P, P], I),
    "gmz_game_winning_scan": ([P, P, P, I, I, I, P, P, P, P], I),
    "gmz_engine_create": ([ctypes.POINTER(EngineCfg), ctypes.POINTER(P)], I),
    "gmz_engine_destroy": ([P], I),
    "gmz_engine_game_state": ([P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P)], I),
    "gmz_engine_copy_state": ([P, I, P, P, P, P, P], I),
    "gmz_engine_reset_games": ([P, P, P], I),
    "gmz_engine_begin_move": ([P, P, U64, P, P], I),
    "gmz_engine_set_root": ([P, P, P, P], I),
    "gmz_engine_select": ([P, P, P, P, P, P], I),
    "gmz_engine_expand_backup": ([P, P, P, P, P], I),
    "gmz_engine_expand_backup_select": ([P, P, P, P, P, P, P, P, P], I),
    "gmz_engine_pending_waves": ([P, P], I),
    "gmz_engine_waves_for_legal": ([ctypes.POINTER(EngineCfg), P, I, P], I),
    "gmz_engine_finish_move": ([P, P, P, P, P], I),
    "gmz_engine_play": ([P, P, P, I, P], I),
    "gmz_engine_root_stats": ([P, P, P, P, P, P, P], I),
    "gmz_engine_max_visited_children": ([P, P], I),
    "gmz_engine_wave_k": ([P, P, P], I),
    "gmz_engine_wave_depth": ([P, P, P], I),
    "gmz_engine_tree_counters": ([P, P, I, P], I),
    "gmz_engine_set_hidden_bases": ([P, P, P], I),
    "gmz_engine_set_hidden_budget": ([P, P, P], I),
    "gmz_engine_errors": ([P, ctypes.POINTER(ctypes.c_int32), I], I),
    "gmz_engine_errors_async": ([P, P, P], I),
    "gmz_hashnet_initial": ([P, I, I, P, P, P, P, P], I),
    "gmz_hashnet_recurrent": ([P, P, P, P, I, I, P, P, P, P], I),
    "gmz_bn_workspace_bytes": ([I, I, I, I, ctypes.POINTER(ctypes.c_size_t)], I),
    "gmz_bn_forward": ([I, I, P, P, P, I, I, I, P, P, ctypes.c_float, ctypes.c_float, P, P, P, I, P, P, P, SZ, P], I),
    "gmz_bn_backward": ([I, I, P, P, P, P, I, I, I, P, P, I, P, P, P, P, P, SZ, P], I),
    "gmz_bn_backward_acc": ([I, I, P, P, P, P, I, I, I, P, P, I, P, P, P, P, P, SZ, P, I], I),
    "gmz_bn_eval": ([I, I, P, P, I, I, I, P, P, P, P, ctypes.c_float, I, P, P, SZ, P], I),
    "gmz_conv3x3_pack": ([I, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, I, P, P], I),
    "gmz_conv3x3_forward": ([I, I, P, P, P, I, P], I),
    "gmz_conv3x3_pack_job_bytes": ([ctypes.POINTER(SZ)], I),
    "gmz_conv3x3_pack_many": ([I, P, I, P], I),
    "gmz_conv3x3_forward_add": ([I, I, P, P, P, P, I, P], I),
    "gmz_conv3x3_stats_slots": ([I, ctypes.POINTER(ctypes.c_int)], I),
    "gmz_conv3x3_wgrad_workspace_bytes": ([I, ctypes.POINTER(ctypes.c_size_t)], I),
    "gmz_conv3x3_wgrad": ([I, I, P, P, I, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, I, P, SZ, P],
                          I),
    "gmz_conv3x3_wgrad_segments": ([I, I, P, P, I, I, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                    I, P, SZ, P], I),
    "gmz_conv3x3_forward_stats": ([I, I, P, P, P, I, P, P, I, P], I),
    "gmz_conv3x3_forward_bwdstats": ([I, I, P, P, P, P, I, P, P, P, P, I, P, I, P], I),
    "gmz_bn_backward_stats": ([I, P, P, P, P, I, I, I, P, P, I, P, P, P, P, P, I, SZ, P, SZ, P, I], I),
    "gmz_grad_add_t": ([I, P, I, I, I, P, P], I),
    "gmz_grad_add_t_cols": ([I, P, I, I, I, I, I, P, P], I),
    "gmz_comm_stamp": ([P, I, P], I),
    "gmz_opt_layout": ([ctypes.POINTER(SZ), ctypes.POINTER(I), ctypes.POINTER(SZ)], I),
    "gmz_opt_step": ([P, I, P, P, P, ctypes.c_longlong, P, I, ctypes.c_float, P, ctypes.c_float, ctypes.c_float,
                      ctypes.c_float, ctypes.c_float, ctypes.c_float, P, P, P, SZ, P], I),
    "gmz_head_conv1x1_forward": ([I, P, L, I, P, P, I, P, P, I, P, P, P], I),
    "gmz_head_conv1x1_workspace_bytes": ([L, I, P], I),
    "gmz_seg_bn_forward": ([I, P, P, I, I, I, I, P, P, ctypes.c_float, P, P, SZ, I, ctypes.c_float, P, P, P, P, P], I),
    "gmz_seg_bn_backward": ([I, P, P, P, I, I, I, I, P, P, SZ, P, P, P, I, P], I),
    "gmz_seg_bn_small_workspace_bytes": ([I, I, ctypes.POINTER(SZ)], I),
    "gmz_seg_bn_forward_small": ([I, P, P, I, I, I, I, P, P, ctypes.c_float, P, P, SZ, I, ctypes.c_float, P, P, P, P, P, SZ,
                                  P], I),
    "gmz_seg_bn_backward_small": ([I, P, P, P, I, I, I, I, P, P, SZ, P, P, P, I, P, SZ, P], I),
    "gmz_head_conv1x1_backward": ([I, P, L, I, P, I, P, I, P, P, P, P, P, P, P, I, P, SZ, P], I),
    "gmz_bn_forward_stats": ([I, P, P, I, I, I, P, P, ctypes.c_float, ctypes.c_float, P, P, P, I, P, P, P, I, SZ, P], I),
    "gmz_bn_forward_seg": ([I, P, P, P, I, I, I, I, P, P, ctypes.c_float, ctypes.c_float, P, P, P, I, P, P, P, SZ, P, SZ,
                            P], I),
    "gmz_conv3x3_forward_board_stats": ([I, I, P, P, P, I, P, P, I, P], I),
    "gmz_conv3x3_forward_stamp": ([I, I, P, P, P, I, P, P, I, P, P, I, SZ, P], I),
    "gmz_conv3x3_forward_bnapply": ([I, I, P, P, P, P, P, I, P, P, P, I, P, P, I, P], I),
    "gmz_bn_forward_deferred": ([I, P, P, I, I, I, ctypes.c_float, ctypes.c_float, P, P, P, P, P, I, SZ, P, SZ, P], I),
    "gmz_bn_forward_m": ([I, I, P, P, P, I, I, I, P, P, ctypes.c_float, ctypes.c_float, P, P, P, I, P, P, P, SZ, P, P], I),
    "gmz_bn_forward_stats_m": ([I, P, P, I, I, I, P, P, ctypes.c_float, ctypes.c_float, P, P, P, I, P, P, P, I, SZ, P, P],
                               I),
    "gmz_bn_backward_acc_m": ([I, I, P, P, P, P, I, I, I, P, P, I, P, P, P, P, P, SZ, P, P, I], I),
}

# symbols added by the network kernels (declared in include/gmz.h too)
_NET_SIGS = {}

_lib = None


class GmzError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GmzError("libgmz.so not built (%s); run __graft_entry__.build() or make -C csrc" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (args, res) in list(_SIGS.items()) + list(_NET_SIGS.items()):
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.gmz_abi_version() != ABI_VERSION:
        raise GmzError("libgmz.so ABI %d != %d" % (lib.gmz_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def register(sigs):
    """Extend the signature table (used by modules that add exported symbols)."""
    _NET_SIGS.update(sigs)
    if _lib is not None:
        for name, (args, res) in sigs.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = res


def check(rc):
    if rc != 0:
        raise GmzError(load().gmz_last_error().decode(errors="replace"))
    return rc


def ptr(t):
    """Device/host pointer of a torch tensor (or None → NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def nbytes(t):
    """Size in bytes of a torch tensor's elements (None → 0): the capacity arguments of ABI 10."""
    return 0 if t is None else t.numel() * t.element_size()


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)
