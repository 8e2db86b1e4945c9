"""weight_sync.broadcast_state_dict with world_size 2 over gloo on the CPU."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from datou_gomoku_muzero_amd import weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    from datou_gomoku_muzero_amd.weight_sync import broadcast_state_dict
    cfg = GmzConfig(BOARD_SIZE=6, NUM_RES_BLOCKS=1)
    sd = W.synthetic_state_dict(cfg, seed=11 if rank == 0 else 99, with_projection=False)
    out = broadcast_state_dict(sd, src=0, device="cpu")
    ref = W.synthetic_state_dict(cfg, seed=11, with_projection=False)
    ok = sorted(out) == sorted(ref) and all(
        np.array_equal(out[k].numpy(), np.asarray(ref[k], np.float32)) for k in ref)
    q.put((rank, ok))
    dist.destroy_process_group()


def test_broadcast_state_dict_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
