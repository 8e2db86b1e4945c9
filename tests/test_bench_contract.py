"""bench.py's multi-process path on CPU (gloo, world_size 2) and its JSON contract."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import REPO

sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, out):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dt = 1.0 + rank  # rank 1 is the slow one
    out[rank] = bench.collective_max(dt, dist, backend="gloo")
    dist.destroy_process_group()


def test_max_over_ranks_gloo_world2():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] == out[1] == 2.0


def test_result_line_schema():
    import bench

    class A:
        steps, warmup, size, sims, mode, blocks = 10, 2, 15, 400, "MuZero", 8
    line = bench.result_line(A, world=8, dt=2.0, waves=1000, G=1024)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line
    assert line["value"] == 8 * 1024 * 10 / 2.0 and line["scaling"] == "weak" and line["n_gpus"] == 8
    assert "workload" in line["config"] and "model" not in line["config"]
