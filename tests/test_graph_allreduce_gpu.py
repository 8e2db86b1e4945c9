"""The data-parallel trainer's capture decision with two ranks on the box's one GPU (gloo: RCCL refuses two ranks on
one device).  A gloo all-reduce of a device tensor cannot be captured into a HIP graph (it stages through the host), so
``Trainer._graph_collectives_ok`` comes back False on BOTH ranks and both fall back to the three-graph step with the
all-reduces between replays, after which the two ranks (different batches, different initial seeds) hold
bit-identical weights: rank 0's broadcast at construction, then the averaged gradients of every step."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r"""
    import os, sys
    sys.path.insert(0, sys.argv[1])
    rank, port = int(sys.argv[2]), int(sys.argv[3])
    import numpy as np, torch
    import torch.distributed as dist
    torch.backends.cudnn.deterministic = True
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=2)
    from datou_gomoku_muzero_amd import trainer as T, weights as W
    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=16, LEARNING_RATE=1e-3)
    obs, act, rew, pol, val = W.synthetic_slices(16, 9, cfg.NUM_UNROLL_STEPS, np.random.RandomState(40 + rank))
    bt = [torch.as_tensor(x).cuda() for x in (obs, act, rew, pol, val)]
    bt[0] = bt[0].float()
    w = torch.ones(16, device="cuda")
    torch.manual_seed(rank)  # different initial weights: the construction broadcast must make them equal
    print("rank %d: process group up" % rank, flush=True)
    tr = T.Trainer(cfg, device="cuda", graph_warmup=2)
    print("rank %d: trainer built" % rank, flush=True)
    for i in range(4):
        tr.step(bt, w, k=i % 4, flip=bool(i % 2))
        torch.cuda.synchronize()
        print("rank %d: step %d done" % (rank, i), flush=True)
    assert tr._graphs is not None and isinstance(tr._graphs, tuple) and not tr.graph_allreduce
    flat = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()])
    w0, w1 = flat.clone(), flat.clone()
    dist.broadcast(w0, 0)  # the same two collectives on both ranks, in the same order
    dist.broadcast(w1, 1)
    assert torch.equal(w0, w1), float((w0 - w1).abs().max())
    dist.barrier()
    dist.destroy_process_group()
    print("rank %d ok: split graphs, replicas identical" % rank, flush=True)
""")


def test_two_gloo_ranks_fall_back_to_split_graphs_together():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    # the children print their progress straight to this process's stdout (a stall shows where it stopped)
    procs = [subprocess.Popen([sys.executable, "-u", "-c", SCRIPT, REPO, str(r), str(port)], env=env, cwd=REPO)
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert rcs == [0, 0], rcs
