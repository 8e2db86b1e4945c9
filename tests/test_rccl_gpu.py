"""RCCL (torch.distributed "nccl" backend) on the GPU box, world size 1.

The box has one GPU and RCCL refuses two ranks on one device, so the N > 1 exchanges run here over
gloo (tests/test_loop.py, test_trainer.py, test_pipeline_gpu.py) and RCCL itself only on the driver's
8-GPU node.  This test runs the RCCL calls the product makes, on real device tensors, with one rank:
  * the weight push (weight_sync.broadcast_state_dict, workers.py:587-593's ModelWeightsUpdate);
  * the small SUM / MAX all-reduces of the sharded PER and of the bench's max-over-ranks timing
    (trainer._allreduce, bench.collective_max);
  * the DDP trainer (trainer.Trainer under an initialised process group: rank 0's weights broadcast at
    construction, then per step the two gradient buckets' all-reduces captured inside the step's HIP
    graph, timed by the in-graph communication clock; and the fallback with the all-reduces between three
    graphs) — equal to the single-process trainer's steps (same kernels; an all-reduce over one rank
    leaves the bucket unchanged).
It runs in a child process so that no process group outlives it."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r"""
    import os, sys, socket
    sys.path.insert(0, sys.argv[1])
    import numpy as np, torch
    import torch.distributed as dist
    torch.backends.cudnn.deterministic = True
    torch.cuda.set_device(0)
    from datou_gomoku_muzero_amd import trainer as T, weights as W
    from datou_gomoku_muzero_amd.weight_sync import broadcast_state_dict
    import bench

    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)
    batches = []
    for i in range(3):
        obs, act, rew, pol, val = W.synthetic_slices(32, 9, cfg.NUM_UNROLL_STEPS, np.random.RandomState(11 + i))
        bt = [torch.as_tensor(x).cuda() for x in (obs, act, rew, pol, val)]
        bt[0] = bt[0].float()
        batches.append(bt)
    w = torch.rand(32, device="cuda") + 0.5

    def run():
        torch.manual_seed(0)
        tr = T.Trainer(cfg, device="cuda", graph_warmup=2)
        logs = [tr.step(batches[i % 3], w, k=i % 4, flip=bool(i % 2))[0] for i in range(5)]
        assert tr._graphs is not None
        return tr, np.array(logs), torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu().numpy()

    tr0, l0, p0 = run()  # no process group: the single-process trainer
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    tr1, l1, p1 = run()  # DDP path: init broadcast + flat-bucket all-reduce per step over RCCL
    assert tr1.dist is not None and tr1.graph_allreduce  # the all-reduces are inside the captured step
    t = tr1.allreduce_times()  # the in-graph communication clock (gmz_comm_stamp): every step stamped
    assert t is not None and t["steps"] == 5 and t["flush_ms"] > 0 and t["wait_ms"] >= 0, t
    print("allreduce_times", t)
    T.GRAPH_ALLREDUCE = False  # the fallback: three graphs, the all-reduces issued between their replays
    tr2, l2, p2 = run()
    T.GRAPH_ALLREDUCE = True
    assert not tr2.graph_allreduce and isinstance(tr2._graphs, tuple)
    assert np.array_equal(l0, l2) and np.array_equal(p0, p2)
    t2 = tr2.allreduce_times()
    assert t2 is not None and t2["steps"] == 5, t2
    assert np.array_equal(l0, l1), (l0, l1)
    assert np.array_equal(p0, p1)
    # the weight push: one flat fp32 broadcast of the trainer's state_dict
    sd = tr1.state_dict_cpu()
    out = broadcast_state_dict(sd, src=0, device="cuda")
    assert set(out) == set(sd)
    for k in sd:
        assert np.array_equal(out[k].cpu().numpy(), np.asarray(sd[k], dtype=np.float32)), k
    # PER / timing all-reduces on device tensors
    t = torch.tensor([3.5], device="cuda")
    assert float(T._allreduce(t.clone(), dist)[0]) == 3.5
    assert float(T._allreduce(t.clone(), dist, max_op=True)[0]) == 3.5
    assert bench.collective_max(2.25, dist, "nccl") == 2.25 and bench.collective_sum(2.0, dist, "nccl") == 2.0
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok")
""")


def test_rccl_world_one_trainer_weight_push_and_allreduces():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, REPO], capture_output=True, text=True, timeout=240, env=env,
                       cwd=REPO)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "rccl ok" in r.stdout
    print([ln for ln in r.stdout.splitlines() if ln.startswith("allreduce_times")])
