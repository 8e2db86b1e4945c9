"""Graph capture of the trainer step beside another thread's HIP event queries.

With a process group, RCCL's watchdog thread queries its work events at any time.  In PyTorch's default GLOBAL
capture mode such a query from another thread while a stream is capturing is refused by HIP ("operation not
permitted when stream is capturing") — one full GPU suite of round 5 died of exactly that race
(profiles/r05_rccl_capture_race.txt).  trainer.Trainer._capture therefore captures in THREAD-LOCAL mode whenever a
process group exists.  This test provokes the race on purpose: a second thread polls ``torch.cuda.Event.query()``
in a tight loop on an event of the same device for the whole time the trainer (world-1 RCCL process group)
captures and replays its step graphs.  Pass = no error in either thread, the graphs were captured, and the steps
equal the single-process trainer's (tests/test_rccl_gpu.py's comparison).  It runs in a child process so that no
process group (or a failed capture) outlives it."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent(r"""
    import os, sys, socket, threading, time
    sys.path.insert(0, sys.argv[1])
    import numpy as np, torch
    import torch.distributed as dist
    torch.backends.cudnn.deterministic = True
    torch.cuda.set_device(0)
    from datou_gomoku_muzero_amd import trainer as T, weights as W

    cfg = T.TrainConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2, PHYSICAL_BATCH_SIZE=32, LEARNING_RATE=1e-3)
    batches = []
    for i in range(3):
        obs, act, rew, pol, val = W.synthetic_slices(32, 9, cfg.NUM_UNROLL_STEPS, np.random.RandomState(21 + i))
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

    _, l0, p0 = run()  # no process group, no poller: the reference steps
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)

    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        torch.ones(1, device="cuda").add_(1)
        ev.record(side)
    stop, errors, polls = threading.Event(), [], [0]

    def poll():  # what RCCL's watchdog does: query device events from another thread, at any time
        try:
            while not stop.is_set():
                ev.query()
                polls[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = threading.Thread(target=poll, daemon=True)
    th.start()
    time.sleep(0.05)
    try:
        tr1, l1, p1 = run()  # captures its graphs (thread-local mode: a process group exists) while poll() runs
    finally:
        stop.set()
        th.join(timeout=30)
    assert not errors, errors
    assert polls[0] > 1000, polls[0]
    assert tr1._graphs is not None and tr1.graph_allreduce
    assert np.array_equal(l0, l1), (l0, l1)
    assert np.array_equal(p0, p1)
    dist.barrier()
    dist.destroy_process_group()
    print("capture race ok, %d event queries during the run" % polls[0])
""")


def test_trainer_capture_beside_an_event_polling_thread():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, REPO], capture_output=True, text=True, timeout=240, env=env,
                       cwd=REPO)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "capture race ok" in r.stdout
    print(r.stdout.strip().splitlines()[-1])
