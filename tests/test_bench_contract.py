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


def test_spawn_ranks_sets_the_distributed_env(tmp_path):
    """bench.py --gpus N without an external launcher: spawn_ranks starts N processes with the
    torch.distributed env contract; they rendezvous (gloo here) and see world_size N."""
    import bench
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, sys, torch, torch.distributed as dist\n"
        "dist.init_process_group('gloo', init_method='env://')\n"
        "t = torch.ones(1)\n"
        "dist.all_reduce(t)\n"
        "open(os.path.join(sys.argv[1], 'r%s' % os.environ['RANK']), 'w').write(\n"
        "    '%d %d %s %d' % (dist.get_rank(), dist.get_world_size(), os.environ['LOCAL_RANK'], int(t.item())))\n"
        "dist.destroy_process_group()\n")
    assert bench.spawn_ranks(2, [str(tmp_path)], script=str(script)) == 0
    for r in range(2):
        assert (tmp_path / ("r%d" % r)).read_text() == "%d 2 %d 2" % (r, r)


def test_spawn_ranks_reports_a_failing_rank(tmp_path):
    import bench
    script = tmp_path / "fail.py"
    script.write_text("import os, sys, time\n"
                      "sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(30)\n")
    assert bench.spawn_ranks(2, [], script=str(script)) == 3  # rank 0 is terminated, not waited for


def test_gpus_must_match_world_size():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "disagrees" in p.stderr


def test_timer_stats_union_of_launch_intervals():
    """busy time = union of the launch intervals of all streams' timers; mean = per launch."""
    import bench

    class Ev:
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

    class T:
        def __init__(self, iv):
            self.pairs = [[Ev(a), Ev(b), 0] for a, b in iv]
    base = Ev(0.0)
    n, mean, busy = bench.timer_stats([T([(0, 2), (5, 6)]), T([(1, 3), (6.5, 7), (10, 10.5)])], base)
    assert n == 5
    assert abs(mean - (2 + 1 + 2 + 0.5 + 0.5) / 5) < 1e-12
    assert abs(busy - (3 + 1 + 0.5 + 0.5)) < 1e-12
    assert bench.timer_stats([], base) == (0, 0.0, 0.0)


def test_pmc_traffic_matches_the_resolved_stream_count():
    """roofline.traffic comes from the committed PMC pass only when that pass measured this
    configuration: C2 with the number of streams the run resolved to (the default two for C2, which
    the command line leaves unset)."""
    import json
    import bench
    pm = json.load(open(os.path.join(REPO, "profiles", "pmc_tower_latest.json")))

    class A:
        size, blocks, precision, streams = 15, 8, pm["precision"], None
    path = os.path.join(REPO, "profiles", "pmc_tower_latest.json")
    assert bench.pmc_traffic(path, A, 1024, False, int(pm["streams"])) == pm["hbm_bytes_per_launch"]
    assert bench.pmc_traffic(path, A, 1024, False, int(pm["streams"]) + 1) is None
    assert bench.pmc_traffic(path, A, 2048, False, int(pm["streams"])) is None
    assert bench.pmc_traffic(path, A, 1024, True, int(pm["streams"])) is None


def _rank_share(rank, world, port, out):
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    class P:  # both ranks report the same device (the one-card rehearsal)
        pci_domain_id, pci_bus_id, pci_device_id = 0, 3, 0
    torch.cuda.get_device_properties = lambda i: P
    torch.cuda.current_device = lambda: 0
    out[rank] = bench.ranks_per_gpu(dist)
    dist.destroy_process_group()


def test_ranks_per_gpu_counts_ranks_sharing_a_device():
    import bench
    assert bench.ranks_per_gpu(None) == 1
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank_share, args=(2, _free_port(), out), nprocs=2, join=True)
    assert out[0] == out[1] == 2


_PHASE_CHILD = r'''
import json, os, sys, time
phase, rank = os.environ["GMZ_BENCH_PHASE"], int(os.environ.get("RANK", "0"))
assert "TORCHELASTIC_USE_AGENT_STORE" not in os.environ
frag = {"selfplay": {"metric": "m", "value": 10.0 + rank, "port": os.environ.get("MASTER_PORT")},
        "extras": {"sublines": {"c1": {"value": 1.0}}, "worker": {"value": 2.0}},
        "trainer": {"trainer": {"value": 3.0}}, "loop": {"loop_c4": {"moves_per_s": 4.0}}}[phase]
if phase == "trainer" and rank == 1:
    sys.exit(3)                      # a rank whose phase fails
if phase == "trainer" and rank == 0 and os.environ.get("WORLD_SIZE") == "2":
    time.sleep(120)                  # its peer, stuck in a collective: stopped by the failure flag
if phase == "loop" and rank == 1:
    time.sleep(120)                  # a hang: stopped by the phase's wall-time cap
if rank == 0:
    print("GMZ_PHASE_RESULT " + json.dumps(frag), flush=True)
'''

_PHASE_PARENT = r'''
import os, sys
sys.path.insert(0, %r)
import bench
import torch.distributed as d
_init = d.init_process_group


def init(*a, **k):  # as under torch.distributed.run: the agent's store flag is in the rank's env
    _init(*a, **k)
    os.environ["TORCHELASTIC_USE_AGENT_STORE"] = "True"


d.init_process_group = init
argv = ["--gpus", "2", "--phase-timeout-loop", "6", "--sublines", "c1", "--worker-moves", "1"]
if "RANK" not in os.environ:
    sys.exit(bench.spawn_ranks(2, [], script=os.path.abspath(__file__)))
args = bench.parse(argv)
sys.exit(bench.orchestrate(args, argv, int(os.environ["RANK"]), 2, script=%r))
'''


def test_isolated_phases_keep_the_headline_when_a_later_phase_fails(tmp_path):
    """bench.orchestrate (N > 1): every phase runs as fresh rank processes; a rank whose trainer phase
    exits non-zero stops its peer (store flag) long before that peer's sleep ends, a hanging loop phase is
    killed at its cap, and rank 0 still prints ONE line: the headline intact, {"error": ...} in the keys
    of the failed phases, the extras merged."""
    import json
    import subprocess
    import time
    child = tmp_path / "child.py"
    child.write_text(_PHASE_CHILD)
    parent = tmp_path / "parent.py"
    parent.write_text(_PHASE_PARENT % (REPO, str(child)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    t0 = time.time()
    p = subprocess.Popen([sys.executable, str(parent)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=200)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 9)  # this test's own process group (the spawned ranks with it)
            p.communicate()
    p.stdout, p.stderr = out, err
    took = time.time() - t0
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["value"] == 10.0 and d["metric"] == "m"
    assert d["sublines"] == {"c1": {"value": 1.0}} and d["worker"] == {"value": 2.0}
    assert "error" in d["trainer"] and "rank 1 exit 3" in d["trainer"]["error"]
    assert "error" in d["loop_c4"] and "timeout" in d["loop_c4"]["error"]
    ranks = d["phases"]["detail"]["trainer"]["ranks"]
    assert ranks[0]["status"].startswith("stopped") and ranks[0]["seconds"] < 60
    assert took < 150


def test_isolated_phases_under_torch_distributed_run(tmp_path):
    """The driver's N > 1 launch: `python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1`
    makes the rank processes (their process group on the launcher's agent store,
    TORCHELASTIC_USE_AGENT_STORE set); bench.orchestrate's phase processes then host their own stores on new
    ports.  Scripted phase processes as above: the one line carries the headline and the phases' errors."""
    import json
    import subprocess
    import time
    child = tmp_path / "child.py"
    child.write_text(_PHASE_CHILD)
    parent = tmp_path / "parent_run.py"
    parent.write_text("import os, sys\nsys.path.insert(0, %r)\nimport bench\n"
                      "argv = ['--gpus', '2', '--phase-timeout-loop', '6', '--sublines', 'c1', '--worker-moves', '1']\n"
                      "assert os.environ.get('TORCHELASTIC_USE_AGENT_STORE') == 'True'\n"
                      "sys.exit(bench.orchestrate(bench.parse(argv), argv, int(os.environ['RANK']), 2, script=%r))\n"
                      % (REPO, str(child)))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    p = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(parent)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    t0 = time.time()
    try:
        out, err = p.communicate(timeout=240)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 9)  # this test's own process group
            out, err = p.communicate()
    assert p.returncode == 0, err[-3000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    assert d["value"] == 10.0 and "error" in d["trainer"] and "error" in d["loop_c4"]
    assert d["sublines"] == {"c1": {"value": 1.0}}
    assert time.time() - t0 < 200


def test_isolated_phases_with_one_gpu(tmp_path, capsys):
    """bench.py --isolate on at N = 1: the phases run one after another as single fresh processes (no
    process group); the line is assembled the same way (here rank 0's trainer phase succeeds)."""
    import json
    import bench
    child = tmp_path / "child.py"
    child.write_text(_PHASE_CHILD)
    argv = ["--gpus", "1", "--isolate", "on", "--sublines", "c1", "--worker-moves", "1", "--loop-iters", "0",
            "--no-cpu-baseline"]
    for k in ("WORLD_SIZE", "RANK"):
        os.environ.pop(k, None)
    assert bench.orchestrate(bench.parse(argv), argv, 0, 1, script=str(child)) == 0
    d = json.loads([l for l in capsys.readouterr().out.splitlines() if l.startswith("{")][-1])
    assert d["value"] == 10.0 and d["trainer"] == {"value": 3.0} and "loop_c4" not in d
    assert set(d["phases"]["detail"]) == {"selfplay", "extras", "trainer"}


_PHASE_CHILD_8 = r'''
import json, os, sys, time
phase, rank = os.environ["GMZ_BENCH_PHASE"], int(os.environ.get("RANK", "0"))
world = int(os.environ.get("WORLD_SIZE", "1"))
frag = {"selfplay": {"metric": "m", "value": 100.0, "world": world},
        "extras": {"sublines": {"c1": {"value": 1.0}}, "worker": {"value": 2.0}},
        "trainer": {"trainer": {"value": 3.0}}, "loop": {"loop_c4": {"moves_per_s": 4.0}}}[phase]
hang, fail = os.environ.get("T_HANG", ""), os.environ.get("T_FAIL", "")
if hang == "%s:%d" % (phase, rank):
    time.sleep(300)                  # a rank stuck in the phase: killed at the (deadline-shrunk) cap
if fail == "%s:%d" % (phase, rank):
    sys.exit(3)                      # a rank whose phase fails
if fail.startswith(phase + ":"):
    time.sleep(300)                  # its peers, waiting in a collective: stopped by the failure flag
if rank == 0:
    print("GMZ_PHASE_RESULT " + json.dumps(frag), flush=True)
'''

_PHASE_PARENT_N = r'''
import os, sys
sys.path.insert(0, %r)
import bench
N = %d
argv = %r
if "RANK" not in os.environ:
    sys.exit(bench.spawn_ranks(N, [], script=os.path.abspath(__file__)))
args = bench.parse(argv)
sys.exit(bench.orchestrate(args, argv, int(os.environ["RANK"]), N, script=%r))
'''


def _run_orchestrated(tmp_path, n, argv, hang, fail, timeout):
    import json
    import subprocess
    import time
    child = tmp_path / "child8.py"
    child.write_text(_PHASE_CHILD_8)
    parent = tmp_path / ("parent%d.py" % n)
    parent.write_text(_PHASE_PARENT_N % (REPO, n, argv, str(child)))
    env = dict(os.environ, T_HANG=hang, T_FAIL=fail)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    t0 = time.time()
    p = subprocess.Popen([sys.executable, str(parent)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    finally:
        if p.poll() is None:
            os.killpg(p.pid, 9)  # this test's own process group (the spawned ranks and phases with it)
            out, err = p.communicate()
    assert p.returncode == 0, err[-3000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0]), time.time() - t0


def test_eight_rank_orchestration_inside_the_deadline(tmp_path):
    """the driver's first N = 8 line.  Eight rank processes (gloo), scripted phases: rank 3
    hangs in the trainer phase (killed at its cap), rank 5 fails in the loop phase (its seven peers, stuck in
    a collective, are stopped by the store flag).  The one line arrives inside --deadline with the headline
    of all 8 ranks' phase intact, the extras merged, and `phases` naming both failures."""
    argv = ["--gpus", "8", "--deadline", "90", "--phase-timeout-trainer", "8", "--sublines", "c1",
            "--worker-moves", "1"]
    d, took = _run_orchestrated(tmp_path, 8, argv, "trainer:3", "loop:5", 200)
    assert d["value"] == 100.0 and d["world"] == 8
    assert d["sublines"] == {"c1": {"value": 1.0}} and d["worker"] == {"value": 2.0}
    det = d["phases"]["detail"]
    assert len(det["selfplay"]["ranks"]) == 8 and all(r["status"] == "ok" for r in det["selfplay"]["ranks"])
    assert det["trainer"]["ranks"][3]["status"].startswith("timeout")
    assert "error" in d["trainer"] and "rank 3 timeout" in d["trainer"]["error"]
    assert det["loop"]["ranks"][5]["status"] == "exit 3"
    assert all(r["status"].startswith("stopped") for i, r in enumerate(det["loop"]["ranks"]) if i != 5)
    assert "error" in d["loop_c4"] and "rank 5 exit 3" in d["loop_c4"]["error"]
    assert all(p["cap_s"] <= 90 for p in det.values())  # each cap = at most what the deadline had left
    assert d["phases"]["seconds"] <= 90 and took < 120


def test_deadline_shrinks_a_later_phase_and_skips_the_rest(tmp_path):
    """--deadline: a hung trainer phase is killed at what the deadline leaves (not its own 150 s cap), and the
    loop phase, with less than 15 s left, is skipped with an error in its keys; the line still arrives in time."""
    argv = ["--gpus", "2", "--deadline", "32", "--sublines", "c1", "--worker-moves", "1"]
    d, took = _run_orchestrated(tmp_path, 2, argv, "trainer:1", "", 120)
    det = d["phases"]["detail"]
    assert d["value"] == 100.0
    assert det["trainer"]["cap_s"] < 32 and det["trainer"]["ranks"][1]["status"].startswith("timeout")
    assert det["loop"]["ranks"][0]["status"].startswith("skipped") and "skipped" in d["loop_c4"]["error"]
    assert d["phases"]["seconds"] <= 32 + 5 and took < 60
