"""Generate golden fixtures by running the REFERENCE's own Python code (this container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only NAME]

Imports /root/reference (read-only; never needed at test time — the outputs below are committed
as small .npz files).  workers.py needs ``torch.utils.tensorboard`` and ``seaborn`` (visualiser-only,
absent here) — they are stubbed with empty modules, as SURVEY.md §8c prescribes.

Fixtures written to tests/golden/:
  game_cases.npz       game.py: do_move / check_win / get_game_ended / get_board_state / legal set
  mcts_<name>.npz      mcts.py: MuZeroMCTS / AlphaZeroMCTS.search driven by HashNet (oracle/hashnet.py)
                       through an inference-server-shaped queue (workers.py:344-369 return types)
  winmoves.npz         workers.py:49-123 find_winning_moves_rebuilt on the 4 test patterns + random boards
  worker_record.npz    workers.py:162-237 universal_worker: GameRecord + TrainingSlices for a scripted game
  net_small.npz        network.py GomokuNetEZ forward (9x9, C=32, 2 blocks) from weights.synthetic_state_dict
  net_c15.npz          network.py GomokuNetEZ forward at 15x15, C=128, 8 blocks (2 rows + summaries)
"""
import argparse
import os
import sys
import tempfile
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REF)

# --- stubs for visualiser-only deps of workers.py (workers.py:18-19) ---
for name in ("seaborn",):
    sys.modules.setdefault(name, types.ModuleType(name))
_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules.setdefault("torch.utils.tensorboard", _tb)

os.chdir(tempfile.mkdtemp(prefix="gmz_golden_"))  # db_manager.py:33 creates outputs/ in CWD

import torch  # noqa: E402
from queue import Empty  # noqa: E402

import config as ref_config_mod  # noqa: E402
ref_config = ref_config_mod.config
import game as ref_game  # noqa: E402
import mcts as ref_mcts  # noqa: E402
import hashnet  # noqa: E402


def set_board(size):
    ref_config.BOARD_SIZE = size
    ref_config.ACTION_SPACE_SIZE = size * size


# ============================================================ game fixtures
def make_game_cases():
    out = {}
    for size in (6, 9, 15, 19):
        set_board(size)
        rs = np.random.RandomState(100 + size)
        A = size * size
        # (1) random full games: per step board-before, move, check_win, ended, obs planes (u8)
        boards, moves, wins, ended, obs, players, lastm, valid = [], [], [], [], [], [], [], []
        game_idx = []
        for g in range(12):
            game = ref_game.GomokuGame(board_size=size, n_in_row=5)
            # bias moves toward a local region so that wins happen
            while True:
                vm = game.get_valid_moves()
                if not vm:
                    break
                if game.last_move is not None and rs.rand() < 0.7:
                    r0, c0 = game.last_move
                    near = [m for m in vm if abs(m[0] - r0) <= 2 and abs(m[1] - c0) <= 2]
                    cand = near if near else vm
                else:
                    cand = vm
                m = cand[rs.randint(len(cand))]
                mv = int(m[0] * size + m[1])
                boards.append(game.board.reshape(-1).copy())
                players.append(game.current_player)
                lastm.append(-1 if game.last_move is None else game.last_move[0] * size + game.last_move[1])
                o = game.get_board_state(game.current_player, game.last_move)
                obs.append(o.reshape(3, -1).astype(np.uint8))
                vmask = np.zeros(A, np.uint8)
                vmask[[a[0] * size + a[1] for a in vm]] = 1
                valid.append(vmask)
                game.do_move(mv)
                moves.append(mv)
                wins.append(bool(game.check_win()))
                e = game.get_game_ended()
                ended.append(2 if e is None else int(e))
                game_idx.append(g)
                if e is not None:
                    break
        # (2) dense random boards: check_win(move=(r,c)) for every cell
        rb, rw = [], []
        for t in range(24):
            p = [0.2, 0.4, 0.4] if t % 2 == 0 else [0.5, 0.25, 0.25]
            b = rs.choice([0, 1, -1], size=(size, size), p=p).astype(np.int8)
            game = ref_game.GomokuGame(board_size=size, n_in_row=5)
            game.board = b
            w = np.zeros(A, np.uint8)
            for r in range(size):
                for c in range(size):
                    w[r * size + c] = 1 if game.check_win(move=(r, c)) else 0
            rb.append(b.reshape(-1))
            rw.append(w)
        pre = "s%d_" % size
        out[pre + "boards"] = np.array(boards, np.int8)
        out[pre + "moves"] = np.array(moves, np.int32)
        out[pre + "wins"] = np.array(wins, np.uint8)
        out[pre + "ended"] = np.array(ended, np.int8)
        out[pre + "obs"] = np.array(obs, np.uint8)
        out[pre + "players"] = np.array(players, np.int8)
        out[pre + "lastmove"] = np.array(lastm, np.int32)
        out[pre + "valid"] = np.array(valid, np.uint8)
        out[pre + "game"] = np.array(game_idx, np.int32)
        out[pre + "rand_boards"] = np.array(rb, np.int8)
        out[pre + "rand_wins"] = np.array(rw, np.uint8)
        print("game size", size, "steps", len(moves), "wins", int(np.sum(out[pre + "wins"])))
    np.savez_compressed(os.path.join(HERE, "game_cases.npz"), **out)


# ============================================================ MCTS fixtures
class ServerQueue:
    """Synchronous stand-in for the request/result queue pair with the inference server's
    exact return types (workers.py:351-369): initial -> (p f32[A], v np.float32, h[1:...]);
    recurrent_batch -> (p f32[k,A], v f32[k,1], h[k,...], r f32[k,1])."""

    def __init__(self, net):
        self.net, self.results, self.log = net, [], []

    def put(self, item):
        wid, kind, data = item
        self.log.append((kind, 1 if kind == "initial" else len(data[1])))
        if kind == "initial":
            p, v, h = self.net.initial(data[None])
            self.results.append((p[0], v[0, 0], h[0:1]))
        else:
            hs, acts = data
            self.results.append(self.net.recurrent(hs, acts))

    def get(self, timeout=None):
        if not self.results:
            raise Empty()
        return self.results.pop(0)

    def get_nowait(self):
        return self.get()


class Rec:
    roots, stats = [], []


class RecNode(ref_mcts.Node):
    def __init__(self, action=None, parent=None):
        super().__init__(action, parent)
        if parent is None:
            Rec.roots.append(self)


class RecMinMax(ref_mcts.MinMaxStats):
    def __init__(self, d):
        super().__init__(d)
        Rec.stats.append(self)


ref_mcts.Node = RecNode
ref_mcts.MinMaxStats = RecMinMax

_orig_gumbel = np.random.gumbel
_gumbel_log = []


def _rec_gumbel(*a, **k):
    g = _orig_gumbel(*a, **k)
    _gumbel_log.append(np.array(g, dtype=np.float64))
    return g


np.random.gumbel = _rec_gumbel

SCENARIOS = [
    # name, size, mode, sims, np seed, moves, opening stones
    ("mz6_400", 6, "MuZero", 400, 11, 5, 0),      # move 0 exercises the all-children-visited f32 path
    ("az6_50", 6, "AlphaZero", 50, 12, 5, 0),
    ("az9_50", 9, "AlphaZero", 50, 13, 8, 0),      # config 1
    ("mz9_50", 9, "MuZero", 50, 14, 6, 6),
    ("mz15_400", 15, "MuZero", 400, 15, 3, 0),    # config 2 search
    ("mz15_400_mid", 15, "MuZero", 400, 16, 3, 40),
    ("mz15_400_late", 15, "MuZero", 400, 17, 6, 212),  # < 16 legal moves: k < 16 schedule
    ("mz15_15", 15, "MuZero", 15, 18, 10, 20),    # tiny search (tests' NUM_SIMULATIONS=15): ties → set order
    ("az15_15", 15, "AlphaZero", 15, 19, 10, 150),
    ("az15_50_late", 15, "AlphaZero", 50, 20, 8, 200),
    ("mz19_800", 19, "MuZero", 800, 21, 2, 10),   # config 5 search
]


def _opening(game, size, n, rs):
    """Random non-terminal opening: n stones, never completing five (so late-game positions exist)."""
    for _ in range(n):
        vm = game.get_valid_moves()
        order = rs.permutation(len(vm))
        for j in order:
            m = vm[j]
            mv = int(m[0] * size + m[1])
            game.board[m[0], m[1]] = game.current_player
            wins = game.check_win(move=(m[0], m[1]))
            game.board[m[0], m[1]] = 0
            if not wins:
                game.do_move(mv)
                break
        else:
            return False
    return True


def _new_game(size, n_open, rs_open):
    for attempt in range(200):
        game = ref_game.GomokuGame(board_size=size, n_in_row=5)
        if _opening(game, size, n_open, rs_open):
            return game
    raise RuntimeError("no opening")


def make_mcts_case(name, size, mode, sims, seed, n_moves, n_open):
    set_board(size)
    ref_config.NUM_SIMULATIONS = sims
    ref_config.MCTS_IMPLEMENTATION = mode
    A = size * size
    net = hashnet.HashNet(A)
    q = ServerQueue(net)
    cls = ref_mcts.MuZeroMCTS if mode == "MuZero" else ref_mcts.AlphaZeroMCTS
    eng = cls(0, q, q)
    rs_open = np.random.RandomState(seed + 7919)
    game = _new_game(size, n_open, rs_open)
    np.random.seed(seed)
    rec = {k: [] for k in ("board", "player", "lastmove", "movecount", "gumbel", "policy", "value",
                           "action", "root_visits", "root_n", "root_w", "mm_max", "mm_min",
                           "n_initial", "n_recurrent", "recurrent_rows")}
    t0 = time.time()
    for mv in range(n_moves):
        if game.get_game_ended() is not None:
            game = _new_game(size, n_open, rs_open)  # game over: continue from a fresh position
        rec["board"].append(game.board.reshape(-1).copy())
        rec["player"].append(game.current_player)
        rec["lastmove"].append(-1 if game.last_move is None else game.last_move[0] * size + game.last_move[1])
        rec["movecount"].append(game.move_count)
        Rec.roots.clear(); Rec.stats.clear(); _gumbel_log.clear(); q.log.clear()
        policy, value, action = eng.search(game)
        assert len(_gumbel_log) == 1 and len(Rec.stats) == 1
        root = Rec.roots[0]
        rec["gumbel"].append(_gumbel_log[0])
        rec["policy"].append(np.asarray(policy, dtype=np.float64))
        assert isinstance(value, np.float32), type(value)
        rec["value"].append(value)
        rec["action"].append(action)
        rv = np.zeros(A, np.int32)
        for a, ch in root.children.items():
            rv[a] = ch.visit_count
        rec["root_visits"].append(rv)
        rec["root_n"].append(root.visit_count)
        rec["root_w"].append(np.float32(root.value_sum))
        st = Rec.stats[0]
        rec["mm_max"].append(np.float32(st.maximum))
        rec["mm_min"].append(np.float32(st.minimum))
        rec["n_initial"].append(sum(1 for k, _ in q.log if k == "initial"))
        rec["n_recurrent"].append(sum(1 for k, _ in q.log if k == "recurrent_batch"))
        rec["recurrent_rows"].append(sum(n for k, n in q.log if k == "recurrent_batch"))
        game.do_move(action)
    out = {"size": size, "mode": mode, "sims": sims, "seed": seed}
    dt = {"board": np.int8, "player": np.int8, "lastmove": np.int32, "movecount": np.int32,
          "gumbel": np.float64, "policy": np.float64, "value": np.float32, "action": np.int32,
          "root_visits": np.int32, "root_n": np.int32, "root_w": np.float32, "mm_max": np.float32,
          "mm_min": np.float32, "n_initial": np.int32, "n_recurrent": np.int32, "recurrent_rows": np.int32}
    for k, v in rec.items():
        out[k] = np.array(v, dtype=dt[k])
    np.savez_compressed(os.path.join(HERE, "mcts_%s.npz" % name), **out)
    print("mcts", name, "moves", len(rec["action"]), "actions", rec["action"], "%.1fs" % (time.time() - t0))


# ============================================================ winning-move scanner
def make_winmoves():
    import workers
    out = {}
    set_board(15)
    rs = np.random.RandomState(77)
    boards, players, five, open4, combo = [], [], [], [], []
    c = 7
    pats = []
    b = np.zeros((15, 15), np.int8); b[c, c - 1:c + 2] = 1; pats.append(b)
    b = np.zeros((15, 15), np.int8); b[c, c - 1] = b[c, c + 1] = b[c - 1, c] = b[c + 1, c] = 1; pats.append(b)
    b = np.zeros((15, 15), np.int8); b[c, c - 2] = -1; b[c, c - 1] = b[c, c + 1] = 1; b[c - 1, c] = b[c + 1, c] = 1; pats.append(b)
    b = np.zeros((15, 15), np.int8); b[c, c - 2] = -1; b[c, c - 1] = b[c, c + 1] = 1; b[c - 2, c] = -1; b[c - 1, c] = b[c + 1, c] = 1; pats.append(b)
    for t in range(200):
        n = rs.randint(5, 90)
        b = np.zeros(225, np.int8)
        idx = rs.choice(225, n, replace=False)
        b[idx[: n // 2]] = 1
        b[idx[n // 2:]] = -1
        pats.append(b.reshape(15, 15))
    for i, b in enumerate(pats):
        p = 1 if i < 4 or i % 2 == 0 else -1
        res = workers.find_winning_moves_rebuilt(b.copy(), p)
        m = [np.zeros(225, np.uint8) for _ in range(3)]
        for j, key in enumerate(("five", "open_four", "combo")):
            for (r, cc) in res[key]:
                m[j][r * 15 + cc] = 1
        boards.append(b.reshape(-1)); players.append(p)
        five.append(m[0]); open4.append(m[1]); combo.append(m[2])
    out = dict(boards=np.array(boards, np.int8), players=np.array(players, np.int8),
               five=np.array(five, np.uint8), open_four=np.array(open4, np.uint8), combo=np.array(combo, np.uint8))
    np.savez_compressed(os.path.join(HERE, "winmoves.npz"), **out)
    print("winmoves", len(boards))


# ============================================================ worker game record
def make_worker_record():
    """Run the reference universal_worker (mode 0) for exactly one scripted game."""
    import workers
    import multiprocessing as mp
    set_board(6)
    ref_config.NUM_SIMULATIONS = 8
    ref_config.MCTS_IMPLEMENTATION = "MuZero"
    A = 36
    script_rs = np.random.RandomState(5)
    # scripted game: player 1 builds a row on row 2, player -1 plays elsewhere -> P1 wins at move 9
    seq = [12, 0, 13, 1, 14, 35, 15, 30, 16]
    pols = [script_rs.dirichlet(np.ones(A)).astype(np.float64) for _ in seq]
    vals = [np.float32(script_rs.uniform(-1, 1)) for _ in seq]

    class FakeMCTS:
        def __init__(self, *a, **k):
            self.i = 0

        def search(self, game):
            i = self.i
            self.i += 1
            return pols[i], vals[i], seq[i]

    workers.MuZeroMCTS = FakeMCTS
    workers.setup_worker_logging = lambda q: None

    class Ev:
        def __init__(self):
            self.flag = False

        def is_set(self):
            return self.flag

        def set(self):
            self.flag = True

    shutdown = Ev()
    captured = {}

    class DataQ:
        def put(self, item):
            captured["item"] = item
            shutdown.set()

    class SinkQ:
        def __init__(self):
            self.items = []

        def put(self, x):
            self.items.append(x)

        def full(self):
            return False

    ui, logq, trq = SinkQ(), SinkQ(), SinkQ()
    pause = Ev()

    class V:
        value = 0

    ver = V(); ver.value = 1234
    workers.universal_worker(0, V(), DataQ(), logq, ui, shutdown, None, None, None, trq, ver, None, pause)
    gr, slices, version = captured["item"]
    out = dict(actions=np.array(gr.actions, np.int32), rewards=np.array(gr.rewards, np.float32),
               values=np.array(gr.values, np.float32), policies=np.array(gr.policies, np.float64),
               observations=np.array(gr.observations, np.float32), board_states=np.array(gr.board_states, np.int8),
               sl_obs=np.array([s.observation for s in slices], np.float32),
               sl_act=np.array([s.action_history for s in slices], np.int32),
               sl_rew=np.array([s.reward_history for s in slices], np.float32),
               sl_pol=np.array([s.policy_history for s in slices], np.float64),
               sl_val=np.array([s.value_history for s in slices], np.float32),
               version=np.int64(version), in_pols=np.array(pols), in_vals=np.array(vals, np.float32),
               in_seq=np.array(seq, np.int32),
               ui_kinds=np.array([type(x).__name__ for x in ui.items]),
               status=np.array([[x.avg_len, x.miss_five, x.miss_total] for x in logq.items], np.float64),
               trainer_kinds=np.array([type(x).__name__ for x in trq.items]))
    np.savez_compressed(os.path.join(HERE, "worker_record.npz"), **out)
    print("worker record: moves", len(gr.actions), "ui", out["ui_kinds"].tolist())


# ============================================================ network
def _net_case(fname, size, C, blocks, hd, seed, n_rows, full_hidden):
    import datou_gomoku_muzero_amd.weights as W
    from datou_gomoku_muzero_amd.config import GmzConfig
    import network as ref_network
    set_board(size)
    ref_config.NUM_FILTERS, ref_config.NUM_RES_BLOCKS, ref_config.HEAD_HIDDEN_DIM = C, blocks, hd
    cfg = GmzConfig(BOARD_SIZE=size, NUM_FILTERS=C, NUM_RES_BLOCKS=blocks, HEAD_HIDDEN_DIM=hd)
    torch.manual_seed(0)
    model = ref_network.GomokuNetEZ(ref_config)
    sd = W.synthetic_state_dict(cfg, seed=seed)
    ref_keys = [(k, tuple(v.shape)) for k, v in model.state_dict().items()]
    my_keys = [(k, tuple(v.shape)) for k, v in sd.items()]
    assert ref_keys == my_keys, "state_dict layout mismatch"
    model.load_state_dict(W.to_torch(sd))
    model.eval()
    torch.set_num_threads(1)
    rs = np.random.RandomState(seed + 1)
    A = size * size
    obs = []
    for i in range(n_rows):
        game = ref_game.GomokuGame(board_size=size, n_in_row=5)
        for _ in range(rs.randint(0, min(A - 1, 30))):
            vm = game.get_valid_moves()
            m = vm[rs.randint(len(vm))]
            game.do_move(int(m[0] * size + m[1]))
        obs.append(game.get_board_state(game.current_player, game.last_move))
    obs = np.array(obs, np.float32)
    actions = rs.randint(0, A, n_rows).astype(np.int64)
    with torch.no_grad():
        p, v, h = model.initial_inference(torch.from_numpy(obs))
        p2, v2, h2, r2 = model.recurrent_inference(h, torch.from_numpy(actions))
    out = dict(size=size, C=C, blocks=blocks, hd=hd, seed=seed, obs=obs, actions=actions.astype(np.int32),
               p=p.numpy(), v=v.numpy(), p2=p2.numpy(), v2=v2.numpy(), r2=r2.numpy(),
               h_sum=h.double().sum(dim=(1, 2, 3)).numpy(), h_sq=(h.double() ** 2).sum(dim=(1, 2, 3)).numpy(),
               h2_sum=h2.double().sum(dim=(1, 2, 3)).numpy(), h2_sq=(h2.double() ** 2).sum(dim=(1, 2, 3)).numpy(),
               wsum=np.array([float(np.sum(np.abs(x.astype(np.float64)))) for x in sd.values()]))
    if full_hidden:
        out["h"] = h.numpy()
        out["h2"] = h2.numpy()
    else:
        out["h_corner"] = h[:, :8, :4, :4].numpy()
        out["h2_corner"] = h2[:, :8, :4, :4].numpy()
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print("net", fname, "p range", float(p.abs().max()), "v", v.view(-1).tolist()[:4])


def make_net():
    _net_case("net_small.npz", 9, 32, 2, 16, seed=3, n_rows=4, full_hidden=True)
    _net_case("net_c15.npz", 15, 128, 8, 64, seed=5, n_rows=2, full_hidden=False)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    jobs = {"game": make_game_cases, "winmoves": make_winmoves, "worker": make_worker_record, "net": make_net}
    for sc in SCENARIOS:
        jobs["mcts_" + sc[0]] = (lambda sc=sc: make_mcts_case(*sc))
    for name, fn in jobs.items():
        if args.only and not name.startswith(args.only):
            continue
        fn()
