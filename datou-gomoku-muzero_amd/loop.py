"""Config C4: the reference's full loop — self-play, replay, training, weight push — on N GPUs.

The reference runs it as a process graph (main.py:91-109): NUM_WORKERS ``universal_worker`` +
one ``inference_server_worker`` for self-play, a ``data_loader_worker`` owning the PER replay buffer
(workers.py:379-439, replay_buffer.py:44-106) and one ``training_worker`` (workers.py:445-628) that
pushes ``ModelWeightsUpdate`` to the inference server every MODEL_UPDATE_INTERVAL steps
(workers.py:587-593).  Here, one process per GPU (rank r of N) holds ALL of those roles for its
own share of the work, time-sliced on its GPU:

  self-play   G games on the HIP engine (engine.BatchedSelfPlayEngine + network.GomokuNetHip), the
              move history kept on the device and harvested one move behind (worker.GameHistory);
  replay      every finished game becomes the reference's TrainingSlices (records.py semantics,
              built as arrays by ``slices_from_game``) appended to THIS rank's device-resident
              replay shard (trainer.ReplayBuffer) — no data crosses ranks;
  training    data-parallel: each rank samples its batch from its own shard; gradients are averaged
              by one flat-bucket all-reduce per step (RCCL over xGMI); PER (sharded):
              IS weights from the global slice count (all-reduce SUM) normalised by the global batch
              max (all-reduce MAX), the admission priority kept global (all-reduce MAX);
  weight push every ``model_update_interval`` trainer steps rank 0's weights are broadcast (one flat
              fp32 bucket, weight_sync.broadcast_state_dict) and every rank hot-swaps them into its
              inference network, as the inference server does on ModelWeightsUpdate.

One *iteration* = ``moves_per_iter`` self-play moves of all G games, then ``train_steps_per_iter``
trainer steps (all ranks together, once every shard holds a batch).  ``concurrent=True`` (GPU): the
iteration's trainer steps and replay-shard updates are enqueued on a HIP stream of their own BEFORE
its moves, so the trainer's many short kernels run beside the self-play towers instead of after them
(the reference's trainer and self-play workers also run at the same time, main.py:91-109); the host
waits for the previous iteration's training before enqueueing the next, so the backlog stays one
iteration.  The self-play source and the inference network are pluggable (``SelfPlay`` on the GPU;
tests drive the same loop on CPU with scripted games over gloo).
"""
import time

import numpy as np
import torch

from . import records as R
from .weight_sync import broadcast_state_dict
from .worker import board_states_to_obs


def slices_from_game(boards, players, lasts, pols, vals, acts, winner, H, discount, n_steps, unroll):
    """One finished game -> the reference's TrainingSlices as stacked arrays (workers.py:183-222,
    same values as records.build_game_record's slice list):
    obs uint8 [n, U+1, 3, H, H], act int32 [n, U], rew f32 [n, U], pol f32 [n, U+1, A], val f32 [n, U+1]."""
    n, U = len(acts), unroll
    A = H * H
    obs = board_states_to_obs(np.asarray(boards).reshape(n, A), np.asarray(players), np.asarray(lasts), H)
    rew = R.final_rewards(n, winner)
    vt = np.asarray(R.compute_n_step_returns(rew.tolist(), list(vals), discount, n_steps), dtype=np.float32)
    pad = lambda x, k, v=0: np.concatenate([x, np.full((k,) + x.shape[1:], v, dtype=x.dtype)])  # noqa: E731
    win = lambda x, w: np.lib.stride_tricks.sliding_window_view(x, w, axis=0)[:n]  # noqa: E731
    o = win(pad(obs.astype(np.uint8), U + 1), U + 1)           # [n, 3, H, H, U+1]
    a = win(pad(np.asarray(acts, np.int32), U, -1), U)         # [n, U]
    r = win(pad(rew.astype(np.float32), U), U)
    p = win(pad(np.asarray(pols, np.float32).reshape(n, A), U + 1), U + 1)  # [n, A, U+1]
    v = win(pad(vt, U + 1), U + 1)
    return (np.ascontiguousarray(np.moveaxis(o, -1, 1)), np.ascontiguousarray(a), np.ascontiguousarray(r),
            np.ascontiguousarray(np.moveaxis(p, -1, 1)), np.ascontiguousarray(v))


class SelfPlay:
    """G games on this rank's GPU (the self-play half of the worker loop, worker.py)."""

    def __init__(self, cfg, num_games, state_dict, seed=0, precision="fp16", streams=None, openings=None):
        from . import engine as E, network as N
        from .worker import GameHistory
        c = cfg
        self.cfg, self.G = c, int(num_games)
        self.net = N.GomokuNetHip(state_dict, c, num_slots=E.hidden_slots(c, self.G), max_rows=self.G,
                                  precision=precision)
        self.eng = E.make_engine(c, num_games=self.G, net=self.net, seed=seed, streams=streams)
        self.eng.reset_games()
        self.hist = GameHistory(self.G, c.ACTION_SPACE_SIZE, self.eng.device, min_game_len=2 * c.N_IN_ROW - 1)
        if openings is not None:  # (boards, players, last_moves, move_counts): e.g. engine.random_openings
            self.eng.set_positions(*openings)
            self.hist.set_start(openings[3])
        dev = self.eng.device
        self.missed = (torch.zeros(self.G, dtype=torch.int32, device=dev), torch.zeros(self.G, dtype=torch.int32, device=dev))
        self.pending = None
        self.moves = 0

    def step(self):
        """Play one move of every game; returns the games that finished one move earlier
        (GameHistory.harvest tuples)."""
        e, h = self.eng, self.hist
        b, p, lm, mc = e.game_state()
        pol, val, act = e.search()
        e.winning_scan(b, p, act, counters=self.missed)
        h.record(b, p, lm, mc, pol, val, act)
        status = e.play(reset_finished=True)
        sn = h.after_play(status, mc, act, *self.missed)
        done = h.harvest(self.pending)
        self.pending = sn
        self.moves += 1
        return done

    def flush(self):
        done = self.hist.harvest(self.pending)
        self.pending = None
        return done

    def load_weights(self, sd):
        self.net.load_state_dict(sd)

    def close(self):
        self.eng.close()


class C4Loop:
    """The composed loop on one rank (see module docstring).  ``dist``: torch.distributed or None."""

    def __init__(self, selfplay, trainer, buffer, cfg, batch_size, dist=None, moves_per_iter=1,
                 train_steps_per_iter=1, model_update_interval=1000, seed=0, device="cuda", concurrent=False):
        self.sp, self.tr, self.rb, self.cfg = selfplay, trainer, buffer, cfg
        self.B, self.dist = int(batch_size), dist
        self.moves_per_iter, self.train_steps_per_iter = int(moves_per_iter), int(train_steps_per_iter)
        self.model_update_interval = int(model_update_interval)
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.rs = np.random.RandomState(seed + 1000003 * self.rank)
        self.device = torch.device(device)
        self.games = self.slices = self.train_steps = self.weight_pushes = 0
        self.game_lengths = []
        self.last_logs = None
        self.concurrent = bool(concurrent) and self.device.type == "cuda"
        # concurrent mode: every replay-shard and trainer operation goes to this stream (one ordering
        # for adds, samples, steps and priority updates); the self-play engines keep theirs
        self.train_stream = torch.cuda.Stream(self.device) if self.concurrent else None
        # the self-play engines fork every move from this stream: weight swaps are enqueued on it
        self.sp_stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        self._train_done = None

    # ---------------------------------------------------------------- pieces
    def _add_games(self, done):
        c = self.cfg
        for (g, winner, n, mf, mt, boards, players, lasts, pols, vals, acts) in done:
            arrs = slices_from_game(boards, players, lasts, pols, vals, acts, winner, c.BOARD_SIZE, c.DISCOUNT,
                                    c.N_STEPS, c.NUM_UNROLL_STEPS)
            self.rb.add_arrays(*arrs)
            self.games += 1
            self.slices += n
            self.game_lengths.append(n)

    def _all_ready(self):
        """Every rank's shard holds a batch (all ranks must step together: the all-reduce)."""
        ok = 1.0 if len(self.rb) >= self.B else 0.0
        if self.dist is None or self.world == 1:
            return ok > 0
        t = torch.tensor([ok], dtype=torch.float32)
        if self.dist.get_backend() != "gloo":
            t = t.to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return float(t.item()) > 0

    def push_weights(self):
        """ModelWeightsUpdate (workers.py:587-593): rank 0's trainer weights -> every rank's inference net."""
        if self.train_stream is not None:
            self.train_stream.synchronize()  # the step that made these weights has finished
        sd = self.tr.state_dict_cpu()
        if self.dist is not None and self.world > 1:
            dev = "cpu" if self.dist.get_backend() == "gloo" else self.device
            sd = broadcast_state_dict(sd, src=0, device=dev)
        if self.sp_stream is not None:
            # on the self-play stream, not the trainer's (concurrent mode calls this from inside the train
            # stream's context): the copies of the new weights are then ordered before the next move's
            # kernels, and after the previous move's, which join this stream.  With RCCL the broadcast
            # filled its device buffers on the CURRENT stream (the trainer's in concurrent mode), so the
            # self-play stream waits for that stream before it reads them
            cur = torch.cuda.current_stream(self.device)
            if cur != self.sp_stream:
                self.sp_stream.wait_stream(cur)
            with torch.cuda.stream(self.sp_stream):
                self.sp.load_weights(sd)
        else:
            self.sp.load_weights(sd)
        self.weight_pushes += 1

    def train_step(self):
        batch, idx, w = self.rb.sample(self.B, self.rs, dist=self.dist)
        logs, td = self.tr.step(batch, w, sync=False)
        self.rb.update_priorities(idx, td, dist=self.dist)
        self.last_logs = logs
        self.train_steps += 1
        if self.train_steps % self.model_update_interval == 0:
            self.push_weights()

    # ---------------------------------------------------------------- one iteration
    def iteration(self):
        if self.concurrent:
            return self._iteration_concurrent()
        for _ in range(self.moves_per_iter):
            self._add_games(self.sp.step())
        if self.train_steps_per_iter > 0 and self._all_ready():
            for _ in range(self.train_steps_per_iter):
                self.train_step()

    def _iteration_concurrent(self):
        ts = self.train_stream
        if self._train_done is not None:
            self._train_done.synchronize()  # the previous iteration's training: backlog <= one iteration
        if self.train_steps_per_iter > 0 and self._all_ready():
            ts.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(ts):
                for _ in range(self.train_steps_per_iter):
                    self.train_step()
        done = []
        for _ in range(self.moves_per_iter):
            done += self.sp.step()
        with torch.cuda.stream(ts):  # after this iteration's steps on the same stream
            self._add_games(done)
        self._train_done = torch.cuda.Event()
        self._train_done.record(ts)

    def run(self, iterations):
        for _ in range(iterations):
            self.iteration()
        if self.train_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.train_stream)
        return self.stats()

    def stats(self):
        return {"moves": int(getattr(self.sp, "moves", 0)), "games": self.games, "slices": self.slices,
                "train_steps": self.train_steps, "weight_pushes": self.weight_pushes, "buffer": len(self.rb)}


def run_c4(args, rank, world, dist, backend, log=print):
    """bench.py's C4 leg: the composed loop on this rank, timed; returns this rank's counts + time."""
    from . import trainer as T, weights as W
    from .config import GmzConfig
    torch.backends.cudnn.benchmark = True
    cfg = GmzConfig(BOARD_SIZE=args.size, NUM_SIMULATIONS=args.sims, NUM_RES_BLOCKS=args.blocks)
    tcfg = T.TrainConfig(BOARD_SIZE=args.size, NUM_RES_BLOCKS=args.blocks, PHYSICAL_BATCH_SIZE=args.trainer_batch,
                         TRAIN_BUFFER_SIZE=args.loop_buffer, ENABLE_PER=True,
                         MODEL_UPDATE_INTERVAL=args.loop_update_interval)
    tr = T.Trainer(tcfg, device="cuda")
    sd = tr.state_dict_cpu()  # the trainer's initial weights (rank 0's, broadcast by Trainer) feed self-play
    openings = None
    if getattr(args, "loop_openings", 0) > 0:  # staggered starts: games at every stage from the first move on
        from .engine import random_openings
        openings = random_openings(args.loop_games, args.size, np.random.RandomState(args.seed + 17 * rank),
                                   args.loop_openings, n_in_row=cfg.N_IN_ROW)
    sp = SelfPlay(cfg, args.loop_games, sd, seed=args.seed + 7919 * rank, precision=getattr(args, "precision", "fp16"),
                  openings=openings)
    rb = T.ReplayBuffer(tcfg, device="cuda")
    if args.loop_prefill:
        from .weights import synthetic_slices
        rb.add_arrays(*synthetic_slices(args.loop_prefill, args.size, tcfg.NUM_UNROLL_STEPS,
                                        np.random.RandomState(args.seed + 31 * rank)))
    loop = C4Loop(sp, tr, rb, tcfg, args.trainer_batch, dist=dist if world > 1 else None,
                  moves_per_iter=args.loop_moves_per_iter, train_steps_per_iter=args.loop_train_per_iter,
                  model_update_interval=args.loop_update_interval, seed=args.seed,
                  concurrent=getattr(args, "loop_concurrent", False))
    t_w = time.perf_counter()
    loop.run(args.loop_warmup)
    torch.cuda.synchronize()
    log("rank %d: C4 loop warm-up %.1f s" % (rank, time.perf_counter() - t_w))
    s0 = loop.stats()
    if dist is not None and world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loop.run(args.loop_iters)
    torch.cuda.synchronize()
    if dist is not None and world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    s1 = loop.stats()
    d = {k: s1[k] - s0[k] for k in ("moves", "games", "slices", "train_steps", "weight_pushes")}
    d["buffer"] = s1["buffer"]
    # one ModelWeightsUpdate (workers.py:587-593) on its own, after the timed window: rank 0's trainer
    # weights -> broadcast -> every rank's inference network; the timed window runs the reference's
    # interval (1000 steps), so this is what a push adds once per interval
    n_push = 3
    if dist is not None and world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_p = time.perf_counter()
    for _ in range(n_push):
        loop.push_weights()
    torch.cuda.synchronize()
    d["push_ms"] = (time.perf_counter() - t_p) / n_push * 1e3
    sp.close()
    return d, dt
