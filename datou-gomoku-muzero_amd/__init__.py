"""datou_gomoku_muzero_amd — MI355X-native batched Gumbel-MuZero/AlphaZero self-play engine.

Drop-in for the reference's self-play hot path:
  * ``mcts.HipMuZeroMCTS`` / ``mcts.HipAlphaZeroMCTS`` — same ``search(game)`` contract as
    /root/reference/mcts.py:50-64 (single-game adapters, request-count compatible);
  * ``engine.BatchedSelfPlayEngine`` — G games per GPU, search + play as HIP kernels;
  * ``worker.gpu_selfplay_worker`` — process target emitting the messages of workers.py:129-241.

Native code: ``csrc/`` → ``libgmz.so`` (C ABI declared in include/gmz.h), loaded by ``_lib``.
"""
from .config import GmzConfig  # noqa: F401

__all__ = ["GmzConfig"]
