"""Inference-queue stand-ins with the reference's protocol (mcts.py:73-85, workers.py:344-369,
tests/test_mcts_logic.py:26-80).  Test infrastructure."""
from queue import Empty

import numpy as np

import hashnet


class ServerQueue:
    """request/result queue pair answering like inference_server_worker, backed by HashNet."""

    def __init__(self, A):
        self.net, self.results, self.log = hashnet.HashNet(A), [], []

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


class MockQueue:
    """tests/test_mcts_logic.py MockInferenceQueue + MockModel semantics: zero logits, value 0.5,
    reward 0, hidden all ones (initial) / all twos (recurrent).  One object is both queues."""

    def __init__(self, A, C=4, H=6):
        self.A, self.C, self.H = A, C, H
        self.request_log, self.put_log = [], []

    def put(self, item):
        self.request_log.append(item)
        self.put_log.append(item)

    def get(self, timeout=None):
        if not self.request_log:
            raise Empty("Mock queue has no requests to process.")
        wid, kind, data = self.request_log.pop(0)
        if kind == "initial":
            return np.zeros(self.A, np.float32), 0.5, np.ones((1, self.C, self.H, self.H), np.float32)
        hs, acts = data
        k = len(acts)
        return (np.zeros((k, self.A), np.float32), np.full((k, 1), 0.5, np.float32), np.ones_like(hs) * 2,
                np.zeros((k, 1), np.float32))

    def get_nowait(self):
        if not self.request_log:
            raise Empty
        return self.request_log.pop(0)


class Game:
    """Minimal GomokuGame-shaped position (game.py:4-11 attributes the adapters read)."""

    def __init__(self, board, player, last_move):
        self.board = np.asarray(board, np.int8).copy()
        self.board_size = self.board.shape[0]
        self.current_player = int(player)
        self.last_move = last_move
        self.move_count = int(np.count_nonzero(self.board))
