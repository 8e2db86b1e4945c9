"""HashNet — deterministic integer-hash stand-in for GomokuNetEZ (TEST INFRASTRUCTURE).

ORACLE / TEST INFRASTRUCTURE ONLY: imported by tests/, tests/golden/make_golden.py,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never part of the product path.

Why it exists: tree-search parity (SURVEY.md §8c "tape" fixtures) must be tested separately from
network floating-point drift.  HashNet plays the role of the reference's MockModel
(/root/reference/tests/test_mcts_logic.py:60-80) but, unlike MockModel, produces *distinct*
outputs per node so that the search tree is non-degenerate.  Every output is an exact small
dyadic rational, so numpy (reference harness), the C oracle (oracle/gmz_oracle.c) and the HIP
engine (csrc/gmz_hashnet.hip) produce bit-identical float32 values.

Definition (all arithmetic mod 2**32):
  mix32(x)       = lowbias32 finaliser
  initial(obs)   : id = mix32(0xA511E9B3 + sum_{j : obs.flat[j] != 0} mix32(j*0x9E3779B1 + 0x7F4A7C15))
                   (obs = float32 [3, H, W] planes of game.py:12-17, j = flat index)
  recurrent(id,a): id' = mix32(id*0x2C1B3C6D + (a+1)*0x297A2D39 + 0x5851F42D)
  logits[i]      = ((mix32(id ^ mix32(i + 0x1000)) >> 20) - 2048) / 256      in [-8, 8)
  value          = ((mix32(id + 0x3C6EF372) >> 16) - 32768) / 32768           in [-1, 1)
  reward         = ((mix32(id + 0xDAA66D2B) >> 24) - 128) / 512               in [-0.25, 0.25)
The "hidden state" is the uint32 id, carried as a uint32 array of shape [1, 1].
"""
import numpy as np

M32 = 0xFFFFFFFF


def mix32(x):
    """lowbias32 integer finaliser on uint32 scalars or arrays (wrapping arithmetic)."""
    x = np.asarray(x, dtype=np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32)


def initial_id(obs):
    flat = np.asarray(obs, dtype=np.float32).reshape(-1)
    j = np.nonzero(flat != 0)[0].astype(np.uint64)
    terms = mix32((j * np.uint64(0x9E3779B1) + np.uint64(0x7F4A7C15)) & M32).astype(np.uint64)
    s = (np.uint64(0xA511E9B3) + (terms.sum(dtype=np.uint64) & M32)) & M32
    return int(mix32(s))


def recurrent_id(hid, action):
    x = (np.uint64(hid) * np.uint64(0x2C1B3C6D) + np.uint64(int(action) + 1) * np.uint64(0x297A2D39)
         + np.uint64(0x5851F42D)) & M32
    return int(mix32(x))


def logits_of(hid, A):
    i = np.arange(A, dtype=np.uint64)
    salt = mix32(i + np.uint64(0x1000)).astype(np.uint64)
    h = mix32(np.uint64(hid) ^ salt)
    return (((h >> np.uint32(20)).astype(np.int64) - 2048).astype(np.float32) / np.float32(256.0))


def value_of(hid):
    h = int(mix32((int(hid) + 0x3C6EF372) & M32))
    return np.float32(((h >> 16) - 32768) / 32768.0)


def reward_of(hid):
    h = int(mix32((int(hid) + 0xDAA66D2B) & M32))
    return np.float32(((h >> 24) - 128) / 512.0)


class HashNet:
    """Batched HashNet with the numpy-in/numpy-out shape contract of the reference's
    inference server (workers.py:351-369): initial -> (p f32[B,A], v f32[B,1], h u32[B,1]);
    recurrent -> (p, v, h, r f32[B,1])."""

    def __init__(self, action_space):
        self.A = int(action_space)

    def initial(self, obs_batch):
        ids = [initial_id(o) for o in obs_batch]
        return self._outs(ids)

    def recurrent(self, hidden_batch, actions):
        ids = [recurrent_id(int(h), int(a)) for h, a in zip(np.asarray(hidden_batch).reshape(-1), actions)]
        p, v, h = self._outs(ids)
        r = np.array([[reward_of(i)] for i in ids], dtype=np.float32)
        return p, v, h, r

    def _outs(self, ids):
        p = np.stack([logits_of(i, self.A) for i in ids]).astype(np.float32)
        v = np.array([[value_of(i)] for i in ids], dtype=np.float32)
        h = np.array(ids, dtype=np.uint32).reshape(-1, 1)
        return p, v, h
