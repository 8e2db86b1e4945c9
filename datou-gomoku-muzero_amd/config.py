"""Hot-path configuration keys, mirroring the reference's global ``config`` singleton
(/root/reference/config.py:4-109).  Only the keys the self-play path reads are kept.

The engine accepts *any* object exposing these attribute names, so the reference's own
``config`` object can be passed unchanged (drop-in); :class:`GmzConfig` is a standalone default.
"""
from dataclasses import dataclass, field, asdict


@dataclass
class GmzConfig:
    BOARD_SIZE: int = 15                 # config.py:18 (reference default 6; configs 2-4 use 15)
    N_IN_ROW: int = 5                    # config.py:19
    NUM_SIMULATIONS: int = 400           # config.py:22
    NUM_TOP_ACTIONS: int = 16            # config.py:23
    MCTS_IMPLEMENTATION: str = "MuZero"  # config.py:25 ("AlphaZero" | "MuZero")
    C_VISIT: float = 30                  # config.py:31
    C_SCALE: float = 1.0                 # config.py:32
    VALUE_MINMAX_DELTA: float = 1e-3     # config.py:33
    DISCOUNT: float = 0.997              # config.py:34
    VALUE_SUPPORT_MIN: int = -1          # config.py:40-42
    VALUE_SUPPORT_MAX: int = 1
    VALUE_SUPPORT_BINS: int = 3
    REWARD_SUPPORT_MIN: int = -1         # config.py:45-47
    REWARD_SUPPORT_MAX: int = 1
    REWARD_SUPPORT_BINS: int = 3
    NUM_RES_BLOCKS: int = 8              # config.py:49
    NUM_FILTERS: int = 128               # config.py:50
    HEAD_HIDDEN_DIM: int = 64            # config.py:51
    NUM_UNROLL_STEPS: int = 5            # config.py:71 (TrainingSlice shape)
    N_STEPS: int = 10                    # config.py:100 (n-step value targets)
    NUM_WORKERS: int = 15                # config.py:13
    REANALYSIS_AGE_THRESHOLD: int = 900  # config.py:89 (re-analysis eligibility, trainer steps)
    ACTION_SPACE_SIZE: int = field(default=None)

    def __post_init__(self):
        if self.ACTION_SPACE_SIZE is None:
            self.ACTION_SPACE_SIZE = self.BOARD_SIZE * self.BOARD_SIZE

    def as_dict(self):
        return asdict(self)


HOT_KEYS = tuple(GmzConfig.__dataclass_fields__.keys())


def from_any(cfg=None, **overrides):
    """Build a GmzConfig from an object with reference-style attributes (or None → defaults)."""
    vals = {}
    if cfg is not None:
        for k in HOT_KEYS:
            if hasattr(cfg, k):
                vals[k] = getattr(cfg, k)
    vals.update(overrides)
    if "BOARD_SIZE" in overrides and "ACTION_SPACE_SIZE" not in overrides:
        vals["ACTION_SPACE_SIZE"] = None
    out = GmzConfig(**vals)
    if out.ACTION_SPACE_SIZE != out.BOARD_SIZE * out.BOARD_SIZE:
        raise ValueError("ACTION_SPACE_SIZE must equal BOARD_SIZE**2 (config.py:20)")
    return out
