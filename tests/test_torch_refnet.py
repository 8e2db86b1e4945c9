"""The float32 PyTorch checker network (tests/torch_refnet.py) equals oracle/netref.py on CPU."""
import numpy as np
import torch

import netref
from torch_refnet import TorchRefNet
from datou_gomoku_muzero_amd import weights as W
from datou_gomoku_muzero_amd.config import GmzConfig


def test_torch_refnet_matches_netref():
    cfg = GmzConfig(BOARD_SIZE=9, NUM_RES_BLOCKS=2)
    sd = W.synthetic_state_dict(cfg, seed=3, with_projection=False)
    net = TorchRefNet(sd, 9, 2, 8, device="cpu")
    obs = (np.random.RandomState(0).rand(3, 3, 9, 9) < 0.2).astype(np.float32)
    lg, v = torch.zeros(3, 81), torch.zeros(3)
    net.initial(torch.from_numpy(obs), torch.tensor([0, 1, -1]), lg, v, None)
    p, vr, h = netref.initial_inference(sd, obs)
    assert np.abs(lg.numpy()[:2] - p[:2]).max() < 1e-5 and np.abs(v.numpy()[:2] - vr[:2, 0]).max() < 1e-5
    assert (lg.numpy()[2] == 0).all()  # skipped row untouched
    lg2, v2, r2 = torch.zeros(2, 81), torch.zeros(2), torch.zeros(2)
    net.recurrent(torch.tensor([0, 1]), torch.tensor([5, 80]), torch.tensor([3, 4]), lg2, v2, r2, None)
    p2, v2r, h2, r2r = netref.recurrent_inference(sd, h[:2], np.array([5, 80]))
    assert np.abs(lg2.numpy() - p2).max() < 1e-5 and np.abs(r2.numpy() - r2r[:, 0]).max() < 1e-5
    assert np.abs(net.pool[3:5].numpy() - h2).max() < 1e-4
