"""float32 GomokuNetEZ inference in PyTorch (test infrastructure / checker, never shipped).

A restatement of the reference's eval-mode forward (/root/reference/network.py:30-152:
representation, prediction and dynamics networks, BatchNorm eps 1e-4 with running statistics,
support_to_scalar over linspace(-1, 1, 3)) on the GPU in float32, exposing the engine's network
backend interface (``initial`` / ``recurrent`` writing into slot-indexed buffers) so that the HIP
engine can run the SAME batched search with a float32 network.  Used to measure how often the f16 /
bf16 HIP network changes a search's decision (tools/action_agreement.py, tests/test_agreement_gpu.py).
Pinned against oracle/netref.py (numpy float32) in tests/test_agreement_gpu.py.
"""
import numpy as np
import torch
import torch.nn.functional as F

EPS = 1e-4


class TorchRefNet:
    def __init__(self, state_dict, board_size, blocks, num_slots, device="cuda"):
        self.H, self.A, self.nb = board_size, board_size * board_size, blocks
        self.dev = torch.device(device)
        self.p = {k: torch.as_tensor(np.asarray(v, dtype=np.float32)).to(self.dev)
                  for k, v in state_dict.items() if not k.endswith("num_batches_tracked")}
        self.pool = torch.zeros(num_slots, 128, board_size, board_size, dtype=torch.float32, device=self.dev)

    # ---------------------------------------------------------------- network.py restated
    def _bn(self, x, pre):
        p = self.p
        return F.batch_norm(x, p[pre + ".running_mean"], p[pre + ".running_var"], p[pre + ".weight"], p[pre + ".bias"],
                            False, 0.0, EPS)

    def _conv(self, x, key, pad=1):
        return F.conv2d(x, self.p[key], self.p.get(key[:-len("weight")] + "bias"), padding=pad)

    def _blocks(self, x, net):
        for i in range(self.nb):
            pre = "%s.resblocks.%d." % (net, i)
            out = F.relu(self._bn(self._conv(x, pre + "conv1.weight"), pre + "bn1"))
            out = self._bn(self._conv(out, pre + "conv2.weight"), pre + "bn2")
            x = F.relu(out + x)
        return x

    @staticmethod
    def _support(logits):
        sup = torch.linspace(-1, 1, 3, device=logits.device)
        return (F.softmax(logits, dim=1) * sup).sum(1)

    def representation(self, obs):
        x = F.relu(self._bn(self._conv(obs, "representation_net.conv.weight"), "representation_net.bn"))
        return self._blocks(x, "representation_net")

    def prediction(self, h):
        p = self.p
        pp = F.relu(self._bn(self._conv(h, "prediction_net.policy_conv.weight", 0), "prediction_net.policy_bn"))
        logits = F.linear(pp.flatten(1), p["prediction_net.policy_fc.weight"], p["prediction_net.policy_fc.bias"])
        v = F.relu(self._bn(self._conv(h, "prediction_net.value_conv.weight", 0), "prediction_net.value_bn"))
        v = F.relu(F.linear(v.flatten(1), p["prediction_net.value_fc1.weight"], p["prediction_net.value_fc1.bias"]))
        vl = F.linear(v, p["prediction_net.value_fc2.weight"], p["prediction_net.value_fc2.bias"])
        return logits, self._support(vl)

    def dynamics(self, h, a):
        p = self.p
        plane = F.one_hot(a.long(), self.A).float().view(-1, 1, self.H, self.H)
        emb = F.conv2d(plane, p["dynamics_net.action_embed_conv.weight"])
        x = torch.cat((h, emb), 1)
        x = F.relu(self._bn(self._conv(x, "dynamics_net.conv.weight"), "dynamics_net.bn"))
        x = self._blocks(x, "dynamics_net")
        r = F.relu(F.linear(x.flatten(1), p["dynamics_net.reward_fc.0.weight"], p["dynamics_net.reward_fc.0.bias"]))
        rl = F.linear(r, p["dynamics_net.reward_fc.2.weight"], p["dynamics_net.reward_fc.2.bias"])
        return x, self._support(rl)

    # ---------------------------------------------------------------- engine backend interface
    def initial(self, obs, out_slot, logits, value, stream):
        rows = torch.nonzero(out_slot >= 0).flatten()
        if rows.numel() == 0:
            return
        h = self.representation(obs[rows])
        lg, v = self.prediction(h)
        self.pool[out_slot[rows].long()] = h
        logits[rows] = lg
        value[rows] = v

    def recurrent(self, in_slot, action, out_slot, logits, value, reward, stream):
        rows = torch.nonzero(out_slot >= 0).flatten()
        if rows.numel() == 0:
            return
        h, r = self.dynamics(self.pool[in_slot[rows].long()], action[rows])
        lg, v = self.prediction(h)
        self.pool[out_slot[rows].long()] = h
        logits[rows] = lg
        value[rows] = v
        reward[rows] = r
