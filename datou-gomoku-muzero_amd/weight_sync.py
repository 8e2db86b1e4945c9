"""Weight exchange between self-play ranks (the only exchange of the self-play tier).

The reference pushes ``ModelWeightsUpdate(weights=state_dict)`` from the trainer to its single
inference server every MODEL_UPDATE_INTERVAL steps (workers.py:587-593).  With one self-play
process per GPU the same state_dict reaches every rank by ONE broadcast of a flat fp32 bucket
(RCCL over xGMI with the "nccl" backend, or gloo on CPU): 6.9 M parameters = 27 MB per update.
Each rank then hot-swaps it into its ``GomokuNetHip`` (``load_state_dict``)."""
import numpy as np
import torch


def broadcast_state_dict(sd, src=0, device=None, group=None):
    """Broadcast ``sd`` (name -> array/tensor; only rank ``src``'s values matter, the others pass
    any dict with the same keys and shapes) as one flat float32 bucket.  Returns name -> float32
    tensor on ``device`` (default: cuda if available else cpu), identical on every rank."""
    import torch.distributed as dist
    dev = torch.device(device) if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
    keys = sorted(sd)
    shapes = [tuple(np.shape(sd[k])) for k in keys]
    sizes = [int(np.prod(s)) if len(s) else 1 for s in shapes]
    flat = torch.empty(sum(sizes), dtype=torch.float32, device=dev)
    rank = dist.get_rank(group) if group is not None else dist.get_rank()
    if rank == src:
        off = 0
        for k, n in zip(keys, sizes):
            flat[off:off + n] = torch.as_tensor(np.asarray(sd[k] if not torch.is_tensor(sd[k]) else sd[k].detach().cpu(),
                                                           dtype=np.float32)).reshape(-1).to(dev)
            off += n
    dist.broadcast(flat, src, group=group)
    out, off = {}, 0
    for k, s, n in zip(keys, shapes, sizes):
        out[k] = flat[off:off + n].view(s)
        off += n
    return out
