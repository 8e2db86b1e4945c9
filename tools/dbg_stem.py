"""Debug: the dynamics stem on the HIP conv (gmz_conv3x3_forward_stamp) against float32 PyTorch convolutions of the
same f16 operands: the hidden-plane conv alone, the stamp alone, and the whole 144-channel conv."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from datou_gomoku_muzero_amd import trainer as T, _lib  # noqa: E402

for H in (9, 15):
    torch.manual_seed(0)
    n = 24
    h = torch.randn(n, 128, H, H, device="cuda").relu().half().contiguous(memory_format=torch.channels_last)
    W = (torch.randn(128, 144, 3, 3, device="cuda") / 30).contiguous(memory_format=torch.channels_last)
    we = torch.randn(16, 1, 1, 1, device="cuda")
    a = torch.randint(0, H * H, (n,), device="cuda")
    a[:3] = torch.tensor([0, H * H - 1, H - 1], device="cuda")
    W16, e16 = W.half().float(), we.half().float().reshape(16)
    plane = F.one_hot(a, H * H).float().reshape(n, 1, H, H)
    emb = plane * e16.reshape(1, 16, 1, 1)
    ref_h = F.conv2d(h.float(), W16[:, :128], padding=1)
    ref_full = F.conv2d(torch.cat([h.float(), emb], 1), W16, padding=1)
    L = _lib.load()
    pk = T._packed_conv_weight(W[:, :128], torch.float16, 0, parent=W)
    y0 = torch.empty_like(h)
    _lib.check(L.gmz_conv3x3_forward(1, H, _lib.ptr(h), _lib.ptr(pk), _lib.ptr(y0), n, _lib.stream_ptr()))
    w2 = W[:, 128:].half().float().reshape(128, 16, 9)
    table = torch.einsum("oct,c->to", w2, e16).contiguous()
    y1 = torch.empty_like(h)
    a32 = a.to(torch.int32)
    _lib.check(L.gmz_conv3x3_forward_stamp(1, H, _lib.ptr(h), _lib.ptr(pk), _lib.ptr(y1), n, None, None, _lib.ptr(a32),
                                           _lib.ptr(table), _lib.stream_ptr()))
    torch.cuda.synchronize()
    sc = float(ref_full.abs().max())
    print("H=%d  |hidden conv - ref| %.4g  |stamp conv - ref full| %.4g  |stamp part - ref stamp part| %.4g  (scale %.3g)"
          % (H, float((y0.float() - ref_h).abs().max()), float((y1.float() - ref_full).abs().max()),
             float(((y1.float() - y0.float()) - (ref_full - ref_h)).abs().max()), sc))
    # where the stamp lands: positions with a non-zero stamp difference, board 0
    d = (ref_full - ref_h)[0].abs().sum(0)
    dh = (y1.float() - y0.float())[0].abs().sum(0)
    print("  ref stamp cells board0:", torch.nonzero(d > 1e-3).tolist()[:9], " hip:", torch.nonzero(dh > 1e-2).tolist()[:9])
