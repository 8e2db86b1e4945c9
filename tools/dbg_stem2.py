"""Debug: _DynStemHIP inside the dynamics module vs MIOpen's 144-channel conv, stage by stage (9x9 and 15x15)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from datou_gomoku_muzero_amd import trainer as T  # noqa: E402

rel = lambda x, y: float((x.float() - y.float()).norm() / (x.float().norm() + 1e-12))  # noqa: E731
for size in (9, 15):
    torch.manual_seed(3)
    B = 48
    dyn0 = T._Dynamics(128, size, 1, 64, 3).cuda().to(memory_format=torch.channels_last)
    h = torch.randn(B, 128, size, size, device="cuda").relu().half().contiguous(memory_format=torch.channels_last)
    a = torch.randint(0, size * size, (B,), device="cuda")
    mask = torch.rand(B, device="cuda") > 0.2
    m8 = mask.contiguous().view(torch.uint8)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        plane = F.one_hot(a, size * size).to(h.dtype).reshape(B, 1, size, size)
        emb = T._conv1x1(dyn0.action_embed_conv, plane).to(h.dtype).contiguous(memory_format=torch.channels_last)
        x = torch.cat((h, emb), dim=1)
        y_ref = dyn0.conv(x)
        y_hip = T._DynStemHIP.apply(h, dyn0.conv.weight, dyn0.action_embed_conv.weight, a, None, None)
        st = T._conv_stats_buffer(B, h.device)
        y_hip2 = T._DynStemHIP.apply(h, dyn0.conv.weight, dyn0.action_embed_conv.weight, a, m8, st[0])
        W16 = dyn0.conv.weight.detach().half().float()
        y32 = F.conv2d(x.float(), W16, padding=1)
        y32h = F.conv2d(h.float(), W16[:, :128], padding=1)
    torch.cuda.synchronize()
    print("size %d: vs fp32 conv of the same f16 operands: MIOpen %.3g  HIP %.3g  (hidden part only %.3g); emb max %.3g"
          % (size, rel(y32, y_ref), rel(y32, y_hip), rel(y32, y32h), float(emb.abs().max())))
    dd = (y_hip.float() - y32).abs()[0].sum(0)
    print("   board0 action", int(a[0]), "cells where HIP differs:", torch.nonzero(dd > 1e-2).tolist()[:12])
    print("size %d: stem conv rel %.3g (no stats) %.3g (stats)  y_ref %s %s  y_hip %s %s" % (
        size, rel(y_ref, y_hip), rel(y_ref, y_hip2), y_ref.dtype, tuple(y_ref.stride()), y_hip.dtype, tuple(y_hip.stride())))
    d1, d2 = copy.deepcopy(dyn0), copy.deepcopy(dyn0)
    d1.train(); d2.train()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
        b_ref = T._bn_act(d1.bn, y_ref, mask)
        y_hip2._gmz_bnstats = st
        b_hip = T._bn_act(d2.bn, y_hip2, mask)
    torch.cuda.synchronize()
    print("   bn out rel %.3g (masked rows %.3g)  running_mean rel %.3g  var rel %.3g" % (
        rel(b_ref, b_hip), rel(b_ref[mask], b_hip[mask]), rel(d1.bn.running_mean, d2.bn.running_mean),
        rel(d1.bn.running_var, d2.bn.running_var)))
    outs = {}
    for hip in (False, True):
        T.DYN_STEM_HIP = hip
        d = copy.deepcopy(dyn0)
        d.train()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            nxt, r = d(h, a, mask=mask)
        outs[hip] = nxt
    # the same stages composed by hand from each stem output (fresh modules): block input and output
    stages = {}
    for name, y in (("ref", y_ref), ("hip", y_hip2)):
        d = copy.deepcopy(dyn0)
        d.train()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.float16):
            if name == "hip":
                y._gmz_bnstats = T._conv_stats_buffer(B, h.device)  # stale on purpose? no: recompute below
                y = T._DynStemHIP.apply(h, d.conv.weight, d.action_embed_conv.weight, a, m8, y._gmz_bnstats[0])
                y._gmz_bnstats = stt = None
            x0 = T._bn_act(d.bn, y, mask)
            x1 = d.resblocks[0](x0, mask)
        stages[name] = (x0, x1)
    torch.cuda.synchronize()
    print("   module out rel %.3g (masked %.3g) | by hand: stem-bn rel %.3g, block rel %.3g | module-hip vs hand-hip %.3g"
          % (rel(outs[False], outs[True]), rel(outs[False][mask], outs[True][mask]), rel(stages["ref"][0], stages["hip"][0]),
             rel(stages["ref"][1], stages["hip"][1]), rel(outs[True], stages["hip"][1])))
