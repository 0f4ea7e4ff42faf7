import sys, torch, torch.nn.functional as F
sys.path.insert(0, '.')
import s2v_import
from s2v_amd import ops
from s2v_amd.ops import NHWC, ConvW
ctx = ops.Ctx('cuda')
g = torch.Generator().manual_seed(0)
n, cin, h, w, cout = 2, 32, 10, 10, 64
wt = torch.rand(cout, cin, 3, 3, generator=g) - 0.5
x = torch.rand(n, cin, h, w, generator=g) * 2 - 1
s = torch.rand(n, cin, generator=g) + 0.5
cw = ConvW(wt, None, 'cuda', padding=1)
xv = NHWC(x.permute(0, 2, 3, 1).contiguous().cuda())
for name, kw, ref in [
    ('plain', {}, F.conv2d(x, wt, padding=1)),
    ('scale', dict(in_scale=s.cuda()), F.conv2d(x * s[:, :, None, None], wt, padding=1)),
    ('lrelu', dict(pre_act=ops.ACT_LRELU, pre_alpha=0.1), F.conv2d(F.leaky_relu(x, 0.1), wt, padding=1)),
    ('both', dict(in_scale=s.cuda(), pre_act=ops.ACT_LRELU, pre_alpha=0.1), F.conv2d(F.leaky_relu(x * s[:, :, None, None], 0.1), wt, padding=1)),
]:
    y = NHWC.empty(n, h, w, cout, 'cuda')
    ops.conv2d(ctx, xv, cw, y, **kw)
    got = y.t.permute(0, 3, 1, 2).cpu()
    p = ops._lib.ConvParams()
    print(name, (got - ref).abs().max().item(), flush=True)
