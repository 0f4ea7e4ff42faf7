"""Load-time weight folding shared by the LNet / ENet / DNet engines."""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC, ConvW


def conv_weight(sd, p):
    """Effective conv weight: eval spectral norm W/(u.(W v)) when the layer is spectral-normed
    (torch.nn.utils.spectral_norm on base_blocks.py:72-76 layers), else the plain weight."""
    if p + "weight_orig" in sd:
        w = sd[p + "weight_orig"].float()
        u, v = sd[p + "weight_u"].float(), sd[p + "weight_v"].float()
        return w / torch.dot(u, torch.mv(w.reshape(w.shape[0], -1), v))
    return sd[p + "weight"].float()


def make_conv(sd, p, device, **kw) -> ConvW:
    return ConvW(conv_weight(sd, p), sd.get(p + "bias"), device, **kw)


def bn_tuple(sd, p):
    return (sd[p + "weight"], sd[p + "bias"], sd[p + "running_mean"], sd[p + "running_var"])


class AdainBank:
    """Every ADAIN head (base_blocks.py:127-157) conditioned on the same vector z, evaluated in two
    launches: one GEMM for all ``mlp_shared`` layers (+ReLU), then one segmented GEMV for all
    gamma/beta heads.  A *group* is a set of ADAINs applied to adjacent channel ranges of one
    tensor (FineADAINLama's bn_l + bn_g), so its gamma/beta come out as one contiguous vector."""

    NH = 128

    def __init__(self, feature_nc: int):
        self.feature_nc = feature_nc
        self.w1, self.b1 = [], []
        self.cols = []          # per output column: (layer index, source tensor, row)
        self.groups = []        # (offset, channels)
        self.total = 0

    def add_group(self, sd, members):
        """members: [(prefix, channels)] in channel order.  Returns the group id."""
        ct = sum(c for _, c in members)
        off = self.total
        g_w, g_b, b_w, b_b, segs = [], [], [], [], []
        for prefix, c in members:
            li = len(self.w1)
            self.w1.append(sd[prefix + "mlp_shared.0.weight"].float())
            self.b1.append(sd[prefix + "mlp_shared.0.bias"].float())
            g_w.append(sd[prefix + "mlp_gamma.weight"].float())
            g_b.append(sd[prefix + "mlp_gamma.bias"].float())
            b_w.append(sd[prefix + "mlp_beta.weight"].float())
            b_b.append(sd[prefix + "mlp_beta.bias"].float())
            segs.append(torch.full((c,), li, dtype=torch.int32))
        self.cols.append((torch.cat(g_w + b_w, 0), torch.cat(g_b + b_b, 0), torch.cat(segs + segs, 0)))
        self.groups.append((off, ct))
        self.total += 2 * ct
        return len(self.groups) - 1

    def build(self, device):
        w1 = torch.cat(self.w1, 0)
        self.layer1 = ConvW(w1, torch.cat(self.b1, 0), device)
        w2 = torch.cat([c[0] for c in self.cols], 0)            # [total, NH]
        self.w2t = w2.t().contiguous().to(device)               # [NH, total]
        self.b2 = torch.cat([c[1] for c in self.cols], 0).contiguous().to(device)
        self.seg = torch.cat([c[2] for c in self.cols], 0).contiguous().to(device)
        self.device = device
        return self

    def run(self, ctx, z: NHWC):
        """z: NHWC [B,1,1,feature_nc] -> params [B, total]."""
        b = z.n
        hid = NHWC.empty(b, 1, 1, self.layer1.cout, self.device)
        ops.conv2d(ctx, z, self.layer1, hid, act=ops.ACT_RELU)
        out = ops.empty((b, self.total), self.device)
        ops.adain_params(ctx, hid.t.view(b, -1), self.NH, self.w2t, self.b2, self.seg, out)
        return out

    def gamma_beta(self, gid, params):
        """(gamma, beta): [B, ct] row views of a group in ``params`` (a ``run`` output; the bank
        itself keeps no per-forward state, so lanes can share it)."""
        off, ct = self.groups[gid]
        return params[:, off: off + ct], params[:, off + ct: off + 2 * ct]
