"""Parameter layout of the RealESRNet super-resolution net (third_part/GPEN/sr_model/rrdbnet_arch.py).

Only the modules and their ``state_dict`` keys / shapes are declared here (the forward runs on
libs2v, engine/rrdb.py); tests/golden/rrdbnet_keys.json pins the layout against the reference.
"""
from __future__ import annotations

from torch import nn


class ResidualDenseBlockParams(nn.Module):
    """rrdbnet_arch.py:8-38: five 3x3 convs over the growing concatenation [x, x1, .., x4]."""

    def __init__(self, num_feat=64, num_grow_ch=32):
        super().__init__()
        for i in range(1, 5):
            setattr(self, f"conv{i}", nn.Conv2d(num_feat + (i - 1) * num_grow_ch, num_grow_ch, 3, 1, 1))
        self.conv5 = nn.Conv2d(num_feat + 4 * num_grow_ch, num_feat, 3, 1, 1)


class RRDBParams(nn.Module):
    """rrdbnet_arch.py:41-61."""

    def __init__(self, num_feat, num_grow_ch=32):
        super().__init__()
        self.rdb1 = ResidualDenseBlockParams(num_feat, num_grow_ch)
        self.rdb2 = ResidualDenseBlockParams(num_feat, num_grow_ch)
        self.rdb3 = ResidualDenseBlockParams(num_feat, num_grow_ch)


class RRDBNetParams(nn.Module):
    """rrdbnet_arch.py:63-116: RRDBNet(num_in_ch, num_out_ch, scale, num_feat, num_block, num_grow_ch).
    scale 2 / 1 feed a pixel-unshuffled input (x4 / x16 channels) to conv_first (:88-92)."""

    def __init__(self, num_in_ch, num_out_ch, scale=4, num_feat=64, num_block=23, num_grow_ch=32):
        super().__init__()
        if scale not in (1, 2, 4):
            raise ValueError(f"RRDBNet: scale must be 1, 2 or 4, got {scale}")
        self.scale = scale
        self.num_in_ch, self.num_out_ch = num_in_ch, num_out_ch
        self.num_feat, self.num_block, self.num_grow_ch = num_feat, num_block, num_grow_ch
        cin = num_in_ch * {4: 1, 2: 4, 1: 16}[scale]
        self.conv_first = nn.Conv2d(cin, num_feat, 3, 1, 1)
        self.body = nn.Sequential(*[RRDBParams(num_feat, num_grow_ch) for _ in range(num_block)])
        self.conv_body = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_up1 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_up2 = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_hr = nn.Conv2d(num_feat, num_feat, 3, 1, 1)
        self.conv_last = nn.Conv2d(num_feat, num_out_ch, 3, 1, 1)


def rrdb_gflop(h: int, w: int, scale: int, num_feat=32, num_block=23, num_grow_ch=32, num_in_ch=3, num_out_ch=3):
    """Algorithmic GFLOP (2 * MAC of every conv) of one RRDBNet forward on an h x w input."""
    r = {4: 1, 2: 2, 1: 4}[scale]
    p = (h // r) * (w // r)                       # body resolution
    mac = p * 9 * num_in_ch * r * r * num_feat
    rdb = sum(9 * (num_feat + i * num_grow_ch) * num_grow_ch for i in range(4)) + 9 * (num_feat + 4 * num_grow_ch) * num_feat
    mac += p * (3 * num_block * rdb + 9 * num_feat * num_feat)
    mac += 4 * p * 9 * num_feat * num_feat + 16 * p * 9 * num_feat * (2 * num_feat + num_out_ch)
    return 2.0 * mac / 1e9
