"""MI355X-native per-frame lip-sync inference path (DNet -> LNet/ENet -> GFPGAN/GPEN-512, mel).

Import name ``s2v_amd`` (see ``s2v_import.py`` at the repo root).  The compute path is the
C-ABI library ``libs2v.so`` built from ``csrc/`` (HIP, gfx950); PyTorch provides device memory,
streams and torch.distributed only.
"""
__version__ = "0.1.0"
