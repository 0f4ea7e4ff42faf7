"""Drop-in model API of the reference's ``models`` package (models/__init__.py, LNet.py,
ENet.py, DNet.py): same class names, constructor arguments, ``state_dict`` keys, forward
signatures and return values; the forward runs on libs2v (HIP, gfx950).

    from s2v_amd.models import LNet, ENet, DNet, load_network, load_DNet
    model = load_network(args)            # ENet(lnet=LNet()) with checkpoints, eval mode
    pred, low = model.cuda()(mel, img, ref)   # inference.py:266

Weights are folded and packed for the device on the first forward (spectral norm, BatchNorm,
modulation layout); call ``refresh()`` after mutating parameters in place.  Inputs must be CUDA
fp32 tensors: there is no CPU path (the checker for CPU is oracle/, test infrastructure).
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC
from . import arch, enhancer_arch, face3d_arch, parse_arch, retinaface_arch, sr_arch


def _fold5(x, dim):
    return torch.cat([x.select(dim, i) for i in range(x.shape[dim])], 0)


def _need_cuda(*ts):
    for t in ts:
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise RuntimeError("s2v_amd models run on the HIP device only: move the module inputs to 'cuda' "
                               "(there is no CPU fallback on the product path)")


class _EngineMixin:
    """Device engines of a module: the folded / packed weights (one engine per device, read-only
    after it is built) and one ``ops.Ctx`` per *lane* — the mutable device state of a forward
    (workspace, side streams, noise counters).  Forwards on different lanes of one module can run
    concurrently (e.g. two captured graphs replayed on two streams); forwards on one lane must not
    overlap.  Copies of a module (copy.copy / deepcopy / pickle) get fresh engines: an engine and its
    lanes are never shared between two modules."""
    _engine_cls = None
    _prefix = ""

    def _engine(self, device, lane: int = 0):
        cache = self.__dict__.setdefault("_s2v_engines", {})
        key = str(device)
        if key not in cache:
            sd = {k: v.detach().to("cpu") for k, v in self.state_dict().items()}
            cache[key] = (self._build_engine(sd, device), {})
        eng, lanes = cache[key]
        if lane not in lanes:
            lanes[lane] = ops.Ctx(device)
        ctx = lanes[lane]
        ctx.keep.clear()        # a new forward on this lane: the previous one's side branches have been joined
        return eng, ctx

    def refresh(self):
        self.__dict__.pop("_s2v_engines", None)
        return self

    def _guarded(self, ctx, fn):
        """Run one eager forward ``fn()`` on lane ``ctx`` under the f16x3 range guard (ops): the
        engine's first forward calibrates every layer's activation pre-scale (one host sync, re-run when
        a layer needed a scale); every eager forward then reads the lane's non-finite flag when it returns
        (one host sync) and, when a launch overflowed, runs again in bf16x3 — so an out-of-range batch
        returns correct outputs instead of silent inf / NaN.  Inside a graph capture the forward is only
        recorded (a replayed graph's flag is read by its caller: pipeline.LipSyncPipeline.run)."""
        if not ops.guard_active() or (ctx.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            return fn()
        eng = self._s2v_engines[str(ctx.device)][0]
        done = eng.__dict__.setdefault("_calibrated", set())
        calibrating = ops.PRECISION not in done
        if calibrating:
            ops.begin_calibration(ctx)
        out = fn()
        state = ops.end_forward(ctx, calibrating)
        done.add(ops.PRECISION)
        for _ in range(ops.CALIB_PASSES):
            if state not in ("scaled", "recalibrate"):
                break
            # "recalibrate": an upstream overflow hid some layer's range; measure it again behind the
            # layers scaled so far.  "scaled": run again with the new pre-scales.
            recal = state == "recalibrate"
            if recal:
                ops.begin_calibration(ctx)
            out = fn()
            state = ops.end_forward(ctx, recal)
        if state:                               # overflow, or calibration still unsettled after the passes
            with ops.precision("bf16x3"):
                out = fn()
            ctx.reruns += 1
        return out

    def __getstate__(self):
        state = dict(self.__dict__)
        state.pop("_s2v_engines", None)
        return state

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self.refresh()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)


class LNet(_EngineMixin, arch.LNetParams):
    """models/LNet.py:80-139."""

    def _build_engine(self, sd, device):
        from ..engine.lnet import LNetEngine
        return LNetEngine(sd, device)

    @torch.no_grad()
    def forward(self, audio_sequences, face_sequences, *, lane: int = 0):
        """``lane`` (keyword-only, not in the reference): the execution lane (see _EngineMixin)."""
        _need_cuda(audio_sequences, face_sequences)
        b = audio_sequences.size(0)
        five = face_sequences.dim() > 4
        if five:
            audio_sequences = _fold5(audio_sequences, 1)
            face_sequences = _fold5(face_sequences, 2)
        eng, ctx = self._engine(face_sequences.device, lane)
        n, _, h, w = face_sequences.shape
        dev = face_sequences.device
        x6 = NHWC.empty(n, h, w, 6, dev)
        ops.nchw_to_nhwc(ctx, face_sequences.float(), x6)
        lo = NHWC.empty(n, h, w, 3, dev)
        self._guarded(ctx, lambda: eng.forward(ctx, audio_sequences.float(), x6, lo))
        out = torch.empty((n, 3, h, w), device=dev)
        ops.nhwc_to_nchw(ctx, lo, out)
        if five:
            out = torch.stack(torch.split(out, b, 0), 2)
        return out


class ENet(_EngineMixin, arch.ENetParams):
    """models/ENet.py:8-139; ``lnet`` is held as ``low_res`` like the reference."""

    def __init__(self, num_style_feat=512, lnet=None, concat=False):
        super().__init__(num_style_feat=num_style_feat, lnet=lnet if lnet is not None else LNet(), concat=concat)

    def _build_engine(self, sd, device):
        from ..engine.enet import ENetEngine
        return ENetEngine(sd, device)

    @torch.no_grad()
    def forward(self, audio_sequences, face_sequences, gt_sequences, noises=None, *, lane: int = 0):
        """``lane`` (keyword-only, not in the reference): the execution lane (see _EngineMixin)."""
        _need_cuda(audio_sequences, face_sequences, gt_sequences)
        b = audio_sequences.size(0)
        five = face_sequences.dim() > 4
        if five:
            audio_sequences = _fold5(audio_sequences, 1)
            face_sequences = _fold5(face_sequences, 2)
            gt_sequences = _fold5(gt_sequences, 2)
        eng, ctx = self._engine(face_sequences.device, lane)
        n = face_sequences.shape[0]
        dev = face_sequences.device
        out = torch.empty((n, 3, 384, 384), device=dev)
        low = torch.empty((n, 3, 96, 96), device=dev)
        self._guarded(ctx, lambda: eng.forward(ctx, audio_sequences.float(), face_sequences.float(),
                                               gt_sequences.float(), out, low, noises))
        if five:
            out = torch.stack(torch.split(out, b, 0), 2)
            # F.interpolate(low_res_img, outputs.size()[3:]) (default mode 'nearest', ENet.py:134)
            up = torch.empty((n, 3) + tuple(out.shape[3:]), device=dev)
            ops.resize(ctx, low, 0, tuple(low.shape), low.stride(), up, 0, tuple(out.shape[3:]), up.stride(), mode=1)
            low = torch.stack(torch.split(up, b, 0), 2)
        return out, low


class DNet(_EngineMixin, arch.DNetParams):
    """models/DNet.py:13-28."""

    def _build_engine(self, sd, device):
        from ..engine.dnet import DNetEngine
        return DNetEngine(sd, device)

    @torch.no_grad()
    def forward(self, input_image, driving_source, stage=None, *, lane: int = 0):
        """``lane`` (keyword-only, not in the reference): the execution lane (see _EngineMixin)."""
        _need_cuda(input_image, driving_source)
        eng, ctx = self._engine(input_image.device, lane)
        return self._guarded(ctx, lambda: eng.forward(ctx, input_image.float(), driving_source.float(), stage=stage))


# ----------------------------------------------------------------------------- enhancers
class GFPGANv1Clean(_EngineMixin, enhancer_arch.GFPGANv1CleanParams):
    """third_part/GFPGAN/gfpgan/archs/gfpganv1_clean_arch.py:154-324 (GFPGANer: out_size=512,
    channel_multiplier=2, different_w=True, input_is_latent=True, sft_half=True)."""

    def _build_engine(self, sd, device):
        from ..engine.gfpgan import GFPGANEngine
        return GFPGANEngine(sd, device, self.num_style_feat, self.sft_half, self.different_w, self.input_is_latent)

    @torch.no_grad()
    def forward(self, x, return_latents=False, return_rgb=True, randomize_noise=True):
        """-> (image [B,3,S,S], list of U-Net RGB images) like the reference (:296-324)."""
        _need_cuda(x)
        eng, ctx = self._engine(x.device)
        out = torch.empty_like(x, dtype=torch.float32)
        return self._guarded(ctx, lambda: eng.forward(ctx, x.float(), out, return_rgb=return_rgb,
                                                      randomize_noise=randomize_noise))


class FullGenerator(_EngineMixin, enhancer_arch.FullGeneratorParams):
    """third_part/GPEN/face_model/gpen_model.py:583-630 (GPEN-BFR-512: FullGenerator(512, 512, 8, 2))."""

    def _build_engine(self, sd, device):
        from ..engine.gpen import GPENEngine
        return GPENEngine(sd, device, n_mlp=self.generator.n_mlp)

    @torch.no_grad()
    def forward(self, inputs, return_latents=False, inject_index=None, truncation=1, truncation_latent=None,
                input_is_latent=False):
        """-> (image, None) or (image, latent [B, n_latent, 512]) (Generator.forward, :450-512)."""
        _need_cuda(inputs)
        if truncation < 1:
            raise NotImplementedError("FullGenerator: truncation < 1 is not on the GPEN inference path "
                                      "(face_gan.py:40 calls model(img_t))")
        eng, ctx = self._engine(inputs.device)
        out = torch.empty_like(inputs, dtype=torch.float32)
        lat = torch.empty((inputs.shape[0], self.style_dim), device=inputs.device) if return_latents else None
        self._guarded(ctx, lambda: eng.forward(ctx, inputs.float(), out, input_is_latent=input_is_latent,
                                               latent_out=lat))
        if return_latents:
            return out, lat.unsqueeze(1).expand(-1, self.generator.n_latent, -1)
        return out, None


class ParseNet(_EngineMixin, parse_arch.ParseNetParams):
    """third_part/GPEN/face_parse/parse_model.py:21-75 (FaceParse: ParseNet(512, 512, 32, 64, 19,
    norm_type='bn', relu_type='LeakyReLU', ch_range=[32, 256]), eval mode)."""

    def _build_engine(self, sd, device):
        from ..engine.parsenet import ParseNetEngine
        return ParseNetEngine(sd, device, self.describe())

    @torch.no_grad()
    def forward(self, x):
        """x [B,3,H,W] in [-1,1] -> (out_mask [B,parsing_ch,H,W], out_img [B,3,H,W]) (:69-75)."""
        _need_cuda(x)
        eng, ctx = self._engine(x.device)
        b, _, h, w = x.shape
        mask = torch.empty((b, self.parsing_ch, h, w), device=x.device)
        img = torch.empty((b, 3, h, w), device=x.device)
        return self._guarded(ctx, lambda: eng.forward(ctx, x.float(), mask, img))


class RRDBNet(_EngineMixin, sr_arch.RRDBNetParams):
    """third_part/GPEN/sr_model/rrdbnet_arch.py:63-116 (RealESRNet: RRDBNet(3, 3, num_feat=32,
    num_block=23, num_grow_ch=32, scale=2|4), real_esrnet.py:22)."""

    def _build_engine(self, sd, device):
        from ..engine.rrdb import RRDBEngine
        return RRDBEngine(sd, device, self.scale, self.num_in_ch)

    @torch.no_grad()
    def forward(self, x):
        """x [B, num_in_ch, H, W] -> [B, num_out_ch, scale H, scale W] (H, W multiples of the
        pixel-unshuffle factor for scale 2 / 1, as arch_util.pixel_unshuffle asserts)."""
        _need_cuda(x)
        eng, ctx = self._engine(x.device)
        r = eng.r
        if x.shape[2] % r or x.shape[3] % r:
            raise RuntimeError(f"RRDBNet(scale={self.scale}): input size {tuple(x.shape[2:])} must be a multiple of {r}")
        b, _, h, w = x.shape
        out = torch.empty((b, self.num_out_ch, h * self.scale, w * self.scale), device=x.device)
        return self._guarded(ctx, lambda: eng.forward(ctx, x.float(), out))


# ----------------------------------------------------------------------------- loaders
class RetinaFace(_EngineMixin, retinaface_arch.RetinaFaceParams):
    """third_part/GPEN/face_detect/facemodels/retinaface.py:47-125 with cfg_re50 (the only
    configuration RetinaFaceDetection builds, retinaface_detection.py:19-27)."""

    def __init__(self, cfg=None, phase="test"):
        cfg = retinaface_arch.CFG_RE50 if cfg is None else cfg
        if cfg.get("name", "Resnet50") != "Resnet50":
            raise NotImplementedError("RetinaFace: only the Resnet50 backbone (cfg_re50) is on the GPEN path")
        super().__init__(cfg)
        self.phase = phase

    def _build_engine(self, sd, device):
        from ..engine.retinaface import RetinaFaceEngine
        return RetinaFaceEngine(sd, device)

    def head_maps(self, x4: NHWC):
        """x4: NHWC [B,H,W,4] fp32 (BGR minus means, channel 3 zero) -> per-level fused head maps."""
        eng, ctx = self._engine(x4.t.device)
        return self._guarded(ctx, lambda: eng.forward_maps(ctx, x4)), ctx

    @torch.no_grad()
    def forward(self, inputs):
        """inputs [B,3,H,W] fp32 (BGR minus (104, 117, 123)) -> (loc [B,P,4], conf [B,P,2] softmaxed in
        phase 'test' (raw logits in 'train'), landms [B,P,10]) (retinaface.py:108-125)."""
        _need_cuda(inputs)
        b, c, h, w = inputs.shape
        if c != 3:
            raise RuntimeError(f"RetinaFace: expected 3 input channels, got {c}")
        eng, ctx = self._engine(inputs.device)
        x4 = NHWC.empty(b, h, w, 4, inputs.device)
        ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, inputs.float(), x4.slice(0, 3))
        maps = self._guarded(ctx, lambda: eng.forward_maps(ctx, x4))
        if self.phase != "test":
            return eng.split_heads(maps)
        return retina_outputs(ctx, maps, h, w)


def retina_outputs(ctx, maps, im_h, im_w):
    """Head maps -> (loc, softmax conf, landms) via s2v_retina_split (phase 'test')."""
    import ctypes
    n, dev = maps[0].n, maps[0].t.device
    P = sum(2 * m.h * m.w for m in maps)
    loc = torch.empty((n, P, 4), device=dev)
    conf = torch.empty((n, P, 2), device=dev)
    lms = torch.empty((n, P, 10), device=dev)
    heads = (ctypes.c_void_p * 3)(*[m.ptr for m in maps])
    hs = (ctypes.c_int * 3)(*[m.h for m in maps])
    ws = (ctypes.c_int * 3)(*[m.w for m in maps])
    ops.check(ctx.lib.s2v_retina_split(heads, hs, ws, maps[0].cs, im_h, im_w, n, loc.data_ptr(), conf.data_ptr(),
                                       lms.data_ptr(), ctx.stream), "s2v_retina_split")
    return loc, conf, lms


class ReconNetWrapper(_EngineMixin, face3d_arch.ReconNetWrapperParams):
    """third_part/face3d/models/networks.py:66-105 with net_recon='resnet50', use_last_fc=False (the
    configuration load_face3d_net builds, futils/inference_utils.py:261-267)."""

    def _build_engine(self, sd, device):
        from ..engine.face3d import ReconNetEngine
        return ReconNetEngine(sd, device)

    def forward_nhwc(self, x4: NHWC) -> torch.Tensor:
        """x4: NHWC [B,H,W,4] fp32 (RGB / 255, channel 3 zero) -> coefficients [B, 257] (view)."""
        eng, ctx = self._engine(x4.t.device)
        return self._guarded(ctx, lambda: eng.forward(ctx, x4))

    @torch.no_grad()
    def forward(self, x):
        """x [B,3,H,W] fp32 (RGB in [0, 1], facing.py:120) -> [B, 257] =
        flatten(cat(id 80, exp 64, tex 80, angle 3, gamma 27, tx,ty 2, tz 1)) (networks.py:98-105)."""
        _need_cuda(x)
        b, c, h, w = x.shape
        if c != 3:
            raise RuntimeError(f"ReconNetWrapper: expected 3 input channels, got {c}")
        eng, ctx = self._engine(x.device)
        x4 = NHWC.empty(b, h, w, 4, x.device)
        ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, x.float(), x4.slice(0, 3))
        return self._guarded(ctx, lambda: eng.forward(ctx, x4)).clone()


def define_net_recon(net_recon, use_last_fc=False, init_path=None):
    """networks.py:59-60."""
    return ReconNetWrapper(net_recon, use_last_fc=use_last_fc, init_path=init_path)


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def load_checkpoint(path, model):
    """models/__init__.py:12-27: ``state_dict`` entry, ``low_res`` keys skipped, ``module.``
    stripped, strict=False; a bare state_dict file is loaded as-is."""
    print("Load checkpoint from: {}".format(path))
    ckpt = _load(path)
    if isinstance(ckpt, dict) and "state_dict" in ckpt and "arcface" not in path:
        sd = {k.replace("module.", ""): v for k, v in ckpt["state_dict"].items() if "low_res" not in k}
        model.load_state_dict(sd, strict=False)
    else:
        model.load_state_dict(ckpt)
    return model


def load_network(args):
    """models/__init__.py:29-35."""
    lnet = load_checkpoint(args.LNet_path, LNet())
    enet = ENet(lnet=lnet)
    return load_checkpoint(args.ENet_path, enet).eval()


def load_DNet(args):
    """models/__init__.py:50-56: DNet weights from ckpt['net_G_ema'], strict=False."""
    dnet = DNet()
    print("Load checkpoint from: {}".format(args.DNet_path))
    ckpt = _load(args.DNet_path)
    dnet.load_state_dict(ckpt["net_G_ema"], strict=False)
    return dnet.eval()


def load_gfpgan(path, **kw):
    """gfpgan/utils.py:40-50, :87-93: GFPGANv1Clean(arch='clean', channel_multiplier=2) with the
    ``params_ema`` (else ``params``) weights, strict=True."""
    cfg = dict(out_size=512, num_style_feat=512, channel_multiplier=2, decoder_load_path=None, fix_decoder=False,
               num_mlp=8, input_is_latent=True, different_w=True, narrow=1, sft_half=True)
    cfg.update(kw)
    net = GFPGANv1Clean(**cfg)
    ckpt = _load(path)
    key = "params_ema" if "params_ema" in ckpt else "params"
    net.load_state_dict(ckpt[key], strict=True)
    return net.eval()


def load_gpen(path, size=512, channel_multiplier=2, narrow=1, key=None):
    """face_gan.py:26-36: FullGenerator(size, 512, 8, channel_multiplier, narrow) + state_dict."""
    net = FullGenerator(size, 512, 8, channel_multiplier, narrow=narrow)
    sd = _load(path)
    if key is not None:
        sd = sd[key]
    net.load_state_dict(sd)
    return net.eval()


def load_parsenet(path, size=512):
    """face_parsing.py:33-37: ParseNet(size, size, 32, 64, 19, 'bn', 'LeakyReLU', [32, 256]) + state_dict."""
    net = ParseNet(**parse_arch.face_parse_net(size))
    net.load_state_dict(_load(path))
    return net.eval()


def load_retinaface(path):
    """RetinaFaceDetection.load_model (retinaface_detection.py:45-58): ``state_dict`` entry or bare
    dict, ``module.`` prefix stripped, strict=False."""
    net = RetinaFace(retinaface_arch.CFG_RE50, phase="test")
    sd = _load(path)
    if "state_dict" in sd:
        sd = sd["state_dict"]
    sd = {(k.split("module.", 1)[-1] if k.startswith("module.") else k): v for k, v in sd.items()}
    if not set(sd) & set(net.state_dict()):
        raise AssertionError("load NONE from pretrained checkpoint")
    net.load_state_dict(sd, strict=False)
    return net.eval()


def load_face3d_net(ckpt_path, device):
    """futils/inference_utils.py:261-267: ReconNetWrapper('resnet50') with checkpoint['net_recon'],
    strict, eval, on ``device``."""
    net = define_net_recon(net_recon="resnet50", use_last_fc=False, init_path="").to(device)
    net.load_state_dict(_load(ckpt_path)["net_recon"])
    return net.eval()


def load_srmodel(path, scale=2, num_feat=32):
    """real_esrnet.py:21-30: RRDBNet(3, 3, num_feat, num_block=23, num_grow_ch=32, scale) with the
    ``params_ema`` weights, strict=True."""
    net = RRDBNet(num_in_ch=3, num_out_ch=3, num_feat=num_feat, num_block=23, num_grow_ch=32, scale=scale)
    net.load_state_dict(_load(path)["params_ema"], strict=True)
    return net.eval()


__all__ = ["LNet", "ENet", "DNet", "GFPGANv1Clean", "FullGenerator", "ParseNet", "RRDBNet", "load_checkpoint",
           "load_network", "load_DNet", "load_gfpgan", "load_gpen", "load_parsenet", "load_srmodel", "RetinaFace",
           "load_retinaface", "ReconNetWrapper", "define_net_recon", "load_face3d_net"]
