"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Runs only in the build container (it imports /root/reference, which does not exist on the GPU
box).  Inputs and weights are regenerated from the portable counter hash in ``s2v_amd.synth``,
so only outputs (full tensors for small cases, fixed-index probes for large ones) are stored.

Import shims (neither touches arithmetic; both documented in SURVEY.md §8c):
  * ``torchsummary`` is imported but unused by models/__init__.py:6 -> empty stub module;
  * ``basicsr.archs.arch_util.default_init_weights`` (models/base_blocks.py:9) -> the reference's
    own vendored copy third_part/GPEN/sr_model/arch_util.py (only used for init, which the
    synthetic state_dict overwrites).

Face detection / alignment (gen_face) adds import-only stubs: ``torchvision`` (retinaface.py /
net.py import it at module level; the FPN / SSH / head classes and RetinaFace.forward never call it:
the ResNet-50 body, the only torchvision user, is replaced by the features under test), ``cv2`` and
``skimage`` (imported by data/ and align_faces.py; cv2.warpAffine is stubbed to None inside
warp_and_crop_face, whose numpy transform math is what the fixture pins).

3DMM extraction (gen_face3d) loads third_part/face3d/util/preprocess.py and models/networks.py by
file path with import-only stubs for ``cv2`` / ``skimage`` / ``kornia`` (none is called by POS,
resize_n_crop_img or ReconNetWrapper) and one numpy alias: preprocess.py:13 names
``np.VisibleDeprecationWarning``, which numpy 2 moved to ``np.exceptions``.  align_img itself cannot
run under numpy >= 1.24 (its ``np.array([w0, h0, s, t[0], t[1]])`` is ragged); the fixture takes
POS and resize_n_crop_img from the reference and assembles trans_params the way facing.py:119
reads it under numpy 1.23 (five floats).  Pillow, which resize_n_crop_img calls, is installed.

Usage:  python tests/golden/make_golden.py [--only lnet,enet,dnet,ops,gfpgan,gpen,gpen2048,parsenet,rrdbnet,face,face3d]
"""
import argparse
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
import s2v_import  # noqa: E402,F401
from s2v_amd import synth  # noqa: E402
from s2v_amd.models import arch  # noqa: E402


def _install_ref_shims():
    ts = types.ModuleType("torchsummary")
    ts.summary = lambda *a, **k: None
    sys.modules.setdefault("torchsummary", ts)
    spec = importlib.util.spec_from_file_location(
        "_ref_arch_util", os.path.join(REF, "third_part/GPEN/sr_model/arch_util.py"))
    au = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(au)
    for name in ("basicsr", "basicsr.archs"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["basicsr.archs.arch_util"] = au
    sys.modules["basicsr"].archs = sys.modules["basicsr.archs"]
    sys.modules["basicsr.archs"].arch_util = au
    if REF not in sys.path:
        sys.path.insert(0, REF)


def _manifest(module):
    return {k: list(v.shape) for k, v in module.state_dict().items()}


def _check_keys(name, ref_mod, mine):
    a, b = _manifest(ref_mod), _manifest(mine)
    if a != b:
        missing = sorted(set(a) - set(b))[:10]
        extra = sorted(set(b) - set(a))[:10]
        diff = [k for k in a if k in b and a[k] != b[k]][:10]
        raise SystemExit(f"{name}: state_dict layout mismatch missing={missing} extra={extra} shape={diff}")
    with open(os.path.join(HERE, f"{name}_keys.json"), "w") as f:
        json.dump(a, f, indent=0, sort_keys=True)
    print(f"{name}: {len(a)} state_dict entries match the reference layout")


def _load_synth(ref_mod):
    sd = synth.synth_torch_state_dict(ref_mod)
    missing, unexpected = ref_mod.load_state_dict(sd, strict=True), None
    return sd


def _probe(t: torch.Tensor, key: str):
    flat = t.detach().reshape(-1).double().numpy()
    idx = synth.probe_indices(flat.size, 4096, key)
    return {"idx": idx, "val": flat[idx].astype(np.float32),
            "stats": np.array([flat.mean(), flat.std(), np.abs(flat).max(), flat.size], dtype=np.float64)}


def _save(name, arrays):
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def gen_lnet():
    from models.LNet import LNet
    ref = LNet().eval()
    _check_keys("lnet", ref, arch.LNetParams())
    _load_synth(ref)
    acts = {}
    hooks = [
        ref.audio_encoder.register_forward_hook(lambda m, i, o: acts.__setitem__("audio_feat", o)),
        ref.decoder.final.model[0].register_forward_hook(lambda m, i, o: acts.__setitem__("logits", o)),
        ref.encoder.register_forward_hook(lambda m, i, o: acts.__setitem__("enc", [t.clone() for t in o])),
        ref.decoder.res2.register_forward_hook(lambda m, i, o: acts.__setitem__("res2", o)),
    ]
    mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
    with torch.no_grad():
        out = ref(torch.from_numpy(mel), torch.from_numpy(face))
    for h in hooks:
        h.remove()
    arrays = {"out": out.numpy(), "logits": acts["logits"].numpy(),
              "audio_feat": acts["audio_feat"].reshape(2, -1).numpy()}
    for i, t in enumerate(acts["enc"]):
        p = _probe(t, f"lnet.enc{i}")
        arrays.update({f"enc{i}_idx": p["idx"], f"enc{i}_val": p["val"], f"enc{i}_stats": p["stats"]})
    p = _probe(acts["res2"], "lnet.res2")
    arrays.update({"res2_idx": p["idx"], "res2_val": p["val"], "res2_stats": p["stats"]})
    _save("lnet_b2_96", arrays)


def gen_enet():
    from models.LNet import LNet
    from models.ENet import ENet
    ref = ENet(lnet=LNet()).eval()
    _check_keys("enet", ref, arch.ENetParams(lnet=arch.LNetParams()))
    _load_synth(ref)
    acts = {}
    ref.final_linear.register_forward_hook(lambda m, i, o: acts.__setitem__("style", o))
    for size, full in ((256, True), (384, False)):
        mel, face, gt = synth.lipsync_inputs(f"golden.enet{size}", 1, size)
        with torch.no_grad():
            out, low = ref(torch.from_numpy(mel), torch.from_numpy(face), torch.from_numpy(gt))
        arrays = {"low": low.numpy(), "style": acts["style"].numpy()}
        if full:
            arrays["out"] = out.numpy()
        else:
            p = _probe(out, "enet.out")
            arrays.update({"out_idx": p["idx"], "out_val": p["val"], "out_stats": p["stats"]})
        _save(f"enet_b1_{size}", arrays)


def gen_dnet():
    from models.DNet import DNet
    ref = DNet().eval()
    _check_keys("dnet", ref, arch.DNetParams())
    _load_synth(ref)
    acts = {}
    ref.mapping_net.register_forward_hook(lambda m, i, o: acts.__setitem__("descriptor", o))
    for size, batch, full in ((128, 2, True), (256, 1, False)):
        src, coeff = synth.dnet_inputs(f"golden.dnet{size}", batch, size)
        with torch.no_grad():
            out = ref(torch.from_numpy(src), torch.from_numpy(coeff))
        arrays = {"descriptor": acts["descriptor"].reshape(batch, -1).numpy(),
                  "flow": out["flow_field"].numpy()}
        for k in ("warp_image", "fake_image"):
            if full:
                arrays[k] = out[k].numpy()
            else:
                p = _probe(out[k], f"dnet.{k}")
                arrays.update({f"{k}_idx": p["idx"], f"{k}_val": p["val"], f"{k}_stats": p["stats"]})
        _save(f"dnet_b{batch}_{size}", arrays)


def gen_ops():
    """GPEN native-op CPU fallbacks (op/fused_act.py:92-96, op/upfirdn2d.py:149-193) and the
    flow_util warp (futils/flow_util.py:3-56) on small shapes."""
    sys.path.insert(0, os.path.join(REF, "third_part/GPEN/face_model"))
    from op.fused_act import fused_leaky_relu
    from op.upfirdn2d import upfirdn2d
    from futils import flow_util
    arrays = {}
    x = torch.from_numpy(synth.hash_array("golden.fba.x", (2, 8, 5, 7)))
    b = torch.from_numpy(synth.hash_array("golden.fba.b", (8,)))
    arrays["fba_out"] = fused_leaky_relu(x, b, 0.2, 2 ** 0.5).numpy()
    x2 = torch.from_numpy(synth.hash_array("golden.fba.x2", (3, 16)))
    b2 = torch.from_numpy(synth.hash_array("golden.fba.b2", (16,)))
    arrays["fba2_out"] = fused_leaky_relu(x2, b2, 0.2, 2 ** 0.5).numpy()
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = k[None, :] * k[:, None]
    k = k / k.sum()
    xi = torch.from_numpy(synth.hash_array("golden.ufd.x", (2, 3, 9, 11)))
    for name, (up, down, pad) in {"up2": (2, 1, (2, 1)), "blur22": (1, 1, (2, 2)),
                                  "blur11": (1, 1, (1, 1)), "down2": (1, 2, (1, 1))}.items():
        arrays[f"ufd_{name}"] = upfirdn2d(xi, k * (4 if up == 2 else 1), up=up, down=down, pad=pad).numpy()
    # the other two dtypes the reference's ops dispatch (fused_bias_act_kernel.cu:79,
    # upfirdn2d_kernel.cu:225), through the same CPU fallbacks: float64, and float16 with
    # fp64 outputs of the half-rounded inputs beside the fallback's own half result
    for dt, tag in ((torch.float64, "f64"), (torch.float16, "f16")):
        xd, bd = x.to(dt), b.to(dt)
        arrays[f"fba_{tag}_out"] = fused_leaky_relu(xd, bd, 0.2, 2 ** 0.5).numpy()
        if dt == torch.float16:
            arrays["fba_f16_exact"] = fused_leaky_relu(xd.double(), bd.double(), 0.2, 2 ** 0.5).numpy()
        for name, (up, down, pad) in {"up2": (2, 1, (2, 1)), "blur22": (1, 1, (2, 2)),
                                      "down2": (1, 2, (1, 1))}.items():
            kd = (k * (4 if up == 2 else 1)).to(dt)
            arrays[f"ufd_{name}_{tag}"] = upfirdn2d(xi.to(dt), kd, up=up, down=down, pad=pad).numpy()
            if dt == torch.float16:
                arrays[f"ufd_{name}_f16_exact"] = upfirdn2d(xi.to(dt).double(), kd.double(), up=up, down=down,
                                                            pad=pad).numpy()
    flow = torch.from_numpy(synth.hash_array("golden.flow", (2, 2, 16, 16), -3.0, 3.0))
    src = torch.from_numpy(synth.hash_array("golden.flow.src", (2, 3, 64, 64)))
    deform = flow_util.convert_flow_to_deformation(flow)
    arrays["warp"] = flow_util.warp_image(src, deform).numpy()
    flow_same = torch.from_numpy(synth.hash_array("golden.flow2", (1, 2, 32, 32), -2.0, 2.0))
    src2 = torch.from_numpy(synth.hash_array("golden.flow2.src", (1, 3, 32, 32)))
    arrays["warp_same"] = flow_util.warp_image(src2, flow_util.convert_flow_to_deformation(flow_same)).numpy()
    _save("ops", arrays)


def _import_gfpgan():
    """GFPGANv1Clean by file path: the gfpgan package __init__ needs basicsr/facexlib, so only
    the two arch files are loaded, with ``basicsr.utils.registry.ARCH_REGISTRY`` stubbed as a
    no-op decorator."""
    reg = types.ModuleType("basicsr.utils.registry")

    class _Registry:
        def register(self, *a, **k):
            return lambda c: c
    reg.ARCH_REGISTRY = _Registry()
    sys.modules.setdefault("basicsr.utils", types.ModuleType("basicsr.utils"))
    sys.modules["basicsr.utils.registry"] = reg
    base = os.path.join(REF, "third_part/GFPGAN/gfpgan/archs")
    pkg = types.ModuleType("_ref_gfpgan_archs")
    pkg.__path__ = [base]
    sys.modules["_ref_gfpgan_archs"] = pkg
    for m in ("stylegan2_clean_arch", "gfpganv1_clean_arch"):
        spec = importlib.util.spec_from_file_location(f"_ref_gfpgan_archs.{m}", os.path.join(base, m + ".py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules[f"_ref_gfpgan_archs.{m}"] = mod
        spec.loader.exec_module(mod)
    return sys.modules["_ref_gfpgan_archs.gfpganv1_clean_arch"].GFPGANv1Clean


GFPGAN_KW = dict(out_size=512, num_style_feat=512, channel_multiplier=2, decoder_load_path=None, fix_decoder=False,
                 num_mlp=8, input_is_latent=True, different_w=True, narrow=1, sft_half=True)


def gen_gfpgan():
    from s2v_amd.models.enhancer_arch import GFPGANv1CleanParams
    ref = _import_gfpgan()(**GFPGAN_KW).eval()
    _check_keys("gfpgan", ref, GFPGANv1CleanParams(**GFPGAN_KW))
    sd = synth.synth_torch_state_dict(ref, **synth.GFPGAN_SYNTH)
    ref.load_state_dict(sd, strict=True)
    acts = {}
    ref.final_linear.register_forward_hook(lambda m, i, o: acts.__setitem__("style", o))
    x = synth.face_inputs("golden.gfpgan", 1)
    with torch.no_grad():
        img, rgbs = ref(torch.from_numpy(x), return_rgb=True, randomize_noise=False)
    arrays = {"style": acts["style"].numpy(), "rgb0": rgbs[0].numpy(), "rgb3": rgbs[3].numpy()}
    for name, t in (("out", img), ("rgb6", rgbs[6])):
        p = _probe(t, f"gfpgan.{name}")
        arrays.update({f"{name}_idx": p["idx"], f"{name}_val": p["val"], f"{name}_stats": p["stats"]})
    _save("gfpgan_b1_512", arrays)


def gen_gpen():
    sys.path.insert(0, os.path.join(REF, "third_part/GPEN/face_model"))
    from gpen_model import FullGenerator
    from s2v_amd.models.enhancer_arch import FullGeneratorParams
    ref = FullGenerator(512, 512, 8, 2, narrow=1, device="cpu").eval()
    _check_keys("gpen", ref, FullGeneratorParams(512, 512, 8, 2, narrow=1))
    sd = synth.synth_torch_state_dict(ref, **synth.GPEN_SYNTH)
    ref.load_state_dict(sd, strict=True)
    acts = {}
    ref.final_linear.register_forward_hook(lambda m, i, o: acts.__setitem__("code", o))
    ref.generator.style.register_forward_hook(lambda m, i, o: acts.__setitem__("latent", o))
    x = synth.face_inputs("golden.gpen", 1)
    with torch.no_grad():
        img, _ = ref(torch.from_numpy(x))
    arrays = {"code": acts["code"].numpy(), "latent": acts["latent"].numpy()}
    p = _probe(img, "gpen.out")
    arrays.update({"out_idx": p["idx"], "out_val": p["val"], "out_stats": p["stats"]})
    _save("gpen_b1_512", arrays)


def gen_gpen2048():
    """GPEN-BFR-2048 (the CLI's `enhancer` face GAN, inference.py:228-231 -> FaceGAN(in_size=2048),
    face_gan.py:26-28): FullGenerator(2048, 512, 8, 2), probes of the 2048x2048 output."""
    sys.path.insert(0, os.path.join(REF, "third_part/GPEN/face_model"))
    from gpen_model import FullGenerator
    from s2v_amd.models.enhancer_arch import FullGeneratorParams
    ref = FullGenerator(2048, 512, 8, 2, narrow=1, device="cpu").eval()
    _check_keys("gpen2048", ref, FullGeneratorParams(2048, 512, 8, 2, narrow=1))
    ref.load_state_dict(synth.synth_torch_state_dict(ref, **synth.GPEN_SYNTH), strict=True)
    acts = {}
    ref.final_linear.register_forward_hook(lambda m, i, o: acts.__setitem__("code", o))
    x = synth.face_inputs("golden.gpen2048", 1, 2048)
    with torch.no_grad():
        img, _ = ref(torch.from_numpy(x))
    arrays = {"code": acts["code"].numpy()}
    p = _probe(img, "gpen2048.out")
    arrays.update({"out_idx": p["idx"], "out_val": p["val"], "out_stats": p["stats"]})
    _save("gpen_b1_2048", arrays)


def gen_parsenet():
    """GPEN ParseNet (face_parse/parse_model.py) at the FaceParse configuration (512, with the
    synthetic weights) and at a small one (128), outputs as full tensors / probes."""
    sys.path.insert(0, os.path.join(REF, "third_part/GPEN/face_parse"))
    from parse_model import ParseNet
    from s2v_amd.models.parse_arch import ParseNetParams, face_parse_net
    cfg = face_parse_net(512)
    ref = ParseNet(512, 512, 32, 64, 19, norm_type="bn", relu_type="LeakyReLU", ch_range=[32, 256]).eval()
    _check_keys("parsenet", ref, ParseNetParams(**cfg))
    for size, batch in ((128, 2), (512, 1)):
        net = ParseNet(size, size, 32, 64, 19, norm_type="bn", relu_type="LeakyReLU", ch_range=[32, 256]).eval()
        sd = synth.synth_torch_state_dict(net, **synth.PARSENET_SYNTH)
        net.load_state_dict(sd, strict=True)
        x = synth.face_inputs(f"golden.parsenet{size}", batch, size)
        with torch.no_grad():
            mask, img = net(torch.from_numpy(x))
        arrays = {"argmax": mask.argmax(1).numpy().astype(np.int8)}
        if size == 128:
            arrays.update({"mask": mask.numpy(), "img": img.numpy()})
        else:
            for name, t in (("mask", mask), ("img", img)):
                pr = _probe(t, f"parsenet.{name}")
                arrays.update({f"{name}_idx": pr["idx"], f"{name}_val": pr["val"], f"{name}_stats": pr["stats"]})
        _save(f"parsenet_b{batch}_{size}", arrays)


# RealESRNet cases (tests/helpers.py): (tag, scale, input [B,3,H,W]) for the forward, (tag, scale,
# frame H, W, tile, tile_pad) for RealESRNet.process on uint8 frames (odd sizes: reflect padding)
sys.path.insert(0, os.path.join(REPO, "tests"))
from helpers import RRDB_FORWARD, RRDB_PROCESS  # noqa: E402


def gen_rrdbnet():
    """third_part/GPEN/sr_model (RRDBNet + RealESRNet.process) at the FaceEnhancement configuration
    num_feat=32, num_block=23, num_grow_ch=32 (face_enhancement.py:58, real_esrnet.py:9-23)."""
    import tempfile
    sys.path.insert(0, os.path.join(REF, "third_part/GPEN/sr_model"))
    from rrdbnet_arch import RRDBNet
    from real_esrnet import RealESRNet
    from s2v_amd.models.sr_arch import RRDBNetParams
    arrays = {}
    for tag, scale, shape in RRDB_FORWARD:
        ref = RRDBNet(3, 3, scale=scale, num_feat=32, num_block=23, num_grow_ch=32).eval()
        _check_keys("rrdbnet" if scale == 2 else f"rrdbnet_x{scale}", ref,
                    RRDBNetParams(3, 3, scale=scale, num_feat=32, num_block=23, num_grow_ch=32))
        ref.load_state_dict(synth.synth_torch_state_dict(ref, **synth.RRDB_SYNTH), strict=True)
        x = synth.hash_array(f"golden.rrdb.{tag}", shape, 0.0, 1.0)
        with torch.no_grad():
            arrays[f"fwd_{tag}"] = ref(torch.from_numpy(x)).numpy()
    for tag, scale, h, w, tile, pad in RRDB_PROCESS:
        ref = RRDBNet(3, 3, scale=scale, num_feat=32, num_block=23, num_grow_ch=32)
        with tempfile.TemporaryDirectory() as d:
            os.makedirs(os.path.join(d, "weights"))
            torch.save({"params_ema": synth.synth_torch_state_dict(ref, **synth.RRDB_SYNTH)},
                       os.path.join(d, "weights", f"realesrnet_x{scale}.pth"))
            sr = RealESRNet(d, None, scale=scale, tile_size=tile, tile_pad=pad, device="cpu")
        img = synth.sr_frame(f"golden.rrdb.{tag}", 1, h, w)[0]
        arrays[f"proc_{tag}"] = sr.process(img)
    _save("rrdbnet_goldens", arrays)


from helpers import FACE_IMG_HW, FACE_LANDMARKS, retina_head_outputs, retina_tail_inputs  # noqa: E402


def _face_stubs():
    class _Any(types.ModuleType):
        def __getattr__(self, name):
            if name.startswith("__"):
                raise AttributeError(name)
            return None
    for name in ("torchvision", "torchvision.models", "torchvision.models._utils",
                 "torchvision.models.detection", "torchvision.models.detection.backbone_utils",
                 "skimage", "skimage.transform"):
        sys.modules.setdefault(name, _Any(name))
        if "." in name:
            parent, child = name.rsplit(".", 1)
            object.__setattr__(sys.modules[parent], child, sys.modules[name])
    cv2 = _Any("cv2")
    cv2.warpAffine = lambda *a, **k: None
    sys.modules["cv2"] = cv2
    for sub in ("face_detect", "face_detect/facemodels", ""):
        path = os.path.join(REF, "third_part/GPEN", sub)
        if path not in sys.path:
            sys.path.insert(0, path)


def gen_face():
    """RetinaFace-R50 detection tail + post-processing and the similarity alignment, from the
    reference's own modules (see the module docstring for the import stubs)."""
    from collections import OrderedDict
    _face_stubs()
    import net as ref_net
    import retinaface as ref_rf
    from data import cfg_re50
    import retinaface_detection as ref_det
    import align_faces as ref_align
    from s2v_amd.models.retinaface_arch import RetinaFaceParams
    arrays = {}
    # FPN + SSH + heads through RetinaFace.forward with the body bypassed (features given)
    rf = ref_rf.RetinaFace.__new__(ref_rf.RetinaFace)
    torch.nn.Module.__init__(rf)
    rf.phase = "test"
    c, oc = cfg_re50["in_channel"], cfg_re50["out_channel"]
    rf.fpn = ref_net.FPN([c * 2, c * 4, c * 8], oc)
    rf.ssh1, rf.ssh2, rf.ssh3 = (ref_net.SSH(oc, oc) for _ in range(3))
    rf.ClassHead = rf._make_class_head(fpn_num=3, inchannels=oc)
    rf.BboxHead = rf._make_bbox_head(fpn_num=3, inchannels=oc)
    rf.LandmarkHead = rf._make_landmark_head(fpn_num=3, inchannels=oc)
    rf.eval()
    mine = {k: list(v.shape) for k, v in RetinaFaceParams().state_dict().items() if not k.startswith("body.")}
    if mine != _manifest(rf):
        raise SystemExit("retinaface: FPN / SSH / head state_dict layout mismatch")
    rf.load_state_dict(synth.synth_torch_state_dict(rf, **synth.RETINA_SYNTH), strict=True)
    rf.body = lambda feats: feats
    feats = retina_tail_inputs()
    with torch.no_grad():
        loc, conf, landms = rf(OrderedDict((str(i), torch.from_numpy(f)) for i, f in enumerate(feats)))
    arrays.update(tail_loc=loc.numpy(), tail_conf=conf.numpy(), tail_landms=landms.numpy())
    # RetinaFaceDetection.detect post-processing with the net's outputs given
    det = ref_det.RetinaFaceDetection.__new__(ref_det.RetinaFaceDetection)
    det.cfg, det.device = cfg_re50, "cpu"
    hl, hc, hm = retina_head_outputs()
    det.net = lambda x: (torch.from_numpy(hl)[None], torch.from_numpy(hc)[None], torch.from_numpy(hm)[None])
    dets, lms = det.detect(np.zeros(FACE_IMG_HW + (3,), np.uint8))
    arrays.update(det_dets=np.asarray(dets, np.float32), det_landms=np.asarray(lms, np.float32))
    print(f"face: detect keeps {len(dets)} of {int((hc[:, 1] > 0.9).sum())} candidates")
    # alignment: reference points and the similarity transforms of warp_and_crop_face
    for size in (512, 2048):
        arrays[f"ref5_{size}"] = np.asarray(ref_align.get_reference_facial_points((size, size), 0.25, (0, 0), True))
    for i, pts in enumerate(FACE_LANDMARKS):
        for size in (512, 2048):
            ref = arrays[f"ref5_{size}"]
            _, tfm_inv = ref_align.warp_and_crop_face(None, np.array(pts), reference_pts=ref, crop_size=(size, size))
            params, _ = ref_align._umeyama(np.float32(np.array(pts)).T, np.float32(ref))
            arrays[f"tfm_{i}_{size}"] = np.asarray(params[:2, :], np.float64)
            arrays[f"tfm_inv_{i}_{size}"] = np.asarray(tfm_inv, np.float64)
    _save("face_goldens", arrays)


def gen_face3d():
    """PIL resize cases, align_img's geometry and pixels, ReconNetWrapper('resnet50') and the
    facing.py:108-129 semantic rows, from the reference's own functions."""
    from PIL import Image
    from helpers import FACE3D_LM3D, PIL_RESIZE_CASES, face3d_frames, face3d_landmarks
    from s2v_amd.models.face3d_arch import ReconNetWrapperParams
    _face_stubs()
    for name in ("kornia", "kornia.geometry"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["kornia"].geometry = sys.modules["kornia.geometry"]
    sys.modules["kornia.geometry"].warp_affine = None
    if not hasattr(np, "VisibleDeprecationWarning"):
        np.VisibleDeprecationWarning = np.exceptions.VisibleDeprecationWarning
    f3d = os.path.join(REF, "third_part/face3d")
    spec = importlib.util.spec_from_file_location("_ref_face3d_pre", os.path.join(f3d, "util/preprocess.py"))
    pre = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pre)
    pkg = types.ModuleType("_ref_face3d_models")
    pkg.__path__ = [os.path.join(f3d, "models")]
    sys.modules["_ref_face3d_models"] = pkg
    spec = importlib.util.spec_from_file_location("_ref_face3d_models.networks", os.path.join(f3d, "models/networks.py"))
    nets = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = nets
    spec.loader.exec_module(nets)
    arrays = {}
    # Pillow resample cases (the arithmetic resize_n_crop_img delegates to)
    for i, (w0, h0, w, h, flt) in enumerate(PIL_RESIZE_CASES):
        img = np.floor(synth.hash_array(f"golden.pil.{i}", (h0, w0, 3), 0.0, 256.0)).astype(np.uint8)
        arrays[f"pil_{i}"] = np.asarray(Image.fromarray(img).resize((w, h), resample=flt))
    # align_img geometry + pixels, one frame per landmark case (facing.py:110-118)
    lm3d = FACE3D_LM3D
    lms = face3d_landmarks()
    frames = face3d_frames(len(lms))
    # futils/inference_utils.py:158-181 split_coeff, compiled alone from the reference file (the module
    # imports cv2 / torchvision / face_detection at the top, none of which split_coeff uses)
    import ast
    src = open(os.path.join(REF, "futils/inference_utils.py")).read()
    fn = next(n for n in ast.parse(src).body if isinstance(n, ast.FunctionDef) and n.name == "split_coeff")
    ns = {}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "futils/inference_utils.py", "exec"), ns)
    split_coeff = ns["split_coeff"]
    net = nets.define_net_recon(net_recon="resnet50", use_last_fc=False, init_path="")
    _check_keys("recon", net, ReconNetWrapperParams())
    net.load_state_dict(synth.synth_torch_state_dict(net, **synth.RETINA_SYNTH), strict=True)
    net.eval()
    rows, ims = [], []
    for i, (frame, lm) in enumerate(zip(frames, lms)):
        H, W = frame.shape[:2]
        lm_idx = lm.reshape([-1, 2]).copy()
        if np.mean(lm_idx) == -1:
            lm_idx = (lm3d[:, :2] + 1) / 2.
            lm_idx = np.concatenate([lm_idx[:, :1] * W, lm_idx[:, 1:2] * H], 1)
        else:
            lm_idx[:, -1] = H - 1 - lm_idx[:, -1]
        lm5p = pre.extract_5p(lm_idx) if lm_idx.shape[0] != 5 else lm_idx
        t, s = pre.POS(lm5p.transpose(), lm3d.transpose())
        s = 102. / s
        im, lm_new, _ = pre.resize_n_crop_img(Image.fromarray(frame), lm_idx, t, s, target_size=224.)
        w, h = (W * s).astype(np.int32), (H * s).astype(np.int32)
        trans = np.array([float(W), float(H), float(s), float(t[0][0]), float(t[1][0])]).astype(np.float32)
        arrays[f"lm_{i}"] = np.asarray(lm_idx, np.float64)
        arrays[f"box_{i}"] = np.array([w, h, (w / 2 - 112. + float(((t[0] - W / 2) * s)[0])),
                                       (h / 2 - 112. + float(((H / 2 - t[1]) * s)[0]))], np.float64)
        arrays[f"im_{i}"] = np.asarray(im)
        arrays[f"lmnew_{i}"] = np.asarray(lm_new, np.float64)
        x = torch.tensor(np.array(im) / 255., dtype=torch.float32).permute(2, 0, 1).to("cpu").unsqueeze(0)
        with torch.no_grad():
            c = {k: v.numpy() for k, v in split_coeff(net(x)).items()}
        rows.append(np.concatenate([c["id"], c["exp"], c["tex"], c["angle"], c["gamma"], c["trans"], trans[None]], 1))
        print(f"face3d case {i}: resized {w}x{h}, box {arrays[f'box_{i}'][2:]}, s={float(s):.4f}")
    arrays["semantic"] = np.concatenate(rows, 0)
    _save("face3d_goldens", arrays)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="lnet,enet,dnet,ops")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 8)
    _install_ref_shims()
    os.chdir("/tmp")
    for part in args.only.split(","):
        globals()[f"gen_{part}"]()
