"""Full-clip per-frame lip-sync path (BASELINE configs 3/4): wav -> mel windows, semantic 3DMM
coefficients -> DNet expression-canonicalised reference faces -> ENet(+LNet) -> uint8 frames.

Reference flow restated (host parts are plain NumPy, device parts libs2v kernels):
  * mel + 16-column windows          inference.py:204-216            (s2v_amd.audio)
  * DNet coefficient windows          futils/inference_utils.py:73-99, preprocessing/facing.py:176-187
  * DNet -> uint8 stabilised frame   facing.py:189-191
  * ENet batch inputs                 inference.py:393-399 (lower half of the crop masked, /255)
  * ENet -> clamp(0,1)*255 -> uint8   inference.py:266-288

Multi-GPU: frames are independent once the per-clip host data exists, so ranks
take contiguous frame ranges; RCCL (torch.distributed 'nccl') carries only the broadcast of the
per-clip host tensors (wav, semantic coefficients, expression) and the final gather of the uint8
frames.  The helpers are backend-agnostic (gloo on CPU in the tests).
"""
from __future__ import annotations

import numpy as np
import torch

from . import audio, ops
from .ops import Ctx


# ----------------------------------------------------------------------------- host precompute
def obtain_seq_index(index: int, num_frames: int):
    """inference_utils.py:73-76: 26-frame window centred on ``index``, clamped to the clip."""
    return [min(max(i, 0), num_frames - 1) for i in range(index - 13, index + 13)]


def transform_semantic(semantic: np.ndarray, frame_index: int, crop_norm_ratio=None) -> np.ndarray:
    """inference_utils.py:78-91 -> float32 [73, 26] (exp 64 | angles 3 | translation 3 | crop 3)."""
    coeff = semantic[obtain_seq_index(frame_index, semantic.shape[0])]
    ex, ang, trans = coeff[:, 80:144], coeff[:, 224:227], coeff[:, 254:257]
    crop = coeff[:, 259:262].copy()
    if crop_norm_ratio:
        crop[:, -3] = crop[:, -3] * crop_norm_ratio
    return np.concatenate([ex, ang, trans, crop], 1).astype(np.float32).T.copy()


def find_crop_norm_ratio(source_coeff: np.ndarray, target_coeffs: np.ndarray):
    """inference_utils.py:93-99 (argmin of 0.3 * exp diff + 0.7 * angle diff)."""
    alpha = 0.3
    exp_diff = np.mean(np.abs(target_coeffs[:, 80:144] - source_coeff[:, 80:144]), 1)
    angle_diff = np.mean(np.abs(target_coeffs[:, 224:227] - source_coeff[:, 224:227]), 1)
    index = np.argmin(alpha * exp_diff + (1 - alpha) * angle_diff)
    return source_coeff[:, -3] / target_coeffs[index: index + 1, -3]


def dnet_coefficients(semantic: np.ndarray, expression=None, one_shot: bool = False, start: int = 0,
                      stop: int | None = None) -> np.ndarray:
    """facing.py:176-187 for frames [start, stop) -> float32 [n, 73, 26]; ``expression`` (64,)
    overwrites the expression rows (the 'hack_3dmm_expression' step)."""
    stop = semantic.shape[0] if stop is None else stop
    out = np.empty((stop - start, 73, 26), dtype=np.float32)
    for k, idx in enumerate(range(start, stop)):
        src = semantic[0:1] if one_shot else semantic[idx: idx + 1]
        ratio = find_crop_norm_ratio(src, semantic)
        out[k] = transform_semantic(semantic, idx, ratio)
        if expression is not None:
            out[k, :64, :] = np.asarray(expression, dtype=np.float32)[:64, None]
    return out


def shard_range(n: int, rank: int, world: int):
    """Contiguous frame range of ``rank`` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


# ----------------------------------------------------------------------------- device path
class LipSyncPipeline:
    """mel windows + DNet source frames + coefficient windows -> uint8 [n, 3, 384, 384] frames.

    Full batches replay captured HIP graphs on ``lanes`` execution lanes (runtime.LaneRunner):
    batch k runs on lane k % lanes, on that lane's stream, so one batch's latency-bound LNet chain
    overlaps the previous batch's MFMA-bound StyleConv decoder.  Each lane has its own workspaces,
    side streams and noise counters (the models' per-lane ops.Ctx) and its own graph buffers."""

    def __init__(self, dnet, enet, device="cuda", batch: int = 16, graph: bool = True, lanes: int = 1,
                 ref_hook=None):
        self.dnet, self.enet = dnet, enet
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            # the modules key their per-device engines (and lane flags, _lane_flags) by the inputs'
            # device, which always carries an index
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.batch = batch
        self.ctx = Ctx(self.device)
        self.graph = graph          # full batches of ``run`` replay captured HIP graphs
        self.lanes = lanes
        self.ref_hook = ref_hook    # Step 5 (inference.py:234-238) on the uint8 references; eager batches only
        self._runner = None
        self.reruns = 0             # replayed batches run again in bf16x3 after an f16x3 range overflow

    @torch.no_grad()
    def run_batch(self, mel: torch.Tensor, src: torch.Tensor, coeff: torch.Tensor, out_u8: torch.Tensor,
                  lane: int = 0):
        """mel [b,1,80,16], src [b,3,256,256] in [-1,1] (DNet input, trans_image layout), coeff
        [b,73,26] -> out_u8 [b,3,384,384] (RGB, NCHW)."""
        b, _, h, w = src.shape
        fake = self.dnet(src, coeff, lane=lane)["fake_image"]
        ref_u8 = torch.empty((b, 3, h, w), dtype=torch.uint8, device=self.device)
        face6 = torch.empty((b, 6, h, w), device=self.device)
        gt = torch.empty((b, 3, h, w), device=self.device)
        ops.S2V.lipsync_inputs_(src.contiguous(), fake, ref_u8, face6, gt)
        if self.ref_hook is not None:                 # the enhanced references replace ref / 255 (datagen)
            ref_u8 = self.ref_hook(ref_u8).contiguous()
            ops.S2V.lipsync_inputs_(src.contiguous(), None, ref_u8, face6, gt)
        pred, _ = self.enet(mel, face6, gt, lane=lane)
        ops.S2V.to_u8_(pred, out_u8, 0.0, 1.0, 255.0, 0.0)             # inference.py:267, :288
        return out_u8

    @torch.no_grad()
    def run(self, mel_chunks: torch.Tensor, src: torch.Tensor, coeffs: torch.Tensor, start: int = 0,
            stop: int | None = None) -> torch.Tensor:
        """Frames [start, stop): ``mel_chunks`` indexed absolutely, ``src`` / ``coeffs`` hold only
        the frames of this range."""
        stop = mel_chunks.shape[0] if stop is None else stop
        n = stop - start
        if not (0 <= start <= stop <= mel_chunks.shape[0]) or src.shape[0] != n or coeffs.shape[0] != n:
            raise ValueError(f"frames [{start}, {stop}) need {n} src frames / coefficient windows and "
                             f"mel windows up to {stop} (got {src.shape[0]}, {coeffs.shape[0]}, {mel_chunks.shape[0]})")
        out = torch.empty((n, 3, 384, 384), dtype=torch.uint8, device=self.device)
        runner = None
        nb = (n + self.batch - 1) // self.batch
        flags = torch.zeros(nb, dtype=torch.int32, device=self.device) if ops.guard_active() else None
        replayed = []
        for k, b0 in enumerate(range(0, n, self.batch)):
            b1 = min(n, b0 + self.batch)
            m, s, c = mel_chunks[start + b0: start + b1], src[b0:b1], coeffs[b0:b1]
            if self.graph and b1 - b0 == self.batch and self.ref_hook is None:
                runner = self._graph_runner(m, s, c)
                dst = out[b0:b1]
                lane = runner.next_lane()

                def take(o, d=dst, k=k, lane=lane):
                    d.copy_(o)
                    if flags is not None:               # this batch's f16x3 non-finite flags, then clear them
                        for f in self._lane_flags(lane):
                            torch.maximum(flags[k:k + 1], f, out=flags[k:k + 1])
                            f.zero_()
                runner(m, s, c, out_fn=take)
                out.record_stream(runner.streams[(runner.k - 1) % runner.lanes])
                replayed.append((k, b0, b1))
            else:
                if runner is not None:
                    runner.join()                 # the eager batch uses lane 0's workspaces
                self.run_batch(m, s, c, out[b0:b1])   # eager: the modules guard their own forwards
        if runner is not None:
            runner.join()
        if flags is not None and replayed:
            bad = set(torch.nonzero(flags).flatten().tolist())
            for k, b0, b1 in replayed:
                if k in bad:                      # a replayed batch left the f16x3 range: again in bf16x3
                    with ops.precision("bf16x3"):
                        self.run_batch(mel_chunks[start + b0: start + b1], src[b0:b1], coeffs[b0:b1], out[b0:b1])
                    self.reruns += 1
        return out

    def _lane_flags(self, lane):
        """The f16x3 non-finite flags of lane ``lane`` of both networks (one per module and lane)."""
        fl = []
        for mdl in (self.dnet, self.enet):
            lanes = mdl.__dict__.get("_s2v_engines", {}).get(str(self.device), (None, {}))[1]
            c = lanes.get(lane)
            f = c.range_flag() if c is not None else None
            if f is not None:
                fl.append(f)
        return fl

    def _graph_runner(self, m, s, c):
        """Captured run_batch per lane for full batches (~2,000 launches -> one graph replay each);
        inputs are copied into a lane's static buffers, its uint8 frames read from its static output."""
        if self._runner is None:
            from .runtime import LaneRunner
            bufs = [torch.empty((self.batch, 3, 384, 384), dtype=torch.uint8, device=self.device)
                    for _ in range(self.lanes)]
            self._runner = LaneRunner(lambda lane, mm, ss, cc: self.run_batch(mm, ss, cc, bufs[lane], lane=lane),
                                      [m.contiguous(), s.contiguous(), c.contiguous()], lanes=self.lanes, warmup=1)
        return self._runner


# ----------------------------------------------------------------------------- distributed helpers
def _dist():
    """(rank, world) of the default process group; (0, 1) when none is initialised (one GPU)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def broadcast_tensor(t: torch.Tensor | None, shape, dtype, device, src: int = 0) -> torch.Tensor:
    """Broadcast a per-clip host tensor from ``src`` (RCCL on GPU, gloo on CPU)."""
    import torch.distributed as dist
    rank, world = _dist()
    if rank == src:
        buf = t.to(device=device, dtype=dtype).contiguous()
    else:
        buf = torch.empty(shape, dtype=dtype, device=device)
    if world > 1:
        dist.broadcast(buf, src)
    return buf


def gather_frames(local: torch.Tensor, n_total: int, dst: int = 0):
    """Gather contiguous frame shards (shard_range layout) to ``dst``; returns [n_total, ...] on
    dst, None elsewhere (a gather to rank 0, not an all-gather).

    Only ``dst`` allocates the whole clip: it copies its own shard into place and posts one
    point-to-point receive per peer straight into that peer's frame range of the output (no padding,
    no concatenation); every other rank sends its shard once and receives nothing.  Over RCCL the
    receives run concurrently on dst's xGMI links (each peer's ~55 MB of a 1000-frame clip on its own
    link); gloo carries the same calls on the CPU."""
    import torch.distributed as dist
    rank, world = _dist()
    if world == 1:
        return local
    s, e = shard_range(n_total, rank, world)
    if local.shape[0] != e - s:
        raise ValueError(f"gather_frames: rank {rank} holds {local.shape[0]} frames, its range [{s}, {e}) has {e - s}")
    if rank != dst:
        if e > s:
            dist.send(local.contiguous(), dst)
        return None
    out = torch.empty((n_total,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    out[s:e].copy_(local)
    ops = []
    for r in range(world):
        rs, re_ = shard_range(n_total, r, world)
        if r != dst and re_ > rs:
            ops.append(dist.P2POp(dist.irecv, out[rs:re_], r))
    for w in dist.batch_isend_irecv(ops) if ops else []:
        w.wait()
    return out


def run_sharded(pipeline: LipSyncPipeline, wav, semantic, expression, src_provider, fps: float = 25.0,
                one_shot: bool = False):
    """The whole clip across all ranks.  Rank 0 holds ``wav`` (float32 [S]), ``semantic`` [N, 262],
    ``expression`` [64]; ``src_provider(start, stop)`` returns this rank's DNet source frames
    [n,3,256,256] on its device.  Returns the uint8 frames [n_chunks, 3, 384, 384] on rank 0."""
    import torch.distributed as dist
    dev = pipeline.device
    rank, world = _dist()
    meta = torch.tensor([0 if wav is None else len(wav), 0 if semantic is None else semantic.shape[0]],
                        dtype=torch.int64, device=dev)
    if world > 1:
        dist.broadcast(meta, 0)
    ns, nf = int(meta[0]), int(meta[1])
    wav_t = broadcast_tensor(None if rank else torch.as_tensor(wav), (ns,), torch.float32, dev)
    sem_t = broadcast_tensor(None if rank else torch.as_tensor(semantic), (nf, 262), torch.float32, dev)
    exp_t = broadcast_tensor(None if rank else torch.as_tensor(expression), (64,), torch.float32, dev)
    mel = audio.melspectrogram(wav_t)
    chunks = audio.mel_chunks(mel, fps=fps)
    n = min(chunks.shape[0], nf)                       # inference.py:220-222 truncation
    start, stop = shard_range(n, rank, world)
    sem = sem_t.cpu().numpy()[:n]
    coeffs = torch.from_numpy(dnet_coefficients(sem, exp_t.cpu().numpy(), one_shot, start, stop)).to(dev)
    local = pipeline.run(chunks, src_provider(start, stop), coeffs, start, stop)
    return gather_frames(local, n)
