"""Host logic of the full-clip pipeline: coefficient windows, crop-norm ratio, sharding, and the
RCCL-path helpers (broadcast + gather) exercised with world_size 2 on the gloo backend."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import s2v_import  # noqa: F401
from s2v_amd import pipeline as P


def test_seq_index_and_transform_semantic():
    assert P.obtain_seq_index(0, 100)[:14] == [0] * 14 and P.obtain_seq_index(0, 100)[-1] == 12
    assert P.obtain_seq_index(99, 100)[-1] == 99 and len(P.obtain_seq_index(50, 100)) == 26
    sem = np.arange(5 * 262, dtype=np.float64).reshape(5, 262)
    c = P.transform_semantic(sem, 2, 2.0)
    assert c.shape == (73, 26) and c.dtype == np.float32
    rows = P.obtain_seq_index(2, 5)
    assert np.array_equal(c[:64, 0], sem[rows[0], 80:144])
    assert np.array_equal(c[64:67, 5], sem[rows[5], 224:227])
    assert np.array_equal(c[67:70, 7], sem[rows[7], 254:257])
    assert c[70, 3] == sem[rows[3], 259] * 2.0 and c[72, 3] == sem[rows[3], 261]


def test_find_crop_norm_ratio_picks_closest_frame():
    rng = np.random.default_rng(0)
    sem = rng.standard_normal((20, 262))
    src = sem[7:8].copy()
    src[:, -3] = 3.0
    sem[7, -3] = 1.5
    r = P.find_crop_norm_ratio(src, sem)          # frame 7 matches exp/angles exactly
    assert np.allclose(r, [2.0])


def test_dnet_coefficients_expression_hack_and_ranges():
    rng = np.random.default_rng(1)
    sem = rng.standard_normal((30, 262))
    exp = rng.standard_normal(64)
    full = P.dnet_coefficients(sem, exp)
    assert full.shape == (30, 73, 26)
    assert np.allclose(full[:, :64, :], exp.astype(np.float32)[None, :, None])
    part = P.dnet_coefficients(sem, exp, start=11, stop=17)
    assert np.array_equal(part, full[11:17])
    one = P.dnet_coefficients(sem, None, one_shot=True)
    r0 = P.find_crop_norm_ratio(sem[0:1], sem)
    assert np.allclose(one[4], P.transform_semantic(sem, 4, r0))


@pytest.mark.parametrize("n,world", [(1000, 8), (997, 8), (5, 8), (16, 2), (3, 1)])
def test_shard_range_partitions(n, world):
    ranges = [P.shard_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a, b), (c, d) in zip(ranges, ranges[1:]):
        assert b == c
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sem = torch.arange(n * 262, dtype=torch.float32).reshape(n, 262) if rank == 0 else None
        got = P.broadcast_tensor(sem, (n, 262), torch.float32, torch.device("cpu"))
        assert float(got[n - 1, 261]) == n * 262 - 1
        s, e = P.shard_range(n, rank, world)
        # per-frame stand-in for the device path: frame i -> constant (i % 251)
        local = torch.stack([torch.full((3, 4, 4), i % 251, dtype=torch.uint8) for i in range(s, e)]) \
            if e > s else torch.zeros((0, 3, 4, 4), dtype=torch.uint8)
        if rank != 0:
            # the gather is rank-0 only: no other rank receives or allocates the clip
            def refuse(*a, **k):
                raise AssertionError(f"rank {rank} must not receive frames")
            dist.recv = dist.irecv = dist.all_gather = dist.all_gather_into_tensor = refuse
        full = P.gather_frames(local, n)
        if rank == 0:
            ref = torch.stack([torch.full((3, 4, 4), i % 251, dtype=torch.uint8) for i in range(n)])
            assert full.shape == (n, 3, 4, 4) and torch.equal(full, ref)      # == the world-1 result
            q.put([int(full[i, 0, 0, 0]) for i in range(n)])
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(7, 2), (16, 2), (1, 2), (13, 4), (3, 4)])
def test_broadcast_and_gather_world2_gloo(n, world):
    """World 2 and 4: at 4, rank 0's batch_isend_irecv pairs three receives with three peers' sends (13
    frames: shards of 4 / 3 / 3 / 3), and at n = 3 one rank holds no frames and sends nothing."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == [i % 251 for i in range(n)]


# ---------------------------------------------------------------- run_sharded end to end
class _CodedPipeline:
    """Stand-in for LipSyncPipeline.run: frame i of the range [start, stop) is coded from everything the
    real device path consumes for it — its mel window (chunks[start + i], indexed absolutely), its DNet
    coefficient window (coeffs[i], this rank's slice of dnet_coefficients) and its source frame
    (src[i] from src_provider) — so a wrong window, coefficient range or source shard changes the clip."""
    device = torch.device("cpu")

    def run(self, chunks, src, coeffs, start, stop):
        n = stop - start
        assert src.shape[0] == n and coeffs.shape[0] == n and stop <= chunks.shape[0]
        out = torch.zeros((n, 3, 4, 4), dtype=torch.uint8)
        for i in range(n):
            out[i, 0] = int(chunks[start + i].double().sum().item()) % 251
            out[i, 1] = int(abs(coeffs[i].double() * torch.arange(1, 27, dtype=torch.float64)).sum().item() * 7) % 251
            out[i, 2] = int(src[i].double().sum().item()) % 251
        return out


def _stub_audio(monkeypatch):
    """CPU stand-ins for the two HIP mel ops: an index-coded [80, 1 + len // 200] 'spectrogram' and the
    real window starts (audio.chunk_starts, inference.py:209-216)."""
    from s2v_amd import audio

    def mel(wav, pad_mode="constant"):
        t = 1 + wav.numel() // 200
        return (torch.arange(t, dtype=torch.float32)[None, :] + torch.arange(80, dtype=torch.float32)[:, None] * 0.5
                + float(wav.double().sum()) * 1e-3)

    def chunks(m, fps=25.0, step=16):
        st = audio.chunk_starts(m.shape[1], fps, step)
        return torch.stack([m[None, :, s: s + step] for s in st])
    monkeypatch.setattr(P.audio, "melspectrogram", mel)
    monkeypatch.setattr(P.audio, "mel_chunks", chunks)


def _clip_inputs(frames, samples):
    rng = np.random.default_rng(5)
    wav = rng.standard_normal(samples).astype(np.float32)
    sem = rng.standard_normal((frames, 262)).astype(np.float32)
    exp = rng.standard_normal(64).astype(np.float32)
    return wav, sem, exp


def _src_provider(start, stop):
    return torch.stack([torch.full((3, 8, 8), float(i % 97), dtype=torch.float32) for i in range(start, stop)]) \
        if stop > start else torch.zeros((0, 3, 8, 8))


def _sharded_worker(rank, world, port, frames, samples, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mp_ = pytest.MonkeyPatch()
        _stub_audio(mp_)
        wav, sem, exp = _clip_inputs(frames, samples)
        if rank != 0:                     # only rank 0 holds the per-clip host data (inference.py:209-222)
            wav = sem = exp = None
        out = P.run_sharded(_CodedPipeline(), wav, sem, exp, _src_provider)
        if rank == 0:
            q.put(out.numpy())
        else:
            q.put(None if out is None else "rank 1 returned frames")
        mp_.undo()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("frames,samples", [(30, 16000), (9, 16000 * 3), (1, 3200)])
def test_run_sharded_world2_gloo_matches_world1(monkeypatch, frames, samples):
    """pipeline.run_sharded at world 2 (gloo): meta broadcast, the per-clip tensor broadcasts, per-rank
    mel windows and coefficient windows, the per-rank pipeline.run on its shard and the gather to rank 0.
    Rank 0's clip equals the world-1 clip and rank 1 gets None (pipeline.py:239-262; reference contract
    inference.py:209-222: n = min(mel chunks, frames)).  The cases cover more frames than mel windows,
    more windows than frames, and a one-frame clip that leaves rank 1 an empty shard."""
    _stub_audio(monkeypatch)
    wav, sem, exp = _clip_inputs(frames, samples)
    ref = P.run_sharded(_CodedPipeline(), wav, sem, exp, _src_provider).numpy()     # world 1
    n_chunks = len(P.audio.chunk_starts(1 + samples // 200))
    assert ref.shape == (min(n_chunks, frames), 3, 4, 4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, frames, samples, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert sum(g is None for g in got) == 1, got
    clip = next(g for g in got if g is not None)
    assert isinstance(clip, np.ndarray) and np.array_equal(clip, ref)
