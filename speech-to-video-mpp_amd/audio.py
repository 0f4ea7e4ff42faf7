"""Device mel front end (reference futils/audio.py:45-51 with futils/hparams.py:21-61) and the
per-frame 16-column mel windows (inference.py:209-216), on libs2v kernels.

    mel = melspectrogram(wav_cuda)                 # [80, 1 + N//200] float32 on the device
    chunks = mel_chunks(mel, fps=25)               # [n_frames, 1, 80, 16] (LNet audio input)

Constant tables (Slaney mel basis, DFT twiddles, periodic Hann window) are built once on the host
in float64 and uploaded as float32.  pad_mode: 'constant' (librosa 0.9.2 stft default, the
pinned reference version) or 'reflect' (librosa <= 0.8).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib, ops
from .ops import Ctx

SR, N_FFT, HOP, N_MELS, FMIN, FMAX = 16000, 800, 200, 80, 55.0, 7600.0
_TABLES = {}
_CTX = {}


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_hz / f_sp + np.log(np.maximum(f, 1e-12) / min_log_hz) / logstep, f / f_sp)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def slaney_mel_basis() -> np.ndarray:
    """[80, 401] float32 triangular Slaney-normalised filterbank (sr 16 kHz, 55..7600 Hz)."""
    freqs = np.fft.rfftfreq(n=N_FFT, d=1.0 / SR)
    edges = _mel_to_hz(np.linspace(_hz_to_mel(FMIN), _hz_to_mel(FMAX), N_MELS + 2))
    widths = np.diff(edges)
    w = np.zeros((N_MELS, freqs.size), dtype=np.float32)
    for i in range(N_MELS):
        rise = (freqs - edges[i]) / widths[i]
        fall = (edges[i + 2] - freqs) / widths[i + 1]
        w[i] = np.maximum(0.0, np.minimum(rise, fall))
    w *= (2.0 / (edges[2:] - edges[:-2]))[:, None]
    return w


def tables(device) -> torch.Tensor:
    key = str(device)
    if key not in _TABLES:
        k = np.arange(N_FFT, dtype=np.float64)
        ang = 2.0 * np.pi * k / N_FFT
        win = 0.5 - 0.5 * np.cos(ang)
        t = np.concatenate([slaney_mel_basis().astype(np.float64).ravel(), np.cos(ang), np.sin(ang), win])
        _TABLES[key] = torch.from_numpy(t.astype(np.float32)).to(device)
    return _TABLES[key]


def _ctx(device):
    key = str(device)
    if key not in _CTX:
        _CTX[key] = Ctx(device)
    return _CTX[key]


def melspectrogram(wav: torch.Tensor, pad_mode: str = "constant") -> torch.Tensor:
    """wav: 1-D float32 device tensor (16 kHz) -> [80, 1 + len//200] float32."""
    if not wav.is_cuda:
        raise _lib.S2VError("melspectrogram runs on the HIP device only")
    wav = wav.contiguous().float()
    n = wav.numel()
    frames = 1 + n // HOP
    out = torch.empty((N_MELS, frames), device=wav.device)
    ops.S2V.melspectrogram_(wav, tables(wav.device), pad_mode == "reflect", out)
    return out


def chunk_starts(n_cols: int, fps: float = 25.0, step: int = 16):
    """inference.py:209-216 window starts (host logic, integer)."""
    starts, i, mult = [], 0, 80.0 / fps
    while True:
        s = int(i * mult)
        if s + step > n_cols:
            starts.append(n_cols - step)
            return starts
        starts.append(s)
        i += 1


def mel_chunks(mel: torch.Tensor, fps: float = 25.0, step: int = 16) -> torch.Tensor:
    """[80, T] device mel -> [n, 1, 80, step] windows (the LNet audio input layout)."""
    T = mel.shape[1]
    st = chunk_starts(T, fps, step)
    starts = torch.tensor(st, dtype=torch.int32).to(mel.device)
    out = torch.empty((len(st), 1, N_MELS, step), device=mel.device)
    ops.S2V.mel_chunks_(mel.contiguous(), starts, step, out)
    return out
