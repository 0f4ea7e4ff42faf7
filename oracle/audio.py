"""CPU restatement of the reference mel front end (futils/audio.py + futils/hparams.py).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  PARITY UNPINNED: the reference computes the
STFT and the mel filterbank through librosa 0.9.2 (requirements.txt:6), which is absent here and
not vendored, so no reference output pins these numbers.  This module restates librosa 0.9.2's
published algorithm in float64 NumPy:

  * preemphasis        audio.py:20-23   scipy.signal.lfilter([1, -0.97], [1], wav)
  * _stft              audio.py:57-61   librosa.stft(n_fft=800, hop_length=200, win_length=800):
                       window 'hann' periodic (scipy.signal.get_window(fftbins=True)), center=True
                       padding by n_fft//2 with ``pad_mode`` (librosa 0.9.2 default 'constant';
                       0.8.x used 'reflect' -- both exposed), frames = 1 + len//hop
  * _linear_to_mel     audio.py:92-103  librosa.filters.mel(sr=16000, n_fft=800, n_mels=80,
                       fmin=55, fmax=7600, htk=False, norm='slaney') cast to float32
  * _amp_to_db         audio.py:104-106 20*log10(max(1e-5, x)), minus ref_level_db = 20
  * _normalize         audio.py:111-117 clip(8*(S+100)/100 - 4, -4, 4)
"""
from __future__ import annotations

import numpy as np

SR, N_FFT, HOP, WIN, N_MELS, FMIN, FMAX = 16000, 800, 200, 800, 80, 55.0, 7600.0
PREEMPH, MIN_LEVEL_DB, REF_LEVEL_DB, MAX_ABS = 0.97, -100.0, 20.0, 4.0


def hz_to_mel(f):
    """Slaney mel scale (librosa.core.convert.hz_to_mel, htk=False)."""
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-12) / min_log_hz) / logstep, mels)


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_basis(sr=SR, n_fft=N_FFT, n_mels=N_MELS, fmin=FMIN, fmax=FMAX) -> np.ndarray:
    """librosa.filters.mel (slaney norm) -> float32 [n_mels, 1 + n_fft//2]."""
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)             # librosa.fft_frequencies
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    weights = np.zeros((n_mels, len(fftfreqs)), dtype=np.float32)  # librosa fills a float32 array
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2: n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, None]
    return weights


def hann_periodic(n=WIN) -> np.ndarray:
    k = np.arange(n)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def preemphasis(wav, k=PREEMPH):
    wav = np.asarray(wav, dtype=np.float64)
    out = wav.copy()
    out[1:] -= k * wav[:-1]
    return out


def stft_mag(y, pad_mode="constant"):
    """|librosa.stft(y, 800, 200, 800, center=True)| as [401, frames] float64."""
    y = np.asarray(y, dtype=np.float64)
    yp = np.pad(y, (N_FFT // 2, N_FFT // 2), mode=pad_mode)
    frames = 1 + (len(yp) - N_FFT) // HOP
    idx = np.arange(N_FFT)[None, :] + HOP * np.arange(frames)[:, None]
    seg = yp[idx] * hann_periodic()[None, :]
    return np.abs(np.fft.rfft(seg, n=N_FFT, axis=1)).T


def melspectrogram(wav, pad_mode="constant"):
    """audio.melspectrogram (audio.py:45-51) -> float64 [80, 1 + len(wav)//200]."""
    S = stft_mag(preemphasis(wav), pad_mode)
    mel = np.dot(mel_basis(), S)
    db = 20.0 * np.log10(np.maximum(np.exp(MIN_LEVEL_DB / 20.0 * np.log(10)), mel)) - REF_LEVEL_DB
    return np.clip((2 * MAX_ABS) * ((db - MIN_LEVEL_DB) / (-MIN_LEVEL_DB)) - MAX_ABS, -MAX_ABS, MAX_ABS)


def mel_chunk_starts(n_cols, n_frames_video=None, fps=25, step=16):
    """inference.py:209-216: window i starts at int(i * 80/fps); the last window is clamped to
    the end of the spectrogram and ends the sequence."""
    starts, i, mult = [], 0, 80.0 / fps
    while True:
        s = int(i * mult)
        if s + step > n_cols:
            starts.append(n_cols - step)
            break
        starts.append(s)
        i += 1
    return starts
