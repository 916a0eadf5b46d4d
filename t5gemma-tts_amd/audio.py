"""Audio I/O and resampling around the codec (reference: data/tokenizer.py:125-143 loads
the prompt with torchaudio and resamples it to the encoder's 16 kHz;
inference_commandline_hf.py:222-231 writes the generated wav with soundfile).

torchaudio and soundfile are not part of this image, so:
* ``load_audio`` reads WAV (PCM 8/16/24/32-bit, IEEE float) with the standard library
  (soundfile, when importable, for other containers), honouring torchaudio.load's
  ``frame_offset`` / ``num_frames`` semantics, as float32 [channels, samples] in [-1, 1];
* ``resample`` restates torchaudio.functional.resample's default band-limited sinc
  interpolation (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99; output length
  ceil(n * new / old)) with torch ops on the waveform's device -- parity against
  torchaudio itself is unpinned here (torchaudio absent);
* ``write_wav`` writes 16-bit PCM like soundfile's default WAV subtype.
"""
from __future__ import annotations

import math
import struct
import wave
from typing import Tuple

import numpy as np
import torch


def _read_wav_stdlib(path: str) -> Tuple[np.ndarray, int]:
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError(f"{path}: missing fmt/data chunk")
    tag, ch, sr, _, _, bits = fmt
    if tag == 0xFFFE:   # WAVE_FORMAT_EXTENSIBLE: sub-format in the extension
        tag = 3 if bits in (32, 64) and b"\x03\x00\x00\x00\x00\x00\x10\x00" in data[:200] else 1
    if tag == 3:
        x = np.frombuffer(pcm, dtype="<f4" if bits == 32 else "<f8").astype(np.float32)
    elif bits == 8:
        x = (np.frombuffer(pcm, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    elif bits == 16:
        x = np.frombuffer(pcm, dtype="<i2").astype(np.float32) / 32768.0
    elif bits == 24:
        b = np.frombuffer(pcm, dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
    elif bits == 32:
        x = np.frombuffer(pcm, dtype="<i4").astype(np.float32) / float(1 << 31)
    else:
        raise ValueError(f"{path}: unsupported {bits}-bit PCM")
    n = len(x) // ch
    return x[:n * ch].reshape(n, ch).T.copy(), int(sr)


def load_audio(path: str, frame_offset: int = 0, num_frames: int = -1) -> Tuple[torch.Tensor, int]:
    """torchaudio.load(path, frame_offset, num_frames) -> (float32 [C, N], sample_rate)."""
    try:
        x, sr = _read_wav_stdlib(path)
    except ValueError:
        try:
            import soundfile as sf
        except ImportError as e:
            raise ValueError(f"{path}: only WAV is readable without soundfile") from e
        a, sr = sf.read(path, dtype="float32", always_2d=True)
        x = a.T.copy()
    start = max(0, int(frame_offset or 0))
    end = x.shape[1] if num_frames is None or num_frames < 0 else min(x.shape[1], start + int(num_frames))
    return torch.from_numpy(np.ascontiguousarray(x[:, start:end])), int(sr)


def audio_info(path: str) -> Tuple[int, int]:
    """(num_frames, sample_rate) of a WAV file (torchaudio.info / soundfile.info)."""
    try:
        with wave.open(path, "rb") as w:
            return w.getnframes(), w.getframerate()
    except wave.Error:
        x, sr = _read_wav_stdlib(path)
        return x.shape[1], sr


def _sinc_kernel(orig: int, new: int, width_f: int = 6, rolloff: float = 0.99, device=None):
    base = min(orig, new) * rolloff
    width = math.ceil(width_f * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64, device=device)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float64, device=device)[:, None, None] / new + idx
    t = (t * base).clamp(-width_f, width_f)
    window = torch.cos(t * math.pi / width_f / 2) ** 2
    t = t * math.pi
    k = torch.where(t == 0, torch.ones_like(t), torch.sin(t) / t) * window * (base / orig)
    return k.to(torch.float32), width


def resample(wav: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.functional.resample(wav, orig_freq, new_freq) with its defaults."""
    if orig_freq == new_freq:
        return wav
    g = math.gcd(int(orig_freq), int(new_freq))
    o, n = int(orig_freq) // g, int(new_freq) // g
    k, width = _sinc_kernel(o, n, device=wav.device)
    shape = wav.shape
    x = wav.reshape(-1, shape[-1]).float()
    L = x.shape[-1]
    x = torch.nn.functional.pad(x, (width, width + o))
    y = torch.nn.functional.conv1d(x[:, None], k.to(x.device), stride=o)
    y = y.transpose(1, 2).reshape(x.shape[0], -1)[..., :math.ceil(n * L / o)]
    return y.reshape(shape[:-1] + y.shape[-1:])


def write_wav(path: str, wav, sample_rate: int) -> None:
    """Mono float waveform -> 16-bit PCM WAV (soundfile.write's default subtype)."""
    a = np.asarray(wav.detach().cpu().numpy() if isinstance(wav, torch.Tensor) else wav, dtype=np.float64).reshape(-1)
    pcm = np.clip(np.round(a * 32767.0), -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sample_rate))
        w.writeframes(pcm.tobytes())
