"""Whisper auto-transcription of a voice-clone prompt.

Reference boundary (inference_commandline_hf.py:144-150): when ``reference_speech`` is
given without ``reference_text``, the reference runs
``whisper.load_model("large-v3-turbo").transcribe(reference_speech)["text"]`` (the pip
``openai-whisper`` package, absent here) and uses the text as the prompt transcript.

This module keeps that call shape -- ``load_model(name_or_path).transcribe(audio)`` ->
``{"text", "segments", "language"}`` -- with the model arithmetic in libt5gtts.so
(``whs_*`` C ABI, include/whisper.h: log-mel, encoder, decoder with its caches, logits;
fp32 on the f32 MFMA) and openai-whisper's host control flow restated here:
* ``transcribe`` -- language detection on the first 30 s, windows of 3000 mel frames,
  seeking by the last timestamp pair, conditioning on previous text, clearing empty
  segments (whisper/transcribe.py);
* ``decode`` -- greedy decoding at temperature 0, categorical sampling above it, with
  the SuppressBlank / SuppressTokens / ApplyTimestampRules logit filters, the no-speech
  probability at the start-of-transcript position and the fallback tests on compression
  ratio and average log-probability (whisper/decoding.py);
* the tiktoken-format byte-level BPE tokenizer with Whisper's special tokens
  (whisper/tokenizer.py), or a transformers ``tokenizer.json``.
The logit filters are pinned against transformers' port of the same rules
(WhisperTimeStampLogitsProcessor, tests/test_whisper_cpu.py); the model against
transformers' WhisperForConditionalGeneration (tests/test_gpu_whisper.py). Parity with the
openai-whisper package itself is unpinned (package and checkpoint absent).

There is no CPU fallback: without the HIP library the model raises.
"""
from __future__ import annotations

import base64
import ctypes as C
import math
import os
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib

F32 = torch.float32
SAMPLE_RATE, HOP, N_FFT, N_FRAMES = 16000, 160, 400, 3000
N_SAMPLES = N_FRAMES * HOP          # 30 s
FFT_K, BINS, BINS_PAD = 416, 201, 224
MAX_LAYERS = 64

# whisper/tokenizer.py LANGUAGES order (the language tokens follow <|startoftranscript|>)
LANGUAGE_CODES = ("en zh de es ru ko fr ja pt tr pl ca nl ar sv it id hi fi vi he uk el ms cs ro da hu ta no th ur "
                  "hr bg lt la mi ml cy sk te fa lv bn sr az sl kn et mk br eu is hy ne mn bs kk sq sw gl mr pa si "
                  "km sn yo so af oc ka be tg sd gu am yi lo uz fo ht ps tk nn mt sa lb my bo tl mg as tt haw ln ha "
                  "ba jw su yue").split()


# ----------------------------------------------------------------------------- dims
@dataclass
class WhisperDims:
    """openai-whisper ModelDimensions (whisper/model.py)."""
    n_mels: int = 128
    n_audio_ctx: int = 1500
    n_audio_state: int = 1280
    n_audio_head: int = 20
    n_audio_layer: int = 32
    n_vocab: int = 51866
    n_text_ctx: int = 448
    n_text_state: int = 1280
    n_text_head: int = 20
    n_text_layer: int = 4

    @property
    def is_multilingual(self) -> bool:
        return self.n_vocab >= 51865

    @property
    def num_languages(self) -> int:
        return self.n_vocab - 51765 - int(self.is_multilingual)

    @classmethod
    def from_hf_config(cls, d: dict) -> "WhisperDims":
        """From a transformers WhisperConfig dict."""
        return cls(n_mels=d["num_mel_bins"], n_audio_ctx=d["max_source_positions"], n_audio_state=d["d_model"],
                   n_audio_head=d["encoder_attention_heads"], n_audio_layer=d["encoder_layers"],
                   n_vocab=d["vocab_size"], n_text_ctx=d["max_target_positions"], n_text_state=d["d_model"],
                   n_text_head=d["decoder_attention_heads"], n_text_layer=d["decoder_layers"])


def dims_large_v3_turbo() -> WhisperDims:
    return WhisperDims()


def dims_tiny() -> WhisperDims:
    """Reduced test dims (head size 64 as the kernels require), multilingual v3 vocabulary."""
    return WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=2, n_text_state=128,
                       n_text_head=2, n_text_layer=2)


# -------------------------------------------------------------------------- weights
def weight_shapes(d: WhisperDims) -> Dict[str, tuple]:
    """openai-whisper state_dict names and shapes (whisper/model.py)."""
    Ca, Ct = d.n_audio_state, d.n_text_state
    s = {"encoder.conv1.weight": (Ca, d.n_mels, 3), "encoder.conv1.bias": (Ca,),
         "encoder.conv2.weight": (Ca, Ca, 3), "encoder.conv2.bias": (Ca,),
         "encoder.positional_embedding": (d.n_audio_ctx, Ca),
         "encoder.ln_post.weight": (Ca,), "encoder.ln_post.bias": (Ca,),
         "decoder.token_embedding.weight": (d.n_vocab, Ct), "decoder.positional_embedding": (d.n_text_ctx, Ct),
         "decoder.ln.weight": (Ct,), "decoder.ln.bias": (Ct,)}

    def attn(p, c):
        s.update({p + "query.weight": (c, c), p + "query.bias": (c,), p + "key.weight": (c, c),
                  p + "value.weight": (c, c), p + "value.bias": (c,), p + "out.weight": (c, c), p + "out.bias": (c,)})

    def block(p, c, cross):
        attn(p + "attn.", c)
        s.update({p + "attn_ln.weight": (c,), p + "attn_ln.bias": (c,), p + "mlp.0.weight": (4 * c, c),
                  p + "mlp.0.bias": (4 * c,), p + "mlp.2.weight": (c, 4 * c), p + "mlp.2.bias": (c,),
                  p + "mlp_ln.weight": (c,), p + "mlp_ln.bias": (c,)})
        if cross:
            attn(p + "cross_attn.", c)
            s.update({p + "cross_attn_ln.weight": (c,), p + "cross_attn_ln.bias": (c,)})

    for i in range(d.n_audio_layer):
        block(f"encoder.blocks.{i}.", Ca, False)
    for i in range(d.n_text_layer):
        block(f"decoder.blocks.{i}.", Ct, True)
    return s


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    """whisper/model.py sinusoids: [sin | cos] of log-spaced timescales."""
    log_timescale_increment = math.log(max_timescale) / (channels // 2 - 1)
    inv_timescales = torch.exp(-log_timescale_increment * torch.arange(channels // 2))
    scaled_time = torch.arange(length)[:, None] * inv_timescales[None, :]
    return torch.cat([torch.sin(scaled_time), torch.cos(scaled_time)], dim=1)


def synthetic_weights(d: WhisperDims, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Seeded random weights at the openai names (no checkpoint is reachable offline)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name, shp in weight_shapes(d).items():
        if name == "encoder.positional_embedding":
            out[name] = sinusoids(*shp)
        elif name.endswith("ln.weight") or name.endswith("ln_post.weight") or name.endswith("_ln.weight"):
            out[name] = 1.0 + 0.1 * torch.randn(shp, generator=g)
        elif len(shp) == 1:
            out[name] = 0.02 * torch.randn(shp, generator=g)
        else:
            fan_in = shp[1] * (shp[2] if len(shp) == 3 else 1)
            scale = 0.02 if "embedding" in name else 1.0 / math.sqrt(fan_in)
            out[name] = scale * torch.randn(shp, generator=g)
    return out


# transformers WhisperForConditionalGeneration name -> openai name
def hf_to_openai_names(hf: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    rep = [("model.encoder.embed_positions.weight", "encoder.positional_embedding"),
           ("model.decoder.embed_positions.weight", "decoder.positional_embedding"),
           ("model.decoder.embed_tokens.weight", "decoder.token_embedding.weight"),
           ("model.encoder.layer_norm.", "encoder.ln_post."), ("model.decoder.layer_norm.", "decoder.ln."),
           ("model.encoder.conv", "encoder.conv"), ("model.encoder.layers.", "encoder.blocks."),
           ("model.decoder.layers.", "decoder.blocks."), (".self_attn_layer_norm.", ".attn_ln."),
           (".encoder_attn_layer_norm.", ".cross_attn_ln."), (".final_layer_norm.", ".mlp_ln."),
           (".self_attn.", ".attn."), (".encoder_attn.", ".cross_attn."), (".q_proj.", ".query."),
           (".k_proj.", ".key."), (".v_proj.", ".value."), (".out_proj.", ".out."), (".fc1.", ".mlp.0."),
           (".fc2.", ".mlp.2.")]
    out = {}
    for k, v in hf.items():
        if k == "proj_out.weight":
            continue                      # tied to the token embedding
        n = k
        for a, b in rep:
            n = n.replace(a, b)
        out[n] = v
    return out


def default_download_root() -> str:
    return os.path.join(os.getenv("XDG_CACHE_HOME", os.path.join(os.path.expanduser("~"), ".cache")), "whisper")


def load_checkpoint(name_or_path: str, download_root: Optional[str] = None
                    ) -> Tuple[WhisperDims, Dict[str, torch.Tensor], Optional[str]]:
    """(dims, openai-named state dict, directory holding it) from
    * an openai-whisper checkpoint ``<name>.pt`` ({"dims", "model_state_dict"}, read with
      torch.load(weights_only=True)) -- a model name resolves to
      ``<download_root or ~/.cache/whisper>/<name>.pt`` as whisper.load_model does, but is
      never downloaded;
    * or a transformers directory (config.json + *.safetensors)."""
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(download_root or default_download_root(), f"{name_or_path}.pt")
    if not os.path.exists(path):
        raise FileNotFoundError(f"Whisper checkpoint {name_or_path!r} not found (looked for {path}); there is no "
                                "download path here: pass a local .pt / transformers directory")
    if os.path.isdir(path):
        import json
        from safetensors.torch import load_file
        with open(os.path.join(path, "config.json")) as f:
            dims = WhisperDims.from_hf_config(json.load(f))
        sd = {}
        for fn in sorted(os.listdir(path)):
            if fn.endswith(".safetensors"):
                sd.update(load_file(os.path.join(path, fn)))
        return dims, hf_to_openai_names(sd), path
    ck = torch.load(path, map_location="cpu", weights_only=True)
    return WhisperDims(**ck["dims"]), ck["model_state_dict"], os.path.dirname(path)


# --------------------------------------------------------------------- host tables
def hann_window() -> torch.Tensor:
    """torch.hann_window(400) (periodic)."""
    n = torch.arange(N_FFT, dtype=torch.float64)
    return (0.5 - 0.5 * torch.cos(2 * math.pi * n / N_FFT)).to(F32)


def dft_basis() -> torch.Tensor:
    """[402][416]: rows 2k / 2k + 1 = cos / -sin(2 pi k n / 400) for n < 400."""
    n = torch.arange(N_FFT, dtype=torch.float64)
    k = torch.arange(BINS, dtype=torch.float64)[:, None]
    ang = 2 * math.pi * k * n / N_FFT
    B = torch.zeros(2 * BINS, FFT_K, dtype=torch.float64)
    B[0::2, :N_FFT] = torch.cos(ang)
    B[1::2, :N_FFT] = -torch.sin(ang)
    return B.to(F32)


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp, min_log_hz, min_log_mel, logstep = 200.0 / 3, 1000.0, 15.0, math.log(6.4) / 27.0
    mels = f / f_sp
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp, min_log_hz, min_log_mel, logstep = 200.0 / 3, 1000.0, 15.0, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filters(n_mels: int) -> torch.Tensor:
    """librosa.filters.mel(sr=16000, n_fft=400, n_mels, htk=False, norm="slaney") -- the
    table whisper/assets/mel_filters.npz holds -- as [n_mels][224] fp32 (zero padded)."""
    fftfreqs = np.linspace(0, SAMPLE_RATE / 2, BINS)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(0.0), _hz_to_mel(SAMPLE_RATE / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    w = np.zeros((n_mels, BINS))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    out = torch.zeros(n_mels, BINS_PAD, dtype=F32)
    out[:, :BINS] = torch.from_numpy(w.astype(np.float32))
    return out


# ------------------------------------------------------------------------ C ABI
class WHSConfig(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("n_mels", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer",
                                         "n_vocab", "n_text_ctx", "n_text_state", "n_text_head", "n_text_layer",
                                         "max_samples")]


class WHSAttn(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("q_w", "q_b", "k_w", "v_w", "v_b", "o_w", "o_b")]


class WHSBlock(C.Structure):
    _fields_ = [("attn_ln_w", C.c_void_p), ("attn_ln_b", C.c_void_p), ("attn", WHSAttn),
                ("cross_ln_w", C.c_void_p), ("cross_ln_b", C.c_void_p), ("cross", WHSAttn),
                ("mlp_ln_w", C.c_void_p), ("mlp_ln_b", C.c_void_p), ("fc1_w", C.c_void_p), ("fc1_b", C.c_void_p),
                ("fc2_w", C.c_void_p), ("fc2_b", C.c_void_p)]


class WHSWeights(C.Structure):
    _fields_ = [("window", C.c_void_p), ("dft", C.c_void_p), ("mel", C.c_void_p), ("conv1_w", C.c_void_p),
                ("conv1_b", C.c_void_p), ("conv2_w", C.c_void_p), ("conv2_b", C.c_void_p),
                ("conv1_kpad", C.c_int32), ("conv2_kpad", C.c_int32), ("enc_pos", C.c_void_p),
                ("enc", WHSBlock * MAX_LAYERS), ("enc_ln_w", C.c_void_p), ("enc_ln_b", C.c_void_p),
                ("tok_emb", C.c_void_p), ("dec_pos", C.c_void_p), ("dec", WHSBlock * MAX_LAYERS),
                ("dec_ln_w", C.c_void_p), ("dec_ln_b", C.c_void_p)]


WHS_SIGNATURES = {
    "whs_create": (C.c_int, [C.POINTER(WHSConfig), C.POINTER(WHSWeights), C.POINTER(C.c_void_p)]),
    "whs_destroy": (C.c_int, [C.c_void_p]),
    "whs_workspace_bytes": (C.c_int64, [C.c_void_p]),
    "whs_mel_frames": (C.c_int32, [C.c_void_p, C.c_int32]),
    "whs_log_mel": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "whs_encode": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "whs_decode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
}


class WhisperModel:
    """Device-resident Whisper (batch 1) behind the whs_* ABI, with openai-whisper's
    ``transcribe`` / ``detect_language`` entry points."""

    def __init__(self, dims: WhisperDims, state_dict: Dict[str, torch.Tensor], device="cuda:0",
                 max_seconds: float = 120.0, tokenizer: Optional["WhisperTokenizer"] = None):
        if dims.n_audio_state != dims.n_text_state or dims.n_audio_state != 64 * dims.n_audio_head or \
                dims.n_text_state != 64 * dims.n_text_head:
            raise ValueError("the Whisper kernels need head size 64 and equal audio / text widths")
        if max(dims.n_audio_layer, dims.n_text_layer) > MAX_LAYERS:
            raise ValueError("layer count exceeds the ABI tables")
        if 2 * dims.n_audio_ctx != N_FRAMES:
            raise ValueError("n_audio_ctx must be 1500 (30 s windows)")
        self.dims, self.device = dims, torch.device(device)
        self.tokenizer = tokenizer
        self.max_samples = int(max_seconds * SAMPLE_RATE)
        self.L = _lib.lib()
        for name, (res, args) in WHS_SIGNATURES.items():
            fn = getattr(self.L, name)
            fn.restype, fn.argtypes = res, args
        self._keep = []
        dev = self.device

        def t(x: torch.Tensor) -> int:
            x = x.to(device=dev, dtype=F32).contiguous()
            self._keep.append(x)
            return x.data_ptr()

        def w(name):
            if name not in state_dict:
                raise KeyError(f"missing Whisper weight {name}")
            return state_dict[name].to(F32)

        def conv(name) -> Tuple[int, int]:
            x = w(name)                                  # [co][ci][k]
            co, ci, k = x.shape
            kpad = (k * ci + 31) // 32 * 32
            tm = torch.zeros(co, kpad, dtype=F32)
            tm[:, :k * ci] = x.permute(0, 2, 1).reshape(co, k * ci)
            return t(tm), kpad

        def attn(p) -> WHSAttn:
            return WHSAttn(q_w=t(w(p + "query.weight")), q_b=t(w(p + "query.bias")), k_w=t(w(p + "key.weight")),
                           v_w=t(w(p + "value.weight")), v_b=t(w(p + "value.bias")), o_w=t(w(p + "out.weight")),
                           o_b=t(w(p + "out.bias")))

        def block(b: WHSBlock, p: str, cross: bool):
            b.attn_ln_w, b.attn_ln_b = t(w(p + "attn_ln.weight")), t(w(p + "attn_ln.bias"))
            b.attn = attn(p + "attn.")
            if cross:
                b.cross_ln_w, b.cross_ln_b = t(w(p + "cross_attn_ln.weight")), t(w(p + "cross_attn_ln.bias"))
                b.cross = attn(p + "cross_attn.")
            b.mlp_ln_w, b.mlp_ln_b = t(w(p + "mlp_ln.weight")), t(w(p + "mlp_ln.bias"))
            b.fc1_w, b.fc1_b = t(w(p + "mlp.0.weight")), t(w(p + "mlp.0.bias"))
            b.fc2_w, b.fc2_b = t(w(p + "mlp.2.weight")), t(w(p + "mlp.2.bias"))

        W = WHSWeights()
        W.window, W.dft, W.mel = t(hann_window()), t(dft_basis()), t(mel_filters(dims.n_mels))
        W.conv1_w, W.conv1_kpad = conv("encoder.conv1.weight")
        W.conv2_w, W.conv2_kpad = conv("encoder.conv2.weight")
        W.conv1_b, W.conv2_b = t(w("encoder.conv1.bias")), t(w("encoder.conv2.bias"))
        W.enc_pos = t(w("encoder.positional_embedding"))
        for i in range(dims.n_audio_layer):
            block(W.enc[i], f"encoder.blocks.{i}.", False)
        W.enc_ln_w, W.enc_ln_b = t(w("encoder.ln_post.weight")), t(w("encoder.ln_post.bias"))
        W.tok_emb, W.dec_pos = t(w("decoder.token_embedding.weight")), t(w("decoder.positional_embedding"))
        for i in range(dims.n_text_layer):
            block(W.dec[i], f"decoder.blocks.{i}.", True)
        W.dec_ln_w, W.dec_ln_b = t(w("decoder.ln.weight")), t(w("decoder.ln.bias"))
        self._w = W
        kc = WHSConfig(n_mels=dims.n_mels, n_audio_ctx=dims.n_audio_ctx, n_audio_state=dims.n_audio_state,
                       n_audio_head=dims.n_audio_head, n_audio_layer=dims.n_audio_layer, n_vocab=dims.n_vocab,
                       n_text_ctx=dims.n_text_ctx, n_text_state=dims.n_text_state, n_text_head=dims.n_text_head,
                       n_text_layer=dims.n_text_layer, max_samples=self.max_samples)
        self._kc = kc
        h = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(self.L.whs_create(C.byref(kc), C.byref(W), C.byref(h)), "whs_create")
        self.h = h
        self.mel_frames = 0
        self._tok = torch.empty(dims.n_text_ctx, dtype=torch.int32, device=dev)
        self._logits = torch.empty(dims.n_text_ctx, dims.n_vocab, dtype=F32, device=dev)

    def close(self):
        if getattr(self, "h", None):
            self.L.whs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def is_multilingual(self) -> bool:
        return self.dims.is_multilingual

    @property
    def num_languages(self) -> int:
        return self.dims.num_languages

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- device steps -------------------------------------------------------------
    def log_mel(self, audio: torch.Tensor, out: bool = False) -> Optional[torch.Tensor]:
        """log_mel_spectrogram(audio, n_mels, padding=N_SAMPLES) into the device buffer
        (frames = n // 160 + 3000); out=True also returns it as [frames][n_mels]."""
        x = audio.reshape(-1).to(device=self.device, dtype=F32).contiguous()
        n = int(x.numel())
        if n > self.max_samples:
            raise ValueError(f"{n} samples exceed the recognizer capacity ({self.max_samples})")
        frames = int(self.L.whs_mel_frames(self.h, n))
        mel = torch.empty(frames, self.dims.n_mels, dtype=F32, device=self.device) if out else None
        _lib.check(self.L.whs_log_mel(self.h, C.c_void_p(x.data_ptr() if n else None), n,
                                      C.c_void_p(mel.data_ptr() if mel is not None else None), self._stream()),
                   "whs_log_mel")
        self.mel_frames = frames
        return mel

    def encode(self, seek: int, seg_frames: int, out: bool = False) -> Optional[torch.Tensor]:
        """AudioEncoder over mel rows [seek, seek + seg_frames), zero padded to 3000."""
        feat = torch.empty(self.dims.n_audio_ctx, self.dims.n_audio_state, dtype=F32,
                           device=self.device) if out else None
        _lib.check(self.L.whs_encode(self.h, int(seek), int(seg_frames),
                                     C.c_void_p(feat.data_ptr() if feat is not None else None), self._stream()),
                   "whs_encode")
        return feat

    def logits(self, tokens: Sequence[int], offset: int) -> torch.Tensor:
        """TextDecoder logits [n][n_vocab] (device) for tokens at positions offset.."""
        n = len(tokens)
        if n == 0 or offset + n > self.dims.n_text_ctx:
            raise ValueError(f"decoder context exceeded ({offset} + {n} > {self.dims.n_text_ctx})")
        self._tok[:n].copy_(torch.tensor(list(tokens), dtype=torch.int32), non_blocking=False)
        _lib.check(self.L.whs_decode(self.h, C.c_void_p(self._tok.data_ptr()), n, int(offset),
                                     C.c_void_p(self._logits.data_ptr()), self._stream()), "whs_decode")
        return self._logits[:n]

    # -- openai-whisper entry points --------------------------------------------------
    def detect_language(self, tokenizer: "WhisperTokenizer") -> Tuple[str, Dict[str, float]]:
        """whisper/decoding.py detect_language on the first 3000 frames of the last log_mel
        (the padded mel, as transcribe passes pad_or_trim(mel, N_FRAMES))."""
        self.encode(0, N_FRAMES)
        logits = self.logits([tokenizer.sot], 0)[0].float().cpu()
        mask = torch.ones(logits.shape[-1], dtype=torch.bool)
        mask[list(tokenizer.all_language_tokens)] = False
        logits[mask] = -np.inf
        probs = logits.softmax(dim=-1)
        lp = {c: probs[j].item() for j, c in zip(tokenizer.all_language_tokens, tokenizer.all_language_codes)}
        return max(lp, key=lp.get), lp

    def transcribe(self, audio, **kwargs) -> dict:
        return transcribe(self, audio, **kwargs)


# -------------------------------------------------------------------------- tokenizer
_PAT = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


class _BPE:
    """tiktoken-format byte-level BPE: regex pre-split, then repeated merge of the adjacent
    pair with the lowest rank (leftmost first) -- tiktoken's _byte_pair_merge."""

    def __init__(self, ranks: Dict[bytes, int]):
        import regex
        self.ranks = ranks
        self.inv = {v: k for k, v in ranks.items()}
        self.pat = regex.compile(_PAT)

    def _merge(self, piece: bytes) -> List[int]:
        if piece in self.ranks:
            return [self.ranks[piece]]
        parts = [piece[i:i + 1] for i in range(len(piece))]
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get(parts[i] + parts[i + 1])
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if bi < 0:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        return [self.ranks[p] for p in parts]

    def encode(self, text: str) -> List[int]:
        out = []
        for m in self.pat.finditer(text):
            out.extend(self._merge(m.group().encode("utf-8")))
        return out

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        return b"".join(self.inv[i] for i in ids)


class _HFCore:
    """A transformers tokenizer.json (byte-level BPE) as the ordinary-token core."""

    def __init__(self, path: str):
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(path)

    def encode(self, text: str) -> List[int]:
        return self.tok.encode(text, add_special_tokens=False).ids

    def decode_bytes(self, ids: Sequence[int]) -> bytes:
        return self.tok.decode(list(ids), skip_special_tokens=False).encode("utf-8")


def load_tiktoken_ranks(path: str) -> Dict[bytes, int]:
    ranks = {}
    with open(path) as f:
        for line in f:
            if line.strip():
                tok, rank = line.split()
                ranks[base64.b64decode(tok)] = int(rank)
    return ranks


class WhisperTokenizer:
    """whisper/tokenizer.py Tokenizer (multilingual): ordinary tokens from the BPE core, then
    <|endoftext|>, <|startoftranscript|>, one token per language, <|translate|>,
    <|transcribe|>, <|startoflm|>, <|startofprev|>, <|nospeech|>, <|notimestamps|> and 1501
    timestamps <|0.00|> .. <|30.00|>."""

    def __init__(self, core, n_ordinary: int, num_languages: int = 100, language: Optional[str] = None,
                 task: str = "transcribe"):
        self.core, self.n_ordinary = core, n_ordinary
        self.num_languages = num_languages
        codes = LANGUAGE_CODES[:num_languages]
        specials = ["<|endoftext|>", "<|startoftranscript|>"] + [f"<|{c}|>" for c in codes] + \
            ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nospeech|>",
             "<|notimestamps|>"] + [f"<|{i * 0.02:.2f}|>" for i in range(1501)]
        self.special = {s: n_ordinary + i for i, s in enumerate(specials)}
        self.special_text = {v: k for k, v in self.special.items()}
        self.n_vocab = n_ordinary + len(specials)
        self.language = language
        self.task = task

    @classmethod
    def from_tiktoken(cls, path: str, num_languages: int = 100, **kw) -> "WhisperTokenizer":
        ranks = load_tiktoken_ranks(path)
        return cls(_BPE(ranks), len(ranks), num_languages, **kw)

    @classmethod
    def from_hf_json(cls, path: str, num_languages: int = 100, **kw) -> "WhisperTokenizer":
        core = _HFCore(path)
        eot = core.tok.token_to_id("<|endoftext|>")
        if eot is None:
            raise ValueError(f"{path}: no <|endoftext|> token")
        return cls(core, eot, num_languages, **kw)

    def with_language(self, language: Optional[str], task: str = "transcribe") -> "WhisperTokenizer":
        t = WhisperTokenizer.__new__(WhisperTokenizer)
        t.__dict__.update(self.__dict__)
        t.language, t.task = language, task
        return t

    # ids
    @property
    def eot(self) -> int:
        return self.special["<|endoftext|>"]

    @property
    def sot(self) -> int:
        return self.special["<|startoftranscript|>"]

    @property
    def transcribe(self) -> int:
        return self.special["<|transcribe|>"]

    @property
    def translate(self) -> int:
        return self.special["<|translate|>"]

    @property
    def sot_lm(self) -> int:
        return self.special["<|startoflm|>"]

    @property
    def sot_prev(self) -> int:
        return self.special["<|startofprev|>"]

    @property
    def no_speech(self) -> int:
        return self.special["<|nospeech|>"]

    @property
    def no_timestamps(self) -> int:
        return self.special["<|notimestamps|>"]

    @property
    def timestamp_begin(self) -> int:
        return self.special["<|0.00|>"]

    @property
    def all_language_codes(self) -> Tuple[str, ...]:
        return tuple(LANGUAGE_CODES[:self.num_languages])

    @property
    def all_language_tokens(self) -> Tuple[int, ...]:
        return tuple(self.special[f"<|{c}|>"] for c in self.all_language_codes)

    @property
    def sot_sequence(self) -> Tuple[int, ...]:
        seq = [self.sot]
        if self.language is not None:
            seq.append(self.sot + 1 + LANGUAGE_CODES.index(self.language))
        if self.task is not None:
            seq.append(self.transcribe if self.task == "transcribe" else self.translate)
        return tuple(seq)

    @property
    def sot_sequence_including_notimestamps(self) -> Tuple[int, ...]:
        return tuple(list(self.sot_sequence) + [self.no_timestamps])

    # text
    def encode(self, text: str) -> List[int]:
        return self.core.encode(text)

    def decode(self, ids: Sequence[int]) -> str:
        """Timestamps dropped, special tokens as their text (whisper Tokenizer.decode)."""
        out, run = [], []
        for i in ids:
            i = int(i)
            if i >= self.timestamp_begin:
                continue
            if i >= self.n_ordinary:
                if run:
                    out.append(self.core.decode_bytes(run))
                    run = []
                out.append(self.special_text[i].encode("utf-8"))
            else:
                run.append(i)
        if run:
            out.append(self.core.decode_bytes(run))
        return b"".join(out).decode("utf-8", errors="replace")

    @property
    def non_speech_tokens(self) -> Tuple[int, ...]:
        """whisper Tokenizer.non_speech_tokens: symbols / speaker tags that are suppressed."""
        symbols = list('"#()*+/:;<=>@[\\]^_`{|}~「」『』')
        symbols += "<< >> <<< >>> -- --- -( -[ (' (\" (( )) ((( ))) [[ ]] {{ }} ♪♪ ♪♪♪".split()
        miscellaneous = set("♩♪♫♬♭♮♯")
        assert all(0x2640 <= ord(c) <= 0x267F for c in miscellaneous)
        result = {self.encode(" -")[0], self.encode(" '")[0]}
        for symbol in symbols + list(miscellaneous):
            for tokens in [self.encode(symbol), self.encode(" " + symbol)]:
                if len(tokens) == 1 or symbol in miscellaneous:
                    result.add(tokens[0])
        return tuple(sorted(result))


def default_tokenizer(num_languages: int, search_dirs: Sequence[Optional[str]] = ()) -> WhisperTokenizer:
    """openai's multilingual.tiktoken (or a transformers tokenizer.json) from the checkpoint's
    directory or ~/.cache/whisper; raises if neither is present (no download path)."""
    dirs = [d for d in search_dirs if d] + [default_download_root()]
    for d in dirs:
        p = os.path.join(d, "multilingual.tiktoken")
        if os.path.exists(p):
            return WhisperTokenizer.from_tiktoken(p, num_languages)
        p = os.path.join(d, "tokenizer.json")
        if os.path.exists(p):
            return WhisperTokenizer.from_hf_json(p, num_languages)
    raise FileNotFoundError(f"Whisper tokenizer (multilingual.tiktoken or tokenizer.json) not found in {dirs}")


def load_model(name: str = "large-v3-turbo", device="cuda:0", download_root: Optional[str] = None,
               tokenizer: Optional[WhisperTokenizer] = None, max_seconds: float = 120.0) -> WhisperModel:
    """whisper.load_model: a local checkpoint by name or path (see load_checkpoint)."""
    dims, sd, where = load_checkpoint(name, download_root)
    if tokenizer is None:
        tokenizer = default_tokenizer(dims.num_languages, [where])
    return WhisperModel(dims, sd, device=device, tokenizer=tokenizer, max_seconds=max_seconds)


# ---------------------------------------------------------------------------- decoding
@dataclass
class DecodingOptions:
    """whisper/decoding.py DecodingOptions (greedy / sampling subset; beam search is not
    used by the reference's transcribe() call)."""
    task: str = "transcribe"
    language: Optional[str] = None
    temperature: float = 0.0
    sample_len: Optional[int] = None
    prompt: Optional[Union[str, List[int]]] = None
    suppress_tokens: Optional[Union[str, Sequence[int]]] = "-1"
    suppress_blank: bool = True
    without_timestamps: bool = False
    max_initial_timestamp: Optional[float] = 1.0


@dataclass
class DecodingResult:
    language: str
    tokens: List[int] = field(default_factory=list)
    text: str = ""
    avg_logprob: float = float("nan")
    no_speech_prob: float = float("nan")
    temperature: float = float("nan")
    compression_ratio: float = float("nan")


def compression_ratio(text: str) -> float:
    b = text.encode("utf-8")
    return len(b) / len(zlib.compress(b))


def suppress_blank(logits: torch.Tensor, tokens: List[int], sample_begin: int, tok: WhisperTokenizer):
    """SuppressBlank: at the first sampled position, no blank and no end-of-text."""
    if len(tokens) == sample_begin:
        logits[tok.encode(" ") + [tok.eot]] = -np.inf


def apply_timestamp_rules(logits: torch.Tensor, tokens: List[int], sample_begin: int, tok: WhisperTokenizer,
                          max_initial_timestamp_index: Optional[int]):
    """ApplyTimestampRules (one sequence): timestamps in pairs except before end-of-text,
    non-decreasing and non-repeating, a timestamp first (at most max_initial), and a forced
    timestamp when their total probability beats every text token."""
    tb = tok.timestamp_begin
    logits[tok.no_timestamps] = -np.inf
    seq = tokens[sample_begin:]
    last_was_timestamp = len(seq) >= 1 and seq[-1] >= tb
    penultimate_was_timestamp = len(seq) < 2 or seq[-2] >= tb
    if last_was_timestamp:
        if penultimate_was_timestamp:
            logits[tb:] = -np.inf
        else:
            logits[:tok.eot] = -np.inf
    timestamps = [t for t in seq if t >= tb]
    if timestamps:
        timestamp_last = timestamps[-1] if (last_was_timestamp and not penultimate_was_timestamp) else timestamps[-1] + 1
        logits[tb:timestamp_last] = -np.inf
    if len(tokens) == sample_begin:
        logits[:tb] = -np.inf
        if max_initial_timestamp_index is not None:
            logits[tb + max_initial_timestamp_index + 1:] = -np.inf
    logprobs = torch.log_softmax(logits.float(), dim=-1)
    if logprobs[tb:].logsumexp(dim=-1) > logprobs[:tb].max():
        logits[:tb] = -np.inf


def suppress_token_list(tok: WhisperTokenizer, suppress_tokens) -> Tuple[int, ...]:
    """DecodingTask._get_suppress_tokens."""
    if suppress_tokens is None:
        st: List[int] = []
    elif isinstance(suppress_tokens, str):
        st = [int(t) for t in suppress_tokens.split(",")]
    else:
        st = list(suppress_tokens)
    if -1 in st:
        st = [t for t in st if t >= 0]
        st.extend(tok.non_speech_tokens)
    st.extend([tok.transcribe, tok.translate, tok.sot, tok.sot_prev, tok.sot_lm])
    if tok.no_speech is not None:
        st.append(tok.no_speech)
    return tuple(sorted(set(st)))


def decode(model: WhisperModel, seek: int, seg_frames: int, options: DecodingOptions,
           tokenizer: WhisperTokenizer, generator: Optional[torch.Generator] = None) -> DecodingResult:
    """whisper/decoding.py DecodingTask.run for one window of the last log_mel (n_group 1)."""
    tok = tokenizer.with_language(options.language, options.task)
    n_ctx = model.dims.n_text_ctx
    sample_len = options.sample_len or n_ctx // 2
    sot_seq = list(tok.sot_sequence_including_notimestamps if options.without_timestamps else tok.sot_sequence)
    initial = list(sot_seq)
    if options.prompt:
        pt = tok.encode(" " + options.prompt.strip()) if isinstance(options.prompt, str) else list(options.prompt)
        initial = [tok.sot_prev] + pt[-(n_ctx // 2 - 1):] + initial
    sample_begin = len(initial)
    sot_index = initial.index(tok.sot)
    suppress = list(suppress_token_list(tok, options.suppress_tokens)) if options.suppress_tokens else []
    max_init = None
    if options.max_initial_timestamp:
        max_init = round(options.max_initial_timestamp / (30.0 / model.dims.n_audio_ctx))
    model.encode(seek, seg_frames)
    tokens = list(initial)
    sum_logprob, no_speech_prob = 0.0, float("nan")
    fed = 0
    for i in range(sample_len):
        lg = model.logits(tokens[fed:], fed)
        if i == 0:
            no_speech_prob = lg[sot_index - fed].float().softmax(-1)[tok.no_speech].item()
        logits = lg[-1].float().cpu()
        fed = len(tokens)
        if options.suppress_blank:
            suppress_blank(logits, tokens, sample_begin, tok)
        if suppress:
            logits[suppress] = -np.inf
        if not options.without_timestamps:
            apply_timestamp_rules(logits, tokens, sample_begin, tok, max_init)
        if options.temperature == 0:
            nxt = int(logits.argmax())
        else:
            probs = torch.softmax(logits / options.temperature, dim=-1)
            nxt = int(torch.multinomial(probs, 1, generator=generator))
        lp = torch.log_softmax(logits, dim=-1)[nxt].item()
        if tokens[-1] != tok.eot:
            sum_logprob += lp
        else:
            nxt = tok.eot
        tokens.append(nxt)
        if nxt == tok.eot or len(tokens) > n_ctx:
            break
    out = tokens[sample_begin:]
    if tok.eot in out:
        out = out[:out.index(tok.eot)]
    text = tok.decode(out).strip()
    return DecodingResult(language=options.language, tokens=out, text=text, avg_logprob=sum_logprob / (len(out) + 1),
                          no_speech_prob=no_speech_prob, temperature=options.temperature,
                          compression_ratio=compression_ratio(text))


def transcribe(model: WhisperModel, audio, *, temperature: Union[float, Tuple[float, ...]] = (0.0, 0.2, 0.4, 0.6,
                                                                                            0.8, 1.0),
               compression_ratio_threshold: Optional[float] = 2.4, logprob_threshold: Optional[float] = -1.0,
               no_speech_threshold: Optional[float] = 0.6, condition_on_previous_text: bool = True,
               initial_prompt: Optional[str] = None, language: Optional[str] = None, task: str = "transcribe",
               tokenizer: Optional[WhisperTokenizer] = None, generator: Optional[torch.Generator] = None,
               **decode_options) -> dict:
    """whisper/transcribe.py transcribe (no word timestamps, clip_timestamps "0").
    audio: path (any rate, resampled to 16 kHz) or 16 kHz float samples."""
    decode_options = dict(decode_options)
    for k in ("fp16", "verbose", "word_timestamps", "clip_timestamps", "hallucination_silence_threshold"):
        decode_options.pop(k, None)
    if decode_options.pop("beam_size", None) is not None or decode_options.pop("best_of", None) is not None:
        raise NotImplementedError("beam search / best-of sampling are not used by the reference and not built")
    tok = tokenizer or model.tokenizer
    if tok is None:
        raise ValueError("a WhisperTokenizer is required (load_model finds multilingual.tiktoken)")
    if not model.is_multilingual:
        raise NotImplementedError("English-only Whisper vocabularies are not supported")
    if isinstance(audio, str):
        from .audio import load_audio, resample
        x, sr = load_audio(audio)
        audio = resample(x, sr, SAMPLE_RATE).mean(0) if x.dim() > 1 else resample(x[None], sr, SAMPLE_RATE)[0]
    audio = torch.as_tensor(audio, dtype=F32).reshape(-1)
    model.log_mel(audio)
    content_frames = model.mel_frames - N_FRAMES
    if language is None:
        language, _ = model.detect_language(tok.with_language("en"))
    tok = tok.with_language(language, task)
    temps = [temperature] if isinstance(temperature, (int, float)) else list(temperature)
    input_stride = N_FRAMES // model.dims.n_audio_ctx
    time_precision = input_stride * HOP / SAMPLE_RATE
    all_tokens: List[int] = []
    all_segments: List[dict] = []
    prompt_reset_since = 0
    initial_prompt_tokens = tok.encode(" " + initial_prompt.strip()) if initial_prompt is not None else []
    all_tokens.extend(initial_prompt_tokens)

    def decode_with_fallback(seek, seg):
        res = None
        for t in temps:
            opts = DecodingOptions(task=task, language=language, temperature=t,
                                   prompt=all_tokens[prompt_reset_since:], **decode_options)
            res = decode(model, seek, seg, opts, tok, generator)
            needs_fallback = False
            if compression_ratio_threshold is not None and res.compression_ratio > compression_ratio_threshold:
                needs_fallback = True
            if logprob_threshold is not None and res.avg_logprob < logprob_threshold:
                needs_fallback = True
            if no_speech_threshold is not None and res.no_speech_prob > no_speech_threshold and \
                    logprob_threshold is not None and res.avg_logprob < logprob_threshold:
                needs_fallback = False
            if not needs_fallback:
                break
        return res

    def new_segment(start, end, tokens, res):
        text_tokens = [t for t in tokens if t < tok.eot]
        return {"seek": seek, "start": start, "end": end, "text": tok.decode(text_tokens), "tokens": list(tokens),
                "temperature": res.temperature, "avg_logprob": res.avg_logprob,
                "compression_ratio": res.compression_ratio, "no_speech_prob": res.no_speech_prob}

    seek = 0
    while seek < content_frames:
        time_offset = seek * HOP / SAMPLE_RATE
        segment_size = min(N_FRAMES, content_frames - seek)
        segment_duration = segment_size * HOP / SAMPLE_RATE
        res = decode_with_fallback(seek, segment_size)
        tokens = res.tokens
        if no_speech_threshold is not None:
            should_skip = res.no_speech_prob > no_speech_threshold
            if logprob_threshold is not None and res.avg_logprob > logprob_threshold:
                should_skip = False
            if should_skip:
                seek += segment_size
                continue
        current = []
        is_ts = [t >= tok.timestamp_begin for t in tokens]
        single_timestamp_ending = is_ts[-2:] == [False, True]
        consecutive = [i + 1 for i in range(len(tokens) - 1) if is_ts[i] and is_ts[i + 1]]
        if consecutive:
            slices = list(consecutive)
            if single_timestamp_ending:
                slices.append(len(tokens))
            last_slice = 0
            for cur in slices:
                st = tokens[last_slice:cur]
                s_pos, e_pos = st[0] - tok.timestamp_begin, st[-1] - tok.timestamp_begin
                current.append(new_segment(time_offset + s_pos * time_precision, time_offset + e_pos * time_precision,
                                           st, res))
                last_slice = cur
            if single_timestamp_ending:
                seek += segment_size
            else:
                seek += (tokens[last_slice - 1] - tok.timestamp_begin) * input_stride
        else:
            duration = segment_duration
            ts = [t for t in tokens if t >= tok.timestamp_begin]
            if ts and ts[-1] != tok.timestamp_begin:
                duration = (ts[-1] - tok.timestamp_begin) * time_precision
            current.append(new_segment(time_offset, time_offset + duration, tokens, res))
            seek += segment_size
        for s in current:
            if s["start"] == s["end"] or s["text"].strip() == "":
                s["text"], s["tokens"] = "", []
        for s in current:
            s["id"] = len(all_segments)
            all_segments.append(s)
        all_tokens.extend([t for s in current for t in s["tokens"]])
        if not condition_on_previous_text or res.temperature > 0.5:
            prompt_reset_since = len(all_tokens)
    return {"text": tok.decode(all_tokens[len(initial_prompt_tokens):]), "segments": all_segments,
            "language": language}
