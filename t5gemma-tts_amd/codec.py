"""XCodec2 codec decoder on MI355X: the `AudioTokenizer.decode` half of the hot path.

Reference boundary: ``AudioTokenizer.decode(frames)`` (data/tokenizer.py:117-123), called
by inference_tts_utils.py:359 and :363 on the frames ``inference_tts`` returns. The
reference delegates to the pip ``xcodec2==0.1.7`` package (absent from the reference
tree); the architecture is restated from the in-container transformers port
([tf] models/xcodec2/modeling_xcodec2.py), whose state-dict key names this module reads.

All compute runs in libt5gtts.so (``xc2_*`` C ABI, include/xc2.h); this module only
lays the fp32 weights out for the kernels (tap-major convolutions, fused q/k/v,
interleaved magnitude/phase head rows, the windowed irfft basis) and calls the ABI.
There is no CPU fallback: a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, Optional, Sequence

import torch

from . import _lib

F32 = torch.float32


@dataclass
class CodecConfig:
    """Decoder hyper-parameters ([tf] configuration_xcodec2.py:61-115)."""
    hidden_size: int = 1024
    intermediate_size: int = 4096
    num_hidden_layers: int = 12
    num_attention_heads: int = 16
    head_dim: int = 64
    quantization_dim: int = 2048
    quantization_levels: Sequence[int] = field(default_factory=lambda: (4,) * 8)
    downsampling_ratios: Sequence[int] = (2, 2, 4, 4, 5)
    sampling_rate: int = 16000
    rope_theta: float = 10000.0
    rms_norm_eps: float = 1e-6
    n_groups: int = 32

    @property
    def hop_length(self) -> int:
        return int(math.prod(self.downsampling_ratios))

    @property
    def n_fft(self) -> int:
        return 4 * self.hop_length

    @property
    def spec_ld(self) -> int:
        return (self.n_fft + 2 + 31) // 32 * 32

    @property
    def codebook_size(self) -> int:
        return int(math.prod(self.quantization_levels))

    @classmethod
    def from_hf_dict(cls, d: dict) -> "CodecConfig":
        rp = d.get("rope_parameters") or {}
        return cls(hidden_size=d.get("hidden_size", 1024), intermediate_size=d.get("intermediate_size", 4096),
                   num_hidden_layers=d.get("num_hidden_layers", 12),
                   num_attention_heads=d.get("num_attention_heads", 16), head_dim=d.get("head_dim", 64) or 64,
                   quantization_dim=d.get("quantization_dim", 2048),
                   quantization_levels=tuple(d.get("quantization_levels", (4,) * 8)),
                   downsampling_ratios=tuple(d.get("downsampling_ratios", (2, 2, 4, 4, 5))),
                   sampling_rate=d.get("sampling_rate", 16000), rope_theta=rp.get("rope_theta", 10000.0),
                   rms_norm_eps=d.get("rms_norm_eps", 1e-6))


def codec_16k() -> CodecConfig:
    """HKUSTAudio/xcodec2 dims (16 kHz, 320 samples per token)."""
    return CodecConfig()


def codec_44k() -> CodecConfig:
    """Anime-XCodec2-44.1kHz-v2 token rate: 882 samples per token (data/tokenizer.py:93,
    config.py:229). Backbone dims assumed equal to the 16 kHz model (unverified: the
    checkpoint is not in the container)."""
    return CodecConfig(downsampling_ratios=(2, 3, 3, 7, 7), sampling_rate=44100)


def codec_tiny() -> CodecConfig:
    """Reduced-width test config (same structure)."""
    return CodecConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                       quantization_dim=512)


def codec_weight_shapes(cfg: CodecConfig) -> Dict[str, tuple]:
    """Decoder tensors under the transformers Xcodec2Model state-dict names."""
    h, q, nl = cfg.hidden_size, cfg.quantization_dim, len(cfg.quantization_levels)
    s = {"quantizer.project_out.weight": (q, nl), "quantizer.project_out.bias": (q,),
         "acoustic_decoder.fc.weight": (h, q), "acoustic_decoder.fc.bias": (h,),
         "acoustic_decoder.embed.weight": (h, h, 7), "acoustic_decoder.embed.bias": (h,)}
    for net in ("prior_net", "post_net"):
        for i in range(2):
            p = f"acoustic_decoder.{net}.{i}."
            for n in ("norm1", "norm2"):
                s[p + n + ".weight"], s[p + n + ".bias"] = (h,), (h,)
            for n in ("conv1", "conv2"):
                s[p + n + ".weight"], s[p + n + ".bias"] = (h, h, 3), (h,)
    for i in range(cfg.num_hidden_layers):
        p = f"acoustic_decoder.layers.{i}."
        for n in ("q_proj", "k_proj", "v_proj", "o_proj"):
            s[p + f"self_attn.{n}.weight"] = (h, h)
        s[p + "mlp.fc1.weight"] = (cfg.intermediate_size, h)
        s[p + "mlp.fc2.weight"] = (h, cfg.intermediate_size)
        s[p + "input_layernorm.weight"] = (h,)
        s[p + "post_attention_layernorm.weight"] = (h,)
    s["acoustic_decoder.norm.weight"], s["acoustic_decoder.norm.bias"] = (h,), (h,)
    s["acoustic_decoder.head.linear.weight"] = (cfg.n_fft + 2, h)
    s["acoustic_decoder.head.linear.bias"] = (cfg.n_fft + 2,)
    return s


def synthetic_codec_weights(cfg: CodecConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Seeded fp32 decoder weights (CPU, deterministic) with realistic scales: unit-gain
    linears/convs (std 1/sqrt(fan_in)), norm gains near 1, a head whose magnitudes stay
    O(1) and whose phases span several radians."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, shp in codec_weight_shapes(cfg).items():
        if k.endswith("norm.weight") or "layernorm" in k or ".norm1.weight" in k or ".norm2.weight" in k:
            t = 1.0 + 0.05 * torch.randn(shp, generator=g)
        elif k.endswith(".bias"):
            t = 0.02 * torch.randn(shp, generator=g)
        else:
            fan_in = int(math.prod(shp[1:]))
            t = torch.randn(shp, generator=g) / math.sqrt(fan_in)
            if k == "acoustic_decoder.head.linear.weight":
                nb = cfg.n_fft // 2 + 1
                t[:nb] *= 0.5     # log-magnitudes ~ N(0, 0.5)
                t[nb:] *= 3.0     # phases ~ N(0, 3)
            elif "fc2" in k or "o_proj" in k or "conv2" in k:
                t *= 0.5          # keep the residual stream bounded over depth
        out[k] = t.to(F32).contiguous()
    return out


# ----------------------------------------------------------------------------- ABI
class XC2Config(C.Structure):
    _fields_ = [("hidden", C.c_int32), ("intermediate", C.c_int32), ("n_layers", C.c_int32),
                ("n_heads", C.c_int32), ("head_dim", C.c_int32), ("n_groups", C.c_int32),
                ("quant_dim", C.c_int32), ("n_levels", C.c_int32), ("level", C.c_int32), ("hop", C.c_int32),
                ("n_fft", C.c_int32), ("spec_ld", C.c_int32), ("attn_scale", C.c_float), ("rms_eps", C.c_float),
                ("gn_eps", C.c_float), ("ln_eps", C.c_float), ("max_batch", C.c_int32), ("max_frames", C.c_int32)]


class XC2ResBlock(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("gn1_w", "gn1_b", "conv1_w", "conv1_b", "gn2_w", "gn2_b", "conv2_w",
                                          "conv2_b")]


class XC2Layer(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("attn_norm", "qkv", "o", "mlp_norm", "fc1", "fc2")]


XC2_MAX_LAYERS = 32


class XC2Weights(C.Structure):
    _fields_ = [("project_out_w", C.c_void_p), ("project_out_b", C.c_void_p), ("fc_w", C.c_void_p),
                ("fc_b", C.c_void_p), ("embed_w", C.c_void_p), ("embed_b", C.c_void_p),
                ("prior", XC2ResBlock * 2), ("layers", XC2Layer * XC2_MAX_LAYERS), ("post", XC2ResBlock * 2),
                ("ln_w", C.c_void_p), ("ln_b", C.c_void_p), ("head_w", C.c_void_p), ("head_b", C.c_void_p),
                ("dft", C.c_void_p), ("window", C.c_void_p), ("rope_cos", C.c_void_p), ("rope_sin", C.c_void_p)]


XC2_SIGNATURES = {
    "xc2_create": (C.c_int, [C.POINTER(XC2Config), C.POINTER(XC2Weights), C.POINTER(C.c_void_p)]),
    "xc2_destroy": (C.c_int, [C.c_void_p]),
    "xc2_workspace_bytes": (C.c_int64, [C.c_void_p]),
    "xc2_decode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]),
    "xc2_gemm": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p,
                           C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]),
    "xc2_time_decode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                  C.c_void_p, C.POINTER(C.c_float)]),
    "xc2_time_gemms": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                                 C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
}


def irfft_basis(n_fft: int, spec_ld: int, window: torch.Tensor) -> torch.Tensor:
    """[n_fft][spec_ld] fp32 matrix B with frame = B @ (re_0, im_0, re_1, im_1, ...):
    window[n] * irfft(X, n_fft, norm="backward")[n] ([tf] :775-776). Built in fp64. Im of
    the DC and Nyquist bins is ignored, as irfft (c2r) does."""
    nb = n_fft // 2 + 1
    n = torch.arange(n_fft, dtype=torch.float64)[:, None]
    k = torch.arange(nb, dtype=torch.float64)[None, :]
    ang = 2.0 * math.pi * ((n * k) % n_fft) / n_fft
    c = torch.full((1, nb), 2.0, dtype=torch.float64)
    c[0, 0] = 1.0
    if n_fft % 2 == 0:
        c[0, -1] = 1.0
    re = c * torch.cos(ang) / n_fft
    im = -c * torch.sin(ang) / n_fft
    im[:, 0] = 0.0
    if n_fft % 2 == 0:
        im[:, -1] = 0.0
    w = window.to(torch.float64)[:, None]
    B = torch.zeros(n_fft, spec_ld, dtype=torch.float64)
    B[:, 0:2 * nb:2] = re * w
    B[:, 1:2 * nb:2] = im * w
    return B.to(F32)


class XCodec2Decoder:
    """Device-resident XCodec2 decoder (the pip package's ``decode_code``)."""

    def __init__(self, cfg: CodecConfig, state_dict: Dict[str, torch.Tensor], device="cuda:0",
                 max_batch: int = 8, max_frames: int = 1024):
        if cfg.head_dim != 64 or cfg.hidden_size != cfg.num_attention_heads * 64:
            raise ValueError("XCodec2 decoder kernels support head_dim 64 with hidden = heads * 64")
        if cfg.num_hidden_layers > XC2_MAX_LAYERS:
            raise ValueError(f"at most {XC2_MAX_LAYERS} transformer layers")
        self.cfg, self.device = cfg, torch.device(device)
        self.max_batch, self.max_frames = int(max_batch), int(max_frames)
        self.L = _lib.lib()
        for name, (res, args) in XC2_SIGNATURES.items():
            fn = getattr(self.L, name)
            fn.restype, fn.argtypes = res, args
        self._keep = []
        h = cfg.hidden_size
        dev = self.device

        def t(x: torch.Tensor) -> int:
            x = x.to(device=dev, dtype=F32).contiguous()
            self._keep.append(x)
            return x.data_ptr()

        def w(name):
            if name not in state_dict:
                raise KeyError(f"missing codec weight {name}")
            return state_dict[name].to(F32)

        def conv(name):   # [co][ci][k] -> tap-major [co][k*ci]
            x = w(name)
            return t(x.permute(0, 2, 1).reshape(x.shape[0], -1))

        W = XC2Weights()
        W.project_out_w, W.project_out_b = t(w("quantizer.project_out.weight")), t(w("quantizer.project_out.bias"))
        W.fc_w, W.fc_b = t(w("acoustic_decoder.fc.weight")), t(w("acoustic_decoder.fc.bias"))
        W.embed_w, W.embed_b = conv("acoustic_decoder.embed.weight"), t(w("acoustic_decoder.embed.bias"))
        for net, arr in (("prior_net", W.prior), ("post_net", W.post)):
            for i in range(2):
                p = f"acoustic_decoder.{net}.{i}."
                rb = arr[i]
                rb.gn1_w, rb.gn1_b = t(w(p + "norm1.weight")), t(w(p + "norm1.bias"))
                rb.conv1_w, rb.conv1_b = conv(p + "conv1.weight"), t(w(p + "conv1.bias"))
                rb.gn2_w, rb.gn2_b = t(w(p + "norm2.weight")), t(w(p + "norm2.bias"))
                rb.conv2_w, rb.conv2_b = conv(p + "conv2.weight"), t(w(p + "conv2.bias"))
        for i in range(cfg.num_hidden_layers):
            p = f"acoustic_decoder.layers.{i}."
            ly = W.layers[i]
            ly.attn_norm = t(w(p + "input_layernorm.weight"))
            ly.qkv = t(torch.cat([w(p + f"self_attn.{n}_proj.weight") for n in ("q", "k", "v")], 0))
            ly.o = t(w(p + "self_attn.o_proj.weight"))
            ly.mlp_norm = t(w(p + "post_attention_layernorm.weight"))
            ly.fc1, ly.fc2 = t(w(p + "mlp.fc1.weight")), t(w(p + "mlp.fc2.weight"))
        W.ln_w, W.ln_b = t(w("acoustic_decoder.norm.weight")), t(w("acoustic_decoder.norm.bias"))
        nb = cfg.n_fft // 2 + 1
        hw, hb = w("acoustic_decoder.head.linear.weight"), w("acoustic_decoder.head.linear.bias")
        iw = torch.empty_like(hw)
        ib = torch.empty_like(hb)
        iw[0::2], iw[1::2] = hw[:nb], hw[nb:]
        ib[0::2], ib[1::2] = hb[:nb], hb[nb:]
        W.head_w, W.head_b = t(iw), t(ib)
        window = torch.hann_window(cfg.n_fft, dtype=F32)
        W.window = t(window)
        W.dft = t(irfft_basis(cfg.n_fft, cfg.spec_ld, window))
        # RoPE over the head axis ([tf] Xcodec2RotaryEmbedding :119-154, position = head)
        inv_freq = 1.0 / (cfg.rope_theta ** (torch.arange(0, cfg.head_dim, 2, dtype=torch.int64).to(F32)
                                             / cfg.head_dim))
        pos = torch.arange(cfg.num_attention_heads, dtype=F32)
        freqs = (inv_freq[None, :, None] @ pos[None, None, :]).transpose(1, 2)[0]   # [H][hd/2]
        W.rope_cos, W.rope_sin = t(freqs.cos()), t(freqs.sin())
        self._w = W
        kc = XC2Config(hidden=h, intermediate=cfg.intermediate_size, n_layers=cfg.num_hidden_layers,
                       n_heads=cfg.num_attention_heads, head_dim=cfg.head_dim, n_groups=cfg.n_groups,
                       quant_dim=cfg.quantization_dim, n_levels=len(cfg.quantization_levels),
                       level=int(cfg.quantization_levels[0]), hop=cfg.hop_length, n_fft=cfg.n_fft,
                       spec_ld=cfg.spec_ld, attn_scale=cfg.head_dim ** -0.5, rms_eps=cfg.rms_norm_eps,
                       gn_eps=1e-6, ln_eps=1e-6, max_batch=self.max_batch, max_frames=self.max_frames)
        if len(set(cfg.quantization_levels)) != 1:
            raise ValueError("FSQ kernels assume equal levels per dimension")
        self._kc = kc
        h_ = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(self.L.xc2_create(C.byref(kc), C.byref(W), C.byref(h_)), "xc2_create")
        self.h = h_

    def close(self):
        if getattr(self, "h", None):
            self.L.xc2_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def decode(self, codes: torch.Tensor, lens: Optional[Sequence[int]] = None) -> torch.Tensor:
        """codes [B, T] or [B, 1, T] (int) -> wav fp32 [B, 1, T * hop] on the device."""
        if codes.dim() == 3:
            if codes.shape[1] != 1:
                raise ValueError(f"codes must be [B, 1, T], got {tuple(codes.shape)}")
            codes = codes[:, 0]
        if codes.dim() != 2:
            raise ValueError(f"codes must be [B, T] or [B, 1, T], got {tuple(codes.shape)}")
        B, T = codes.shape
        if B < 1 or T < 1:
            raise ValueError("empty codes")
        if B > self.max_batch or T > self.max_frames:
            raise ValueError(f"codes [{B}, {T}] exceed capacity [{self.max_batch}, {self.max_frames}]")
        dev = self.device
        # ids >= 2^31 never occur; negative ids are outside the reference's vocabulary
        if (codes < 0).any():
            raise ValueError("negative codec ids")
        c32 = codes.to(device=dev, dtype=torch.int32).contiguous()
        l32 = None
        if lens is not None:
            l32 = torch.tensor([int(v) for v in lens], dtype=torch.int32, device=dev)
            if l32.numel() != B or int(l32.min()) < 1 or int(l32.max()) > T:
                raise ValueError("lens must be B values in [1, T]")
        wav = torch.empty(B, T * self.cfg.hop_length, dtype=F32, device=dev)
        _lib.check(self.L.xc2_decode(self.h, C.c_void_p(c32.data_ptr()),
                                     C.c_void_p(l32.data_ptr() if l32 is not None else None), B, T,
                                     C.c_void_p(wav.data_ptr()), self._stream()), "xc2_decode")
        return wav.unsqueeze(1)


class AudioTokenizer:
    """Mirror of the reference's ``AudioTokenizer`` (data/tokenizer.py:53-123).
    ``decode(frames)`` accepts [B, T] or [B, 1, T] codes and returns the waveform
    [B, 1, T * hop] (fp32, on the codec's device), as ``decode_code`` does.
    ``encode(wav)`` (16 kHz, [B, 1, N] / [1, N] / [N]) returns codes [B, 1, N // 320 + 1]
    (int64, on the device) through the XCodec2 encoder (codec_enc.py) when encoder weights
    are given (``encoder_state_dict``, transformers ``Xcodec2Model`` names)."""

    def __init__(self, backend: str = "xcodec2", device=None, signature=None, model_name=None,
                 sample_rate: Optional[int] = None, cfg: Optional[CodecConfig] = None,
                 state_dict: Optional[Dict[str, torch.Tensor]] = None, encoder_cfg=None,
                 encoder_state_dict: Optional[Dict[str, torch.Tensor]] = None, max_encode_seconds: float = 30.0,
                 **kw):
        if backend != "xcodec2":
            raise ValueError(f"Only xcodec2 backend is supported now (got {backend}).")
        if device is None:
            device = torch.device("cuda")
        cfg = cfg or codec_16k()
        if state_dict is None:
            raise ValueError("state_dict required (no network: pass safetensors weights loaded locally)")
        self.codec = XCodec2Decoder(cfg, state_dict, device=device, **kw)
        self._device = torch.device(device)
        self.signature, self.model_name = signature, model_name
        self.sample_rate = int(sample_rate or cfg.sampling_rate)
        self.encode_sample_rate = 16000
        self.channels = 1
        self.encoder = None
        if encoder_state_dict is not None:
            from .codec_enc import XCodec2Encoder, encoder_16k
            self.encoder = XCodec2Encoder(encoder_cfg or encoder_16k(), encoder_state_dict, device=device,
                                          max_seconds=max_encode_seconds)

    @property
    def device(self):
        return self._device

    def encode(self, wav: torch.Tensor) -> torch.Tensor:
        """data/tokenizer.py:105-115: 16 kHz waveform -> codes [B, 1, T] (one utterance per
        encoder call, as the pip encode_code's semantic features are of row 0 only)."""
        if self.encoder is None:
            raise ValueError("AudioTokenizer has no encoder weights (pass encoder_state_dict)")
        if wav.ndim == 3:
            wav = wav.squeeze(1)
        if wav.ndim == 1:
            wav = wav.unsqueeze(0)
        return torch.cat([self.encoder.encode(wav[b]) for b in range(wav.shape[0])], dim=0)

    def decode(self, frames: torch.Tensor) -> torch.Tensor:
        codes = frames
        if codes.ndim == 2:
            codes = codes.unsqueeze(1)
        return self.codec.decode(codes.long())
