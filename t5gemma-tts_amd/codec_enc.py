"""XCodec2 codec encoder on MI355X: the ``AudioTokenizer.encode`` half of the codec
(voice-clone prompts from audio).

Reference boundary: ``AudioTokenizer.encode(wav)`` (data/tokenizer.py:105-115), called by
``tokenize_audio`` (:125-143) from inference_tts_utils.py:182-188 on the reference clip
resampled to 16 kHz. The reference delegates to the pip ``xcodec2`` package's
``encode_code`` (absent from the reference tree); the architecture is restated from the
in-container transformers port ([tf] models/xcodec2/modeling_xcodec2.py:974-1024,
[tf] models/wav2vec2_bert/modeling_wav2vec2_bert.py) whose state-dict names this module
reads, with the SeamlessM4T Kaldi fbank the pip package feeds its semantic model.

All compute runs in libt5gtts.so (``xc2e_*`` C ABI, include/xc2.h); this module builds
the constant tables (DFT basis, Kaldi mel filters, povey window, Kaiser-sinc filters),
lays the fp32 weights out for the kernels (tap-major padded convolutions, fused q/k/v)
and calls the ABI. There is no CPU fallback: a missing library raises.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

import torch

from . import _lib

F32 = torch.float32
HOP = 320


@dataclass
class EncoderConfig:
    """Encoder hyper-parameters ([tf] configuration_xcodec2.py + Wav2Vec2BertConfig with
    num_hidden_layers = 16, the layer the pip package reads)."""
    sem_hidden: int = 1024
    sem_heads: int = 16
    sem_intermediate: int = 4096
    sem_layers: int = 16
    dw_kernel: int = 31
    rel_left: int = 64
    rel_right: int = 8
    sem_ln_eps: float = 1e-5
    ac_channels0: int = 48
    strides: Sequence[int] = (2, 2, 4, 4, 5)
    hidden: int = 1024
    levels: Sequence[int] = (4,) * 8

    @property
    def fc_dim(self) -> int:
        return self.sem_hidden + self.hidden

    @classmethod
    def from_hf_dict(cls, d: dict) -> "EncoderConfig":
        """From a transformers ``Xcodec2Config`` dict (config.json of an Xcodec2Model dir)."""
        s = d.get("semantic_model_config") or {}
        if s.get("position_embeddings_type", "relative_key") != "relative_key":
            raise ValueError("semantic encoder: only relative_key position embeddings are implemented")
        if s.get("hidden_act", "swish") not in ("swish", "silu"):
            raise ValueError("semantic encoder: only swish activations are implemented")
        if s.get("feature_projection_input_dim", 160) != 160:
            raise ValueError("semantic encoder: 160-dim stacked fbank input expected")
        return cls(sem_hidden=s.get("hidden_size", 1024), sem_heads=s.get("num_attention_heads", 16),
                   sem_intermediate=s.get("intermediate_size", 4096), sem_layers=s.get("num_hidden_layers", 16),
                   dw_kernel=s.get("conv_depthwise_kernel_size", 31),
                   rel_left=s.get("left_max_position_embeddings", 64),
                   rel_right=s.get("right_max_position_embeddings", 8), sem_ln_eps=s.get("layer_norm_eps", 1e-5),
                   ac_channels0=d.get("encoder_hidden_size", 48),
                   strides=tuple(d.get("downsampling_ratios", (2, 2, 4, 4, 5))), hidden=d.get("hidden_size", 1024),
                   levels=tuple(d.get("quantization_levels", (4,) * 8)))


def encoder_16k() -> EncoderConfig:
    """HKUSTAudio/xcodec2 (and the Anime-XCodec2 encoder, which also runs at 16 kHz)."""
    return EncoderConfig()


def encoder_tiny() -> EncoderConfig:
    """Reduced-width test config (same structure)."""
    return EncoderConfig(sem_hidden=128, sem_heads=2, sem_intermediate=256, sem_layers=2, ac_channels0=4, hidden=128)


def num_codes(n_samples: int) -> int:
    """Codes for n samples at 16 kHz: the input is padded with 1 sample, then to a
    multiple of the 320-sample hop ([tf] feature_extraction_xcodec2.py:149-159)."""
    return int(n_samples) // HOP + 1


# ---------------------------------------------------------------------- weights
def encoder_weight_shapes(cfg: EncoderConfig) -> Dict[str, tuple]:
    """Encoder tensors under the transformers ``Xcodec2Model`` state-dict names."""
    H, I, K = cfg.sem_hidden, cfg.sem_intermediate, cfg.dw_kernel
    s = {"semantic_encoder.feature_projection.layer_norm.weight": (160,),
         "semantic_encoder.feature_projection.layer_norm.bias": (160,),
         "semantic_encoder.feature_projection.projection.weight": (H, 160),
         "semantic_encoder.feature_projection.projection.bias": (H,)}
    for i in range(cfg.sem_layers):
        p = f"semantic_encoder.encoder.layers.{i}."
        for ln in ("ffn1_layer_norm", "self_attn_layer_norm", "conv_module.layer_norm",
                   "conv_module.depthwise_layer_norm", "ffn2_layer_norm", "final_layer_norm"):
            s[p + ln + ".weight"], s[p + ln + ".bias"] = (H,), (H,)
        for f in ("ffn1", "ffn2"):
            s[p + f + ".intermediate_dense.weight"], s[p + f + ".intermediate_dense.bias"] = (I, H), (I,)
            s[p + f + ".output_dense.weight"], s[p + f + ".output_dense.bias"] = (H, I), (H,)
        for n in ("linear_q", "linear_k", "linear_v", "linear_out"):
            s[p + f"self_attn.{n}.weight"], s[p + f"self_attn.{n}.bias"] = (H, H), (H,)
        s[p + "self_attn.distance_embedding.weight"] = (cfg.rel_left + cfg.rel_right + 1, 64)
        s[p + "conv_module.pointwise_conv1.weight"] = (2 * H, H, 1)
        s[p + "conv_module.depthwise_conv.weight"] = (H, 1, K)
        s[p + "conv_module.pointwise_conv2.weight"] = (H, H, 1)
    for j in range(1, 5):
        s[f"semantic_adapter.conv{j}.weight"] = (H, H, 3)
        if j in (2, 3):
            s[f"semantic_adapter.conv{j}.bias"] = (H,)
    c = cfg.ac_channels0
    s["acoustic_encoder.conv1.weight"], s["acoustic_encoder.conv1.bias"] = (c, 1, 7), (c,)
    for b, st in enumerate(cfg.strides):
        p = f"acoustic_encoder.block.{b}."
        for r in range(1, 4):
            q = p + f"res_unit{r}."
            for sn in ("snake1", "snake2"):
                s[q + sn + ".act.alpha"], s[q + sn + ".act.beta"] = (c,), (c,)
            s[q + "conv1.weight"], s[q + "conv1.bias"] = (c, c, 7), (c,)
            s[q + "conv2.weight"], s[q + "conv2.bias"] = (c, c, 1), (c,)
        s[p + "snake1.act.alpha"], s[p + "snake1.act.beta"] = (c,), (c,)
        s[p + "conv1.weight"], s[p + "conv1.bias"] = (2 * c, c, 2 * st), (2 * c,)
        c *= 2
    s["acoustic_encoder.snake1.act.alpha"], s["acoustic_encoder.snake1.act.beta"] = (c,), (c,)
    s["acoustic_encoder.conv2.weight"], s["acoustic_encoder.conv2.bias"] = (cfg.hidden, c, 3), (cfg.hidden,)
    W2 = cfg.fc_dim
    s["fc_encoder.weight"], s["fc_encoder.bias"] = (W2, W2), (W2,)
    s["quantizer.project_in.weight"], s["quantizer.project_in.bias"] = (len(cfg.levels), W2), (len(cfg.levels),)
    return s


def synthetic_encoder_weights(cfg: EncoderConfig, seed: int = 0) -> Dict[str, torch.Tensor]:
    """Seeded fp32 encoder weights (CPU, deterministic) at realistic scales: unit-gain
    linears / convs, norm gains near 1, residual branches halved, SnakeBeta
    log-parameters near 0, project_in giving unit-variance latents (so the FSQ digits
    spread over all levels)."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, shp in encoder_weight_shapes(cfg).items():
        if k.endswith(".act.alpha") or k.endswith(".act.beta"):
            t = 0.2 * torch.randn(shp, generator=g)
        elif "norm" in k and k.endswith(".weight"):
            t = 1.0 + 0.05 * torch.randn(shp, generator=g)
        elif k.endswith(".bias"):
            t = 0.02 * torch.randn(shp, generator=g)
        elif k.endswith("distance_embedding.weight"):
            t = 0.5 * torch.randn(shp, generator=g)
        else:
            fan_in = int(math.prod(shp[1:]))
            t = torch.randn(shp, generator=g) / math.sqrt(fan_in)
            if any(n in k for n in ("output_dense", "linear_out", "pointwise_conv2", ".conv2.weight")):
                t *= 0.5
        out[k] = t.to(F32).contiguous()
    return out


# ------------------------------------------------------------------ constant tables
def fbank_dft_basis() -> torch.Tensor:
    """[544][512]: row 2k = cos(2 pi k n / 512), row 2k + 1 = -sin(...) for the 257 bins
    of the 512-point real FFT (np.fft.rfft), rows >= 514 zero. Built in fp64."""
    n = torch.arange(512, dtype=torch.float64)[None, :]
    k = torch.arange(257, dtype=torch.float64)[:, None]
    ang = 2.0 * math.pi * ((k * n) % 512) / 512
    B = torch.zeros(544, 512, dtype=torch.float64)
    B[0:514:2] = torch.cos(ang)
    B[1:514:2] = -torch.sin(ang)
    return B.to(F32)


def kaldi_mel_filters() -> torch.Tensor:
    """[80][288]: transformers mel_filter_bank(257, 80, 20, 8000, 16000, norm=None,
    mel_scale="kaldi", triangularize_in_mel_space=True) (audio_utils.py:638-730),
    transposed and zero-padded; fp64 then fp32."""
    def mel(f):
        return 1127.0 * torch.log(1.0 + f / 700.0)
    mel_freqs = torch.linspace(float(mel(torch.tensor(20.0, dtype=torch.float64))),
                               float(mel(torch.tensor(8000.0, dtype=torch.float64))), 82, dtype=torch.float64)
    fft_freqs = mel((16000 / 512) * torch.arange(257, dtype=torch.float64))
    diff = mel_freqs[1:] - mel_freqs[:-1]
    slopes = mel_freqs[None, :] - fft_freqs[:, None]
    down = -slopes[:, :-2] / diff[:-1]
    up = slopes[:, 2:] / diff[1:]
    fb = torch.clamp(torch.minimum(down, up), min=0.0)            # [257][80]
    out = torch.zeros(80, 288, dtype=torch.float64)
    out[:, :257] = fb.T
    return out.to(F32)


def povey_window() -> torch.Tensor:
    """window_function(400, "povey", periodic=False): np.hanning(400) ** 0.85."""
    n = torch.arange(400, dtype=torch.float64)
    return ((0.5 - 0.5 * torch.cos(2.0 * math.pi * n / 399)) ** 0.85).to(F32)


def kaiser_sinc_filter(cutoff: float = 0.25, half_width: float = 0.3, kernel_size: int = 12) -> torch.Tensor:
    """[tf] kaiser_sinc_filter1d (modeling_xcodec2.py:417-460) for the even 12-tap case."""
    half = kernel_size // 2
    delta_f = 4 * half_width
    att = 2.285 * (half - 1) * math.pi * delta_f + 7.95
    beta = 0.1102 * (att - 8.7) if att > 50.0 else (0.5842 * (att - 21) ** 0.4 + 0.07886 * (att - 21.0)
                                                    if att >= 21.0 else 0.0)
    win = torch.kaiser_window(kernel_size, beta=beta, periodic=False, dtype=torch.float32)
    t = torch.arange(-half, half) + 0.5
    f = 2 * cutoff * win * torch.sinc(2 * cutoff * t)
    return (f / f.sum()).to(F32)


# ----------------------------------------------------------------------------- ABI
XC2E_MAX_LAYERS = 32
XC2E_MAX_BLOCKS = 8


class XC2EConfig(C.Structure):
    _fields_ = [("sem_hidden", C.c_int32), ("sem_heads", C.c_int32), ("sem_intermediate", C.c_int32),
                ("sem_layers", C.c_int32), ("feat_dim", C.c_int32), ("dw_kernel", C.c_int32),
                ("rel_left", C.c_int32), ("rel_right", C.c_int32), ("sem_ln_eps", C.c_float),
                ("ac_channels0", C.c_int32), ("n_blocks", C.c_int32), ("strides", C.c_int32 * XC2E_MAX_BLOCKS),
                ("hidden", C.c_int32), ("n_levels", C.c_int32), ("level", C.c_int32), ("max_samples", C.c_int32)]


class XC2EConv(C.Structure):
    _fields_ = [("w", C.c_void_p), ("b", C.c_void_p), ("cin", C.c_int32), ("cout", C.c_int32), ("k", C.c_int32),
                ("stride", C.c_int32), ("dil", C.c_int32), ("pad", C.c_int32), ("kpad", C.c_int32)]


class XC2ESnake(C.Structure):
    _fields_ = [("alpha", C.c_void_p), ("beta", C.c_void_p)]


class XC2EResUnit(C.Structure):
    _fields_ = [("s1", XC2ESnake), ("c1", XC2EConv), ("s2", XC2ESnake), ("c2", XC2EConv)]


class XC2EBlock(C.Structure):
    _fields_ = [("ru", XC2EResUnit * 3), ("s", XC2ESnake), ("down", XC2EConv)]


_LAYER_FIELDS = ("ffn1_ln_w", "ffn1_ln_b", "ffn1_w1", "ffn1_b1", "ffn1_w2", "ffn1_b2", "attn_ln_w", "attn_ln_b",
                 "qkv_w", "qkv_b", "o_w", "o_b", "dist_emb", "conv_ln_w", "conv_ln_b", "pw1_w", "dw_w", "dw_ln_w",
                 "dw_ln_b", "pw2_w", "ffn2_ln_w", "ffn2_ln_b", "ffn2_w1", "ffn2_b1", "ffn2_w2", "ffn2_b2",
                 "final_ln_w", "final_ln_b")


class XC2ELayer(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in _LAYER_FIELDS]


class XC2EWeights(C.Structure):
    _fields_ = [("dft", C.c_void_p), ("mel", C.c_void_p), ("window", C.c_void_p), ("fp_ln_w", C.c_void_p),
                ("fp_ln_b", C.c_void_p), ("fp_w", C.c_void_p), ("fp_b", C.c_void_p),
                ("layers", XC2ELayer * XC2E_MAX_LAYERS), ("adapter", XC2EConv * 4), ("ac_in", XC2EConv),
                ("blocks", XC2EBlock * XC2E_MAX_BLOCKS), ("ac_snake", XC2ESnake), ("ac_out", XC2EConv),
                ("fc_w", C.c_void_p), ("fc_b", C.c_void_p), ("pin_w", C.c_void_p), ("pin_b", C.c_void_p),
                ("aa_up", C.c_void_p), ("aa_down", C.c_void_p)]


XC2E_SIGNATURES = {
    "xc2e_create": (C.c_int, [C.POINTER(XC2EConfig), C.POINTER(XC2EWeights), C.POINTER(C.c_void_p)]),
    "xc2e_destroy": (C.c_int, [C.c_void_p]),
    "xc2e_workspace_bytes": (C.c_int64, [C.c_void_p]),
    "xc2e_num_codes": (C.c_int32, [C.c_void_p, C.c_int32]),
    "xc2e_encode": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "xc2e_features": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
}


class XCodec2Encoder:
    """Device-resident XCodec2 encoder (the pip package's ``encode_code``)."""

    def __init__(self, cfg: EncoderConfig, state_dict: Dict[str, torch.Tensor], device="cuda:0",
                 max_seconds: float = 30.0):
        if cfg.sem_hidden != cfg.sem_heads * 64:
            raise ValueError("semantic attention kernels support head size 64")
        if cfg.sem_layers > XC2E_MAX_LAYERS or len(cfg.strides) > XC2E_MAX_BLOCKS:
            raise ValueError("encoder depth exceeds the ABI tables")
        if len(set(cfg.levels)) != 1:
            raise ValueError("FSQ kernels assume equal levels per dimension")
        if math.prod(cfg.strides) != HOP:
            raise ValueError(f"acoustic strides must multiply to {HOP}")
        self.cfg, self.device = cfg, torch.device(device)
        self.max_samples = int(max_seconds * 16000)
        self.L = _lib.lib()
        for name, (res, args) in XC2E_SIGNATURES.items():
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
                raise KeyError(f"missing codec encoder weight {name}")
            return state_dict[name].to(F32)

        def conv(wname, bname, stride=1, dil=1, pad=0) -> XC2EConv:
            x = w(wname)                                    # [co][ci][k]
            co, ci, k = x.shape
            kpad = (k * ci + 31) // 32 * 32
            tm = torch.zeros(co, kpad, dtype=F32)
            tm[:, :k * ci] = x.permute(0, 2, 1).reshape(co, k * ci)
            return XC2EConv(w=t(tm), b=t(w(bname)) if bname else None, cin=ci, cout=co, k=k, stride=stride, dil=dil,
                            pad=pad, kpad=kpad)

        def snake(p) -> XC2ESnake:
            return XC2ESnake(alpha=t(w(p + ".act.alpha")), beta=t(w(p + ".act.beta")))

        W = XC2EWeights()
        W.dft, W.mel, W.window = t(fbank_dft_basis()), t(kaldi_mel_filters()), t(povey_window())
        fp = "semantic_encoder.feature_projection."
        W.fp_ln_w, W.fp_ln_b = t(w(fp + "layer_norm.weight")), t(w(fp + "layer_norm.bias"))
        W.fp_w, W.fp_b = t(w(fp + "projection.weight")), t(w(fp + "projection.bias"))
        for i in range(cfg.sem_layers):
            p = f"semantic_encoder.encoder.layers.{i}."
            ly = W.layers[i]
            for f in ("ffn1", "ffn2"):
                setattr(ly, f + "_ln_w", t(w(p + f + "_layer_norm.weight")))
                setattr(ly, f + "_ln_b", t(w(p + f + "_layer_norm.bias")))
                setattr(ly, f + "_w1", t(w(p + f + ".intermediate_dense.weight")))
                setattr(ly, f + "_b1", t(w(p + f + ".intermediate_dense.bias")))
                setattr(ly, f + "_w2", t(w(p + f + ".output_dense.weight")))
                setattr(ly, f + "_b2", t(w(p + f + ".output_dense.bias")))
            a = p + "self_attn."
            ly.attn_ln_w, ly.attn_ln_b = t(w(p + "self_attn_layer_norm.weight")), t(w(p + "self_attn_layer_norm.bias"))
            ly.qkv_w = t(torch.cat([w(a + f"linear_{n}.weight") for n in "qkv"], 0))
            ly.qkv_b = t(torch.cat([w(a + f"linear_{n}.bias") for n in "qkv"], 0))
            ly.o_w, ly.o_b = t(w(a + "linear_out.weight")), t(w(a + "linear_out.bias"))
            ly.dist_emb = t(w(a + "distance_embedding.weight"))
            cm = p + "conv_module."
            ly.conv_ln_w, ly.conv_ln_b = t(w(cm + "layer_norm.weight")), t(w(cm + "layer_norm.bias"))
            ly.pw1_w = t(w(cm + "pointwise_conv1.weight")[:, :, 0])
            ly.dw_w = t(w(cm + "depthwise_conv.weight")[:, 0, :])
            ly.dw_ln_w, ly.dw_ln_b = t(w(cm + "depthwise_layer_norm.weight")), t(w(cm + "depthwise_layer_norm.bias"))
            ly.pw2_w = t(w(cm + "pointwise_conv2.weight")[:, :, 0])
            ly.final_ln_w, ly.final_ln_b = t(w(p + "final_layer_norm.weight")), t(w(p + "final_layer_norm.bias"))
        for j in range(4):
            W.adapter[j] = conv(f"semantic_adapter.conv{j + 1}.weight",
                                f"semantic_adapter.conv{j + 1}.bias" if j in (1, 2) else None, pad=1)
        W.ac_in = conv("acoustic_encoder.conv1.weight", "acoustic_encoder.conv1.bias", pad=3)
        for b, st in enumerate(cfg.strides):
            p = f"acoustic_encoder.block.{b}."
            blk = W.blocks[b]
            for r, dil in enumerate((1, 3, 9)):
                q = p + f"res_unit{r + 1}."
                ru = blk.ru[r]
                ru.s1, ru.s2 = snake(q + "snake1"), snake(q + "snake2")
                ru.c1 = conv(q + "conv1.weight", q + "conv1.bias", dil=dil, pad=3 * dil)
                ru.c2 = conv(q + "conv2.weight", q + "conv2.bias")
            blk.s = snake(p + "snake1")
            blk.down = conv(p + "conv1.weight", p + "conv1.bias", stride=st, pad=(st + 1) // 2)
        W.ac_snake = snake("acoustic_encoder.snake1")
        W.ac_out = conv("acoustic_encoder.conv2.weight", "acoustic_encoder.conv2.bias", pad=1)
        W.fc_w, W.fc_b = t(w("fc_encoder.weight")), t(w("fc_encoder.bias"))
        W.pin_w, W.pin_b = t(w("quantizer.project_in.weight")), t(w("quantizer.project_in.bias"))
        filt = kaiser_sinc_filter()
        W.aa_up, W.aa_down = t(filt), t(filt)
        self._w = W
        strides = (C.c_int32 * XC2E_MAX_BLOCKS)(*list(cfg.strides))
        kc = XC2EConfig(sem_hidden=cfg.sem_hidden, sem_heads=cfg.sem_heads, sem_intermediate=cfg.sem_intermediate,
                        sem_layers=cfg.sem_layers, feat_dim=160, dw_kernel=cfg.dw_kernel, rel_left=cfg.rel_left,
                        rel_right=cfg.rel_right, sem_ln_eps=cfg.sem_ln_eps, ac_channels0=cfg.ac_channels0,
                        n_blocks=len(cfg.strides), strides=strides, hidden=cfg.hidden, n_levels=len(cfg.levels),
                        level=int(cfg.levels[0]), max_samples=self.max_samples)
        self._kc = kc
        h = C.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(self.L.xc2e_create(C.byref(kc), C.byref(W), C.byref(h)), "xc2e_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.xc2e_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def workspace_bytes(self) -> int:
        return int(self.L.xc2e_workspace_bytes(self.h))

    def encode(self, wav: torch.Tensor, return_latent: bool = False):
        """wav: 16 kHz mono, [N] / [1, N] / [1, 1, N] float -> codes int64 [1, 1, N // 320 + 1]
        on the device (+ the project_in latents [T][n_levels] before the FSQ bound)."""
        x = wav.reshape(-1) if wav.dim() == 1 or (wav.dim() >= 2 and math.prod(wav.shape[:-1]) == 1) else None
        if x is None:
            raise ValueError(f"one mono utterance expected, got {tuple(wav.shape)}")
        n = int(x.numel())
        if n > self.max_samples:
            raise ValueError(f"{n} samples exceed the encoder capacity ({self.max_samples})")
        xd = x.to(device=self.device, dtype=F32).contiguous()
        T = num_codes(n)
        codes = torch.empty(T, dtype=torch.int32, device=self.device)
        lat = torch.empty(T, len(self.cfg.levels), dtype=F32, device=self.device) if return_latent else None
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.L.xc2e_encode(self.h, C.c_void_p(xd.data_ptr()), n, C.c_void_p(codes.data_ptr()),
                                      C.c_void_p(lat.data_ptr() if lat is not None else None), st), "xc2e_encode")
        out = codes.long().view(1, 1, T)
        return (out, lat) if return_latent else out

    def features(self, wav: torch.Tensor) -> torch.Tensor:
        """Diagnostics: the semantic model's input features [T][160] (fbank front end)."""
        x = wav.reshape(-1).to(device=self.device, dtype=F32).contiguous()
        n = int(x.numel())
        if n > self.max_samples:
            raise ValueError(f"{n} samples exceed the encoder capacity ({self.max_samples})")
        out = torch.empty(num_codes(n), 160, dtype=F32, device=self.device)
        st = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _lib.check(self.L.xc2e_features(self.h, C.c_void_p(x.data_ptr()), n, C.c_void_p(out.data_ptr()), st),
                   "xc2e_features")
        return out
