"""Configuration for the MI355X T5Gemma-TTS generate() engine.

Mirrors the inference-relevant fields of the reference's ``T5GemmaVoiceConfig``
(``hf_export/configuration_t5gemma_voice.py:50-151``) plus the T5Gemma backbone
shape constants that the reference takes from ``t5_config_dict`` /
transformers' ``T5GemmaModuleConfig`` defaults (2b-2b: d 2304, FFN 9216,
8 q heads / 4 kv heads x 256, 26+26 layers, sliding window 4096 on even layers).

Field names follow the reference so a ``config.json`` written by
``scripts/export_t5gemma_voice_hf.py`` maps 1:1 (``from_hf_dict``).
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from typing import Any, Dict, List, Optional


@dataclasses.dataclass
class BackboneDims:
    """T5Gemma encoder/decoder stack shape (one per side; 2b-2b uses equal sides)."""

    hidden_size: int = 2304
    intermediate_size: int = 9216
    num_encoder_layers: int = 26
    num_decoder_layers: int = 26
    num_attention_heads: int = 8
    num_key_value_heads: int = 4
    head_dim: int = 256
    text_vocab_size: int = 256000
    query_pre_attn_scalar: float = 256.0
    rope_theta: float = 10000.0
    rms_norm_eps: float = 1e-6
    sliding_window: int = 4096
    # per-layer "sliding_attention"/"full_attention"; None -> T5Gemma default
    # (sliding on even layer indices: [tf] configuration_t5gemma.py __post_init__)
    encoder_layer_types: Optional[List[str]] = None
    decoder_layer_types: Optional[List[str]] = None
    attn_logit_softcapping: Optional[float] = 50.0
    # "sdpa" drops the softcap (transformers sdpa integration ignores it);
    # "eager" applies tanh softcap. The released model trained with sdpa.
    attn_implementation: str = "sdpa"

    def layer_types(self, side: str) -> List[str]:
        n = self.num_encoder_layers if side == "encoder" else self.num_decoder_layers
        lt = self.encoder_layer_types if side == "encoder" else self.decoder_layer_types
        if lt is None:
            lt = ["sliding_attention" if (i + 1) % 2 else "full_attention" for i in range(n)]
        assert len(lt) == n
        return list(lt)

    @property
    def q_dim(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def softcap(self) -> float:
        """Effective attention-logit softcap: 0 means none (sdpa path)."""
        if self.attn_implementation == "eager" and self.attn_logit_softcapping:
            return float(self.attn_logit_softcapping)
        return 0.0

    @property
    def attn_scale(self) -> float:
        return float(self.query_pre_attn_scalar) ** -0.5


@dataclasses.dataclass
class VoiceConfig:
    """Inference-time voice-model fields (reference ``T5GemmaVoiceConfig``)."""

    backbone: BackboneDims = dataclasses.field(default_factory=BackboneDims)
    audio_vocab_size: int = 65536
    n_special: int = 5
    empty_token: int = 65536
    eog: int = 65537
    audio_pad_token: int = 65538
    eos: int = 65539
    y_sep_token: int = 65540
    x_sep_token: int = 255999
    special_first: int = 0
    encodec_sr: float = 50.0
    progress_scale: float = 2000.0
    progress_lookahead_secs: float = 2.0
    extra_cutoff: float = 5.0
    text_guard_frames_per_token: int = 0
    add_eos_to_text: int = 0
    add_bos_to_text: int = 0
    use_pm_rope: int = 1
    precision: str = "bfloat16"
    # carried for the host pipeline / provenance (configuration_t5gemma_voice.py:54-88)
    n_codebooks: int = 1
    parallel_pattern: int = 0
    audio_max_length: float = 40.0
    prune_text_modules: int = 0
    audio_mask_token: int = 1024
    audio_tokenizer: str = "xcodec2"
    codec_audio_sr: Optional[float] = None
    xcodec2_model_name: Optional[str] = None
    text_tokenizer_name: Optional[str] = None
    t5gemma_model_name: str = "google/t5gemma-2b-2b-ul2"

    @property
    def n_audio_tokens(self) -> int:
        return self.audio_vocab_size + self.n_special

    @property
    def eog_inference(self) -> int:
        # hf_export/modeling_t5gemma_voice.py:590-592
        return self.eos if self.eos > 0 else self.eog

    @property
    def eos_guard_steps(self) -> int:
        # `cur_num_gen <= self.args.encodec_sr // 5` (:727)
        return int(self.encodec_sr // 5)

    @property
    def extra_budget(self) -> float:
        # `int(self.args.encodec_sr) * extra_cutoff` (:776)
        return int(self.encodec_sr) * self.extra_cutoff

    # ------------------------------------------------------------------
    @staticmethod
    def from_hf_dict(d: Dict[str, Any]) -> "VoiceConfig":
        """Build from the ``config.json`` of the reference's HF export
        (``scripts/export_t5gemma_voice_hf.py:117-171``), the way
        ``T5GemmaVoiceForConditionalGeneration.__init__`` reads it (:343-478):

        * backbone shape from ``t5_config_dict`` (``T5GemmaConfig(**t5_config_dict)``, :361-364);
        * ``attn_implementation`` from the voice config, default ``"eager"`` (:365-367 and
          configuration_t5gemma_voice.py:59) -- eager applies the 50.0 logit softcap;
        * ``n_codebooks != 1`` is reset to 1 (:347-349) and a list ``audio_vocab_size``
          contributes its first entry (:451-459: only codebook 0 is built);
        * anything the engine does not implement raises ValueError instead of running a
          different model (activation other than tanh-GELU, attention bias, no PM-RoPE).
        """
        t5 = d.get("t5_config_dict") or {}
        enc = t5.get("encoder", t5) if isinstance(t5, dict) else {}
        dec = t5.get("decoder", enc) if isinstance(t5, dict) else {}
        for side in (enc, dec):
            act = side.get("hidden_activation", "gelu_pytorch_tanh")
            if act != "gelu_pytorch_tanh":
                raise ValueError(f"unsupported backbone activation {act!r} (engine implements gelu_pytorch_tanh)")
            if side.get("attention_bias", False):
                raise ValueError("unsupported backbone: attention_bias=True")
        rope = enc.get("rope_parameters") or {}
        if rope.get("rope_type", "default") != "default":
            raise ValueError(f"unsupported rope_type {rope.get('rope_type')!r}")
        bb = BackboneDims(
            hidden_size=enc.get("hidden_size", 2304),
            intermediate_size=enc.get("intermediate_size", 9216),
            num_encoder_layers=enc.get("num_hidden_layers", 26),
            num_decoder_layers=dec.get("num_hidden_layers", 26),
            num_attention_heads=enc.get("num_attention_heads", 8),
            num_key_value_heads=enc.get("num_key_value_heads", 4),
            head_dim=enc.get("head_dim", 256),
            text_vocab_size=enc.get("vocab_size", 256000),
            query_pre_attn_scalar=enc.get("query_pre_attn_scalar", 256),
            rope_theta=rope.get("rope_theta", enc.get("rope_theta", 10000.0)),
            rms_norm_eps=enc.get("rms_norm_eps", 1e-6),
            sliding_window=enc.get("sliding_window", 4096) or 1 << 30,
            encoder_layer_types=enc.get("layer_types"),
            decoder_layer_types=dec.get("layer_types"),
            attn_logit_softcapping=enc.get("attn_logit_softcapping", 50.0),
            attn_implementation=d.get("attn_implementation") or "eager",
        )
        for k in ("hidden_size", "intermediate_size", "num_attention_heads", "num_key_value_heads", "head_dim"):
            if k in dec and dec[k] != enc.get(k, dec[k]):
                raise ValueError(f"encoder/decoder {k} differ ({enc.get(k)} vs {dec[k]}): unsupported")
        kw = {}
        for f in dataclasses.fields(VoiceConfig):
            if f.name == "backbone":
                continue
            if f.name in d and d[f.name] is not None:
                kw[f.name] = d[f.name]
        avs = kw.get("audio_vocab_size")
        if isinstance(avs, (list, tuple)):
            kw["audio_vocab_size"] = int(avs[0])
        kw["n_codebooks"] = 1
        if int(kw.get("use_pm_rope", 1)) != 1:
            raise ValueError("use_pm_rope=0 (plain cross-attention) is not implemented by the engine")
        return VoiceConfig(backbone=bb, **kw)

    @staticmethod
    def from_pretrained(model_dir: str) -> "VoiceConfig":
        with open(os.path.join(model_dir, "config.json")) as f:
            return VoiceConfig.from_hf_dict(json.load(f))


# ----------------------------------------------------------------------
# Named configurations used by tests / bench
# ----------------------------------------------------------------------
def config_2b2b(attn_implementation: str = "sdpa", **voice_kw) -> VoiceConfig:
    """T5Gemma-TTS-2b-2b as released (examples/training/t5gemma_2b-2b.sh). ``voice_kw``
    overrides VoiceConfig fields (e.g. a short ``extra_cutoff`` for bounded golden runs)."""
    return VoiceConfig(backbone=BackboneDims(attn_implementation=attn_implementation), **voice_kw)


def config_mid(attn_implementation: str = "sdpa", layers: int = 2) -> VoiceConfig:
    """True 2b-2b widths at reduced depth and a reduced text vocab (parity tests)."""
    bb = BackboneDims(num_encoder_layers=layers, num_decoder_layers=layers,
                      text_vocab_size=4096, attn_implementation=attn_implementation)
    return VoiceConfig(backbone=bb, x_sep_token=4095, extra_cutoff=0.5)


def config_tiny(attn_implementation: str = "sdpa", sliding_window: int = 24) -> VoiceConfig:
    """Small golden-vector config: GQA 2:1, head_dim 64, 64+5 audio tokens."""
    bb = BackboneDims(hidden_size=128, intermediate_size=256, num_encoder_layers=2,
                      num_decoder_layers=2, num_attention_heads=2, num_key_value_heads=1,
                      head_dim=64, text_vocab_size=512, query_pre_attn_scalar=64,
                      sliding_window=sliding_window, attn_implementation=attn_implementation)
    V = 64
    return VoiceConfig(backbone=bb, audio_vocab_size=V, empty_token=V, eog=V + 1,
                       audio_pad_token=V + 2, eos=V + 3, y_sep_token=V + 4, x_sep_token=511,
                       extra_cutoff=1.0)


def named_config(name: str, **kw) -> VoiceConfig:
    return {"2b2b": config_2b2b, "mid": config_mid, "tiny": config_tiny}[name](**kw)


def param_count(cfg: VoiceConfig) -> int:
    bb = cfg.backbone
    d, f = bb.hidden_size, bb.intermediate_size
    attn = d * bb.q_dim * 2 + d * bb.kv_dim * 2
    mlp = 3 * d * f
    enc_layer = attn + mlp + 4 * d
    dec_layer = attn + (d * bb.q_dim * 2 + d * bb.kv_dim * 2) + mlp + 6 * d
    V = cfg.n_audio_tokens
    return (bb.text_vocab_size * d + bb.num_encoder_layers * enc_layer + d
            + bb.num_decoder_layers * dec_layer + d
            + V * d + d * d + d + d * V + V)


def decode_weight_bytes(cfg: VoiceConfig) -> int:
    """Bytes of bf16 weights one decode step must stream.

    Per decoder layer: self q/k/v/o + cross q/o + MLP (cross k/v are consumed
    once at prefill), plus the predict head.
    """
    bb = cfg.backbone
    d, f = bb.hidden_size, bb.intermediate_size
    per_layer = d * bb.q_dim * 2 + d * bb.kv_dim * 2 + d * bb.q_dim * 2 + 3 * d * f + 6 * d
    V = cfg.n_audio_tokens
    head = d * d + d + d * V + V
    return 2 * (bb.num_decoder_layers * per_layer + head + d)
