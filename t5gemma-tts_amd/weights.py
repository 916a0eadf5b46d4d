"""Weight tables for the engine: seeded synthetic weights and HF safetensors loading.

Key names are the reference's HF export layout (SURVEY 3.4;
``scripts/export_t5gemma_voice_hf.py:152-171``, ``hf_export/modeling_t5gemma_voice.py:497-506``):
``backbone.model.{encoder,decoder}.*``, ``audio_embedding.0.weight``,
``predict_layer.0.{0,2}.{weight,bias}`` with ``prune_text_modules=2`` (no decoder
``embed_tokens``, no ``lm_head``).

The seeded generator is deterministic on CPU (torch's CPU Philox/MT stream), so the
GPU box regenerates exactly the weights the golden fixtures were produced with.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Tuple

import torch

from .config import VoiceConfig

ENC = "backbone.model.encoder"
DEC = "backbone.model.decoder"


def weight_shapes(cfg: VoiceConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Ordered (name, shape) list of every tensor the generate() path reads."""
    bb = cfg.backbone
    d, f, q, kv = bb.hidden_size, bb.intermediate_size, bb.q_dim, bb.kv_dim
    V = cfg.n_audio_tokens
    out: List[Tuple[str, Tuple[int, ...]]] = [(f"{ENC}.embed_tokens.weight", (bb.text_vocab_size, d))]
    for side, n in ((ENC, bb.num_encoder_layers), (DEC, bb.num_decoder_layers)):
        for i in range(n):
            p = f"{side}.layers.{i}"
            out += [
                (f"{p}.self_attn.q_proj.weight", (q, d)),
                (f"{p}.self_attn.k_proj.weight", (kv, d)),
                (f"{p}.self_attn.v_proj.weight", (kv, d)),
                (f"{p}.self_attn.o_proj.weight", (d, q)),
            ]
            if side == DEC:
                out += [
                    (f"{p}.cross_attn.q_proj.weight", (q, d)),
                    (f"{p}.cross_attn.k_proj.weight", (kv, d)),
                    (f"{p}.cross_attn.v_proj.weight", (kv, d)),
                    (f"{p}.cross_attn.o_proj.weight", (d, q)),
                ]
            out += [
                (f"{p}.mlp.gate_proj.weight", (f, d)),
                (f"{p}.mlp.up_proj.weight", (f, d)),
                (f"{p}.mlp.down_proj.weight", (d, f)),
                (f"{p}.pre_self_attn_layernorm.weight", (d,)),
                (f"{p}.post_self_attn_layernorm.weight", (d,)),
            ]
            if side == DEC:
                out += [
                    (f"{p}.pre_cross_attn_layernorm.weight", (d,)),
                    (f"{p}.post_cross_attn_layernorm.weight", (d,)),
                ]
            out += [
                (f"{p}.pre_feedforward_layernorm.weight", (d,)),
                (f"{p}.post_feedforward_layernorm.weight", (d,)),
            ]
        out.append((f"{side}.norm.weight", (d,)))
    out += [
        ("audio_embedding.0.weight", (V, d)),
        ("predict_layer.0.0.weight", (d, d)),
        ("predict_layer.0.0.bias", (d,)),
        ("predict_layer.0.2.weight", (V, d)),
        ("predict_layer.0.2.bias", (V,)),
    ]
    return out


def _std_for(name: str) -> float:
    if name.endswith("layernorm.weight") or name.endswith("norm.weight"):
        return 0.05   # RMSNorm scales are (1 + w)
    return 0.02


def synthetic_weights(cfg: VoiceConfig, seed: int, device: str = "cpu",
                      dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    """Seeded N(0, std) weights at the exact tensor shapes of ``cfg``.

    On CPU the stream is reproducible bit-for-bit across machines (same torch);
    on a GPU device the values are random but not comparable to the CPU stream
    (used for throughput runs only).
    """
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    sd: Dict[str, torch.Tensor] = {}
    for name, shape in weight_shapes(cfg):
        t = torch.empty(shape, dtype=torch.float32, device=device)
        t.normal_(0.0, _std_for(name), generator=g)
        sd[name] = t.to(dtype)
    return sd


def state_dict_digest(sd: Dict[str, torch.Tensor]) -> str:
    """sha256 over names + raw bytes (order-independent of dict insertion)."""
    h = hashlib.sha256()
    for k in sorted(sd):
        t = sd[k].detach().contiguous().cpu()
        h.update(k.encode())
        h.update(t.view(torch.uint8).numpy().tobytes() if t.dtype != torch.bfloat16
                 else t.view(torch.int16).numpy().tobytes())
    return h.hexdigest()


def load_hf_checkpoint(model_dir: str) -> Dict[str, torch.Tensor]:
    """Read every ``*.safetensors`` shard of an HF export (no pickle)."""
    import glob
    import os

    from safetensors.torch import load_file

    files = sorted(glob.glob(os.path.join(model_dir, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no safetensors in {model_dir}")
    sd: Dict[str, torch.Tensor] = {}
    for fn in files:
        sd.update(load_file(fn))
    return sd


def check_state_dict(cfg: VoiceConfig, sd: Dict[str, torch.Tensor]) -> None:
    """Raise ValueError if a required tensor is missing or mis-shaped."""
    for name, shape in weight_shapes(cfg):
        if name not in sd:
            raise ValueError(f"missing weight {name}")
        if tuple(sd[name].shape) != tuple(shape):
            raise ValueError(f"{name}: shape {tuple(sd[name].shape)} != {shape}")
