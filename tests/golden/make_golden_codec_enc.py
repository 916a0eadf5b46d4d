"""Golden vectors for the XCodec2 ENCODER (tests/test_gpu_codec_enc.py), from the
in-container transformers port -- the architecture oracle SURVEY 8(c)#4 names (the pip
``xcodec2`` package the reference calls is absent; parity against it is unpinned).

Run here: ``python tests/golden/make_golden_codec_enc.py``. For each config (tiny; and the
real 16 kHz dims) it builds ``transformers.Xcodec2Model`` with the repo's seeded encoder
weights (``t5gemma_tts_amd.codec_enc.synthetic_encoder_weights``), computes the semantic
input features the way the pip ``encode_code`` does -- ``SeamlessM4TFeatureExtractor`` on
the hop-padded waveform with 160 zeros either side (the port's own extractor needs
torchaudio, absent here) -- and records ``Xcodec2Model.encode``'s codes plus the
project_in latents, for a seeded speech-like waveform of a length that is not a
multiple of the hop.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from t5gemma_tts_amd.codec_enc import (HOP, EncoderConfig, encoder_16k, encoder_tiny,  # noqa: E402
                                       synthetic_encoder_weights)


def test_wave(n: int, seed: int) -> torch.Tensor:
    """Seeded speech-like signal: harmonic voiced segments with a wandering pitch and an
    amplitude envelope, plus low-level noise (amplitude <= ~0.5)."""
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64) / 16000.0
    f0 = 120.0 + 40.0 * torch.sin(2 * np.pi * 1.3 * t) + 10.0 * torch.randn(1, generator=g, dtype=torch.float64)
    phase = 2 * np.pi * torch.cumsum(f0, 0) / 16000.0
    x = sum((0.3 / k) * torch.sin(k * phase + float(torch.rand(1, generator=g))) for k in range(1, 8))
    env = 0.5 + 0.5 * torch.sin(2 * np.pi * 3.0 * t) ** 2
    x = x * env + 0.01 * torch.randn(n, generator=g, dtype=torch.float64)
    return x.to(torch.float32)


def hf_config(cfg: EncoderConfig):
    from transformers import Xcodec2Config
    sem = dict(hidden_size=cfg.sem_hidden, num_attention_heads=cfg.sem_heads, intermediate_size=cfg.sem_intermediate,
               num_hidden_layers=cfg.sem_layers, conv_depthwise_kernel_size=cfg.dw_kernel,
               left_max_position_embeddings=cfg.rel_left, right_max_position_embeddings=cfg.rel_right,
               layer_norm_eps=cfg.sem_ln_eps, feature_projection_input_dim=160)
    # decoder dims are irrelevant to encode(); keep them small
    return Xcodec2Config(hidden_size=cfg.hidden, intermediate_size=256, num_hidden_layers=1,
                         num_attention_heads=cfg.hidden // 64, encoder_hidden_size=cfg.ac_channels0,
                         downsampling_ratios=list(cfg.strides), quantization_levels=list(cfg.levels),
                         quantization_dim=cfg.fc_dim, semantic_model_config=sem)


def features(wav: torch.Tensor) -> torch.Tensor:
    """pip encode_code's semantic input: hop-padded waveform, +160 zeros either side,
    SeamlessM4TFeatureExtractor (Kaldi fbank, per-bin normalisation, 2-frame stacking)."""
    from transformers import SeamlessM4TFeatureExtractor
    n = wav.numel()
    n_pad = (n // HOP + 1) * HOP
    x = F.pad(wav, (0, n_pad - n))
    fe = SeamlessM4TFeatureExtractor()
    return fe(F.pad(x, (160, 160)).numpy(), sampling_rate=16000, return_tensors="pt")["input_features"]


def run(name: str, cfg: EncoderConfig, seed: int, n: int, wave_seed: int):
    from transformers import Xcodec2Model
    torch.manual_seed(0)
    model = Xcodec2Model(hf_config(cfg)).eval()
    sd = synthetic_encoder_weights(cfg, seed)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    enc_missing = [k for k in missing if not (k.startswith("acoustic_decoder.") or k.startswith("quantizer.project_out")
                                              or k == "semantic_encoder.masked_spec_embed")]
    assert not enc_missing, enc_missing[:10]
    wav = test_wave(n, wave_seed)
    n_pad = (n // HOP + 1) * HOP
    feat = features(wav)
    lat = {}
    h = model.quantizer.project_in.register_forward_hook(lambda m, i, o: lat.setdefault("p", o.detach().clone()))
    with torch.no_grad():
        out = model.encode(input_values=F.pad(wav, (0, n_pad - n))[None, None], input_features=feat)
    h.remove()
    codes = out.audio_codes.reshape(-1).to(torch.int32)
    p = lat["p"][0]
    # distance of each latent from its nearest FSQ rounding boundary (after the double bound)
    lv = torch.tensor(cfg.levels, dtype=torch.float32)
    half_range = (lv - 1) * (1 + 1e-3) / 2
    offset = torch.where(lv % 2 == 0, 0.5, 0.0)
    shift = torch.atanh(offset / half_range)
    b = (p + shift).tanh() * half_range - offset
    b = (b + shift).tanh() * half_range - offset
    margin = (b - torch.floor(b) - 0.5).abs().min().item()
    np.savez_compressed(os.path.join(HERE, f"golden_codec_enc_{name}.npz"), wav=wav.numpy(),
                        features=feat[0].numpy().astype(np.float32), codes=codes.numpy(),
                        latent=p.numpy().astype(np.float32))
    meta = {"source": "tests/golden/make_golden_codec_enc.py (transformers Xcodec2Model.encode + "
                      "SeamlessM4TFeatureExtractor)", "config": cfg.__dict__ | {"strides": list(cfg.strides),
                                                                                 "levels": list(cfg.levels)},
            "weight_seed": seed, "n_samples": n, "wave_seed": wave_seed, "n_codes": int(codes.numel()),
            "distinct_codes": int(codes.unique().numel()), "min_rounding_margin": margin,
            "torch_threads": torch.get_num_threads()}
    with open(os.path.join(HERE, f"golden_codec_enc_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(name, meta)


if __name__ == "__main__":
    torch.set_num_threads(8)
    run("tiny", encoder_tiny(), seed=31, n=13_337, wave_seed=5)
    run("full16k", encoder_16k(), seed=32, n=20_111, wave_seed=6)
