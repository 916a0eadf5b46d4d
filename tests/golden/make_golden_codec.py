"""Generate the XCodec2 decoder golden vectors (run HERE, on CPU; never on the GPU box).

The architecture oracle is the in-container transformers ``Xcodec2Model`` (SURVEY
8(c)#4): it is built from a config, loaded with this repo's seeded synthetic decoder
weights (t5gemma_tts_amd.codec.synthetic_codec_weights), and ``decode(audio_codes)``
is run in fp32. Committed per case: the config, the weight seed, the codes and the
waveform (golden_codec_<case>.json + .npz). The weights themselves are regenerated
from the seed by the tests.

    python tests/golden/make_golden_codec.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd.codec import CodecConfig, codec_16k, codec_tiny, synthetic_codec_weights  # noqa: E402

CASES = {
    # name: (config, weight seed, B, T, code seed)
    "tiny": (codec_tiny(), 11, 2, 37, 101),
    "full16k": (codec_16k(), 12, 1, 40, 102),
    "hop882": (CodecConfig(hidden_size=256, intermediate_size=512, num_hidden_layers=1, num_attention_heads=4,
                           quantization_dim=512, downsampling_ratios=(2, 3, 3, 7, 7), sampling_rate=44100),
               13, 1, 23, 103),
}


def hf_model(cfg: CodecConfig):
    from transformers import Xcodec2Config, Xcodec2Model
    sem_h = cfg.quantization_dim - cfg.hidden_size
    hc = Xcodec2Config(hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                       num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                       num_key_value_heads=cfg.num_attention_heads, head_dim=cfg.head_dim,
                       quantization_dim=cfg.quantization_dim, downsampling_ratios=list(cfg.downsampling_ratios),
                       sampling_rate=cfg.sampling_rate,
                       semantic_model_config={"model_type": "wav2vec2-bert", "hidden_size": sem_h,
                                              "num_hidden_layers": 1, "num_attention_heads": 4,
                                              "intermediate_size": 2 * sem_h, "output_hidden_size": sem_h})
    return Xcodec2Model(hc).eval()


def cfg_dict(cfg: CodecConfig) -> dict:
    return {"hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
            "num_hidden_layers": cfg.num_hidden_layers, "num_attention_heads": cfg.num_attention_heads,
            "head_dim": cfg.head_dim, "quantization_dim": cfg.quantization_dim,
            "quantization_levels": list(cfg.quantization_levels),
            "downsampling_ratios": list(cfg.downsampling_ratios), "sampling_rate": cfg.sampling_rate,
            "rms_norm_eps": cfg.rms_norm_eps}


def main():
    torch.set_num_threads(8)
    for name, (cfg, wseed, B, T, cseed) in CASES.items():
        model = hf_model(cfg)
        sd = synthetic_codec_weights(cfg, wseed)
        missing = [k for k in sd if k not in model.state_dict()]
        assert not missing, missing
        res = model.load_state_dict(sd, strict=False)
        assert not [k for k in res.unexpected_keys], res.unexpected_keys
        g = torch.Generator().manual_seed(cseed)
        codes = torch.randint(0, cfg.codebook_size, (B, T), generator=g)
        with torch.no_grad():
            wav = model.decode(audio_codes=codes[:, None, :]).audio_values
        wav = wav.float().numpy()
        assert wav.shape == (B, 1, T * cfg.hop_length), wav.shape
        meta = {"case": name, "config": cfg_dict(cfg), "weight_seed": wseed, "B": B, "T": T,
                "codes": codes.tolist(), "threads": torch.get_num_threads(),
                "wav_rms": float(np.sqrt((wav.astype(np.float64) ** 2).mean())),
                "generator": "transformers Xcodec2Model.decode (fp32 CPU), transformers "
                             + __import__("transformers").__version__}
        with open(os.path.join(HERE, f"golden_codec_{name}.json"), "w") as f:
            json.dump(meta, f)
        np.savez_compressed(os.path.join(HERE, f"golden_codec_{name}.npz"), wav=wav)
        print(name, wav.shape, "rms", meta["wav_rms"], "max", float(np.abs(wav).max()))


if __name__ == "__main__":
    main()
