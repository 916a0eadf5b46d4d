"""Checkpoint boundary: an export-shaped directory -- the
``config.json`` and safetensors names the reference's ``scripts/export_t5gemma_voice_hf.py``
writes, captured from the reference in tests/golden/make_golden_export.py -- read by
``VoiceConfig.from_pretrained`` / ``weights.load_hf_checkpoint``:

* every tensor name and shape the engine reads is exactly the reference export's
  (``prune_text_modules = 2``), and the text-side extras of an unpruned export are ignored;
* ``config.json`` maps onto the engine config: backbone shape from ``t5_config_dict``,
  ``attn_implementation`` (default ``"eager"`` => softcap 50, configuration_t5gemma_voice.py:59),
  special token ids, ``add_eos_to_text`` / ``add_bos_to_text``, ``n_codebooks`` reset to 1
  (modeling_t5gemma_voice.py:347-349);
* the directory's tensors are the ones the reference model held (sha256 pinned);
* sharded safetensors with an index load like a single file."""
import json
import os
import tempfile

import pytest
import torch

from conftest import GOLDEN

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd.config import VoiceConfig, named_config
from t5gemma_tts_amd.weights import (check_state_dict, load_hf_checkpoint, state_dict_digest, synthetic_weights,
                                     weight_shapes)


def _fixture():
    with open(os.path.join(GOLDEN, "golden_export.json")) as f:
        return json.load(f)


def write_export(path, fx=None, config_overrides=None, unpruned=False, shards=2):
    """An export directory of the golden_tiny_eager model: config.json + safetensors shards
    (+ model.safetensors.index.json), tensors under the reference export's names."""
    from safetensors.torch import save_file
    fx = fx or _fixture()
    cfg = named_config(fx["config"], **fx["config_kw"])
    sd = synthetic_weights(cfg, fx["weight_seed"])
    tensors = {k: sd[k] for k in fx["state_dict"]}
    if unpruned:
        for k, shape in fx["state_dict_unpruned_extra"].items():
            tensors[k] = torch.zeros(shape, dtype=torch.bfloat16)
    conf = dict(fx["config_json"])
    conf.update(config_overrides or {})
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(conf, f, indent=2)
    names = sorted(tensors)
    weight_map = {}
    for i in range(shards):
        part = names[i::shards]
        fn = f"model-{i + 1:05d}-of-{shards:05d}.safetensors"
        save_file({k: tensors[k].contiguous() for k in part}, os.path.join(path, fn), metadata={"format": "pt"})
        weight_map.update({k: fn for k in part})
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {}, "weight_map": weight_map}, f)
    return cfg, sd


def test_export_tensor_names_are_the_engine_weight_table():
    fx = _fixture()
    cfg = named_config(fx["config"], **fx["config_kw"])
    ours = {n: list(s) for n, s in weight_shapes(cfg)}
    assert ours == fx["state_dict"]


def test_config_json_maps_onto_engine_config():
    fx = _fixture()
    want = named_config(fx["config"], **fx["config_kw"])
    got = VoiceConfig.from_hf_dict(fx["config_json"])
    assert got.backbone.attn_implementation == "eager" and got.backbone.softcap == 50.0
    for f in ("hidden_size", "intermediate_size", "num_encoder_layers", "num_decoder_layers", "num_attention_heads",
              "num_key_value_heads", "head_dim", "text_vocab_size", "query_pre_attn_scalar", "rope_theta",
              "rms_norm_eps", "sliding_window", "softcap", "attn_scale"):
        assert getattr(got.backbone, f) == getattr(want.backbone, f), f
    for side in ("encoder", "decoder"):
        assert got.backbone.layer_types(side) == want.backbone.layer_types(side)
    for f in ("audio_vocab_size", "n_special", "empty_token", "eog", "audio_pad_token", "eos", "y_sep_token",
              "x_sep_token", "encodec_sr", "progress_scale", "extra_cutoff", "text_guard_frames_per_token",
              "add_eos_to_text", "add_bos_to_text", "n_audio_tokens", "eog_inference", "eos_guard_steps"):
        assert getattr(got, f) == getattr(want, f), f


def test_config_json_field_variants():
    base = _fixture()["config_json"]

    def conf(**kw):
        d = json.loads(json.dumps(base))
        for k, v in kw.items():
            if v is None:
                d.pop(k, None)
            else:
                d[k] = v
        return VoiceConfig.from_hf_dict(d)

    # a config without the field falls back to the reference default "eager" (softcap on)
    assert conf(attn_implementation=None).backbone.softcap == 50.0
    assert conf(attn_implementation="sdpa").backbone.softcap == 0.0
    c = conf(add_eos_to_text=1, add_bos_to_text=2, text_guard_frames_per_token=7)
    assert (c.add_eos_to_text, c.add_bos_to_text, c.text_guard_frames_per_token) == (1, 2, 7)
    c = conf(n_codebooks=2, audio_vocab_size=[64, 32])
    assert c.n_codebooks == 1 and c.audio_vocab_size == 64 and c.n_audio_tokens == 69
    with pytest.raises(ValueError):
        conf(use_pm_rope=0)
    d = json.loads(json.dumps(base))
    d["t5_config_dict"]["encoder"]["hidden_activation"] = "gelu"
    with pytest.raises(ValueError):
        VoiceConfig.from_hf_dict(d)


def test_voice_defaults_match_reference_config_class():
    """VoiceConfig's defaults are T5GemmaVoiceConfig's (configuration_t5gemma_voice.py:54-88),
    except ``precision``: the engine always computes in bf16 (the reference's CLI loads with
    dtype=bf16, inference_commandline_hf.py:102-106) and the backbone's
    ``attn_implementation`` default lives on the from_hf_dict path (tested above)."""
    ref = _fixture()["voice_defaults"]
    ours = VoiceConfig()
    for k, v in ref.items():
        if k in ("precision", "attn_implementation", "t5_config_dict", "tie_word_embeddings",
                 "tie_input_output_embeddings"):
            continue
        assert hasattr(ours, k), k
        assert getattr(ours, k) == v, (k, getattr(ours, k), v)


def test_load_sharded_export_directory():
    fx = _fixture()
    with tempfile.TemporaryDirectory() as td:
        cfg, sd = write_export(td, fx, unpruned=True, shards=3)
        loaded = load_hf_checkpoint(td)
        check_state_dict(cfg, loaded)
        assert set(fx["state_dict_unpruned_extra"]) <= set(loaded)
        req = {k: loaded[k] for k in fx["state_dict"]}
        assert state_dict_digest(req) == fx["weight_digest"]
        c2 = VoiceConfig.from_pretrained(td)
        assert c2.backbone.softcap == cfg.backbone.softcap and c2.eos == cfg.eos


def test_missing_or_misshaped_tensor_is_rejected():
    fx = _fixture()
    cfg = named_config(fx["config"], **fx["config_kw"])
    sd = synthetic_weights(cfg, 1)
    bad = dict(sd)
    bad.pop("predict_layer.0.2.bias")
    with pytest.raises(ValueError):
        check_state_dict(cfg, bad)
    bad = dict(sd)
    bad["audio_embedding.0.weight"] = bad["audio_embedding.0.weight"][:-1]
    with pytest.raises(ValueError):
        check_state_dict(cfg, bad)
    with tempfile.TemporaryDirectory() as td:
        with pytest.raises(FileNotFoundError):
            load_hf_checkpoint(td)
