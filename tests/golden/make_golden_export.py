"""Fixture for the checkpoint boundary: what the reference's HF
export writes, captured from the reference's own code in this container.

Run here only (``python tests/golden/make_golden_export.py``): it reads
``/root/reference`` (absent on the GPU box). Output: ``tests/golden/golden_export.json``:

* ``voice_defaults`` -- the ``T5GemmaVoiceConfig.__init__`` keyword defaults
  (``hf_export/configuration_t5gemma_voice.py:54-88``), read off the source with ``ast``
  (the module itself cannot be imported: SyntaxError);
* ``config_json`` -- the ``config.json`` an export of the golden_tiny_eager model writes:
  ``export_t5gemma_voice_hf.py:117-150`` builds the config from the checkpoint args and
  ``t5_config_dict = T5GemmaConfig.to_dict()``; serialised here the way
  ``PretrainedConfig.save_pretrained`` does it (transformers 5.15), with the reference's
  attribute set;
* ``state_dict`` -- name -> shape of every tensor the export's safetensors hold: the
  reference model's ``state_dict()`` (``models/t5gemma.py`` T5GemmaVoiceModel, identical
  module tree to the HF class) minus the ``encoder_module.`` / ``decoder_module.`` aliases
  the HF class drops on save (``hf_export/modeling_t5gemma_voice.py:497-506``), with
  ``prune_text_modules = 2`` (no ``backbone.lm_head``, no decoder ``embed_tokens``:
  ``export_t5gemma_voice_hf.py:156-163``) and, as a second listing, ``prune_text_modules
  = 0`` (extra text-side tensors the loader must ignore);
* ``weight_digest`` -- sha256 of the reference model's tensors after loading the repo's
  seeded weights (so the exported directory's contents are pinned too).
"""
from __future__ import annotations

import ast
import json
import os
import sys
import tempfile

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
REF = "/root/reference"

from make_golden import _import_reference, build_reference_model  # noqa: E402
from t5gemma_tts_amd.config import named_config  # noqa: E402
from t5gemma_tts_amd.weights import state_dict_digest  # noqa: E402


def voice_defaults() -> dict:
    with open(os.path.join(REF, "hf_export/configuration_t5gemma_voice.py"), encoding="utf-8") as f:
        tree = ast.parse(f.read())
    for node in ast.walk(tree):
        if isinstance(node, ast.ClassDef) and node.name == "T5GemmaVoiceConfig":
            for fn in node.body:
                if isinstance(fn, ast.FunctionDef) and fn.name == "__init__":
                    names = [a.arg for a in fn.args.args][1:]
                    defs = [ast.literal_eval(d) for d in fn.args.defaults]
                    return dict(zip(names[len(names) - len(defs):], defs))
    raise RuntimeError("T5GemmaVoiceConfig.__init__ not found")


def export_config_json(cfg, t5_dict: dict, defaults: dict) -> dict:
    """config.json of ``export_t5gemma_voice_hf.py`` for a checkpoint trained with ``cfg``'s
    args (fields the args do not set keep the script's getattr defaults)."""
    from transformers import PretrainedConfig

    fields = dict(defaults)
    fields.update(t5gemma_model_name="google/t5gemma-2b-2b-ul2", t5_config_dict=t5_dict,
                  attn_implementation=cfg.backbone.attn_implementation, precision="bfloat16",
                  prune_text_modules=2, tie_word_embeddings=False, tie_input_output_embeddings=False,
                  audio_vocab_size=cfg.audio_vocab_size, empty_token=cfg.empty_token, eog=cfg.eog,
                  eos=cfg.eos, audio_pad_token=cfg.audio_pad_token, y_sep_token=cfg.y_sep_token,
                  x_sep_token=cfg.x_sep_token, extra_cutoff=cfg.extra_cutoff)

    class _VoiceConfig(PretrainedConfig):
        model_type = "t5gemma_voice"
        is_encoder_decoder = True

        def __init__(self, **kw):
            kw = {**defaults, **kw}
            ids = dict(bos_token_id=kw["empty_token"], eos_token_id=kw["eos"], pad_token_id=kw["audio_pad_token"])
            super().__init__(**ids)
            for k, v in kw.items():
                setattr(self, k, v)
            self.text_input_type = "text"
            self.auto_map = {"AutoConfig": "configuration_t5gemma_voice.T5GemmaVoiceConfig",
                             "AutoModelForSeq2SeqLM": "modeling_t5gemma_voice.T5GemmaVoiceForConditionalGeneration"}

    with tempfile.TemporaryDirectory() as td:
        _VoiceConfig(**fields).save_pretrained(td)
        with open(os.path.join(td, "config.json")) as f:
            return json.load(f)


def main():
    RT, _ = _import_reference()
    with open(os.path.join(HERE, "golden_tiny_eager.json")) as f:
        meta = json.load(f)
    cfg = named_config(meta["config"], **meta["config_kw"])
    defaults = voice_defaults()
    out = {"source": "tests/golden/make_golden_export.py", "golden": "golden_tiny_eager",
           "config": meta["config"], "config_kw": meta["config_kw"], "weight_seed": meta["weight_seed"],
           "voice_defaults": defaults}
    with tempfile.TemporaryDirectory() as td:
        m, sd_seed = build_reference_model(RT, cfg, meta["weight_seed"], td)
        sd = {k: v for k, v in m.state_dict().items()
              if not (k.startswith("encoder_module.") or k.startswith("decoder_module."))}
        pruned = {k: v for k, v in sd.items() if not k.startswith("backbone.lm_head.")
                  and not k.startswith("backbone.model.decoder.embed_tokens.")}
        out["state_dict"] = {k: list(v.shape) for k, v in sorted(pruned.items())}
        # prune_text_modules 0 keeps the text-side decoder embedding and lm_head
        from transformers import T5GemmaForConditionalGeneration
        bcfg = m.backbone.config
        with torch.device("meta"):
            full = T5GemmaForConditionalGeneration(bcfg)
        out["state_dict_unpruned_extra"] = {
            "backbone." + k: list(v.shape) for k, v in sorted(full.state_dict().items())
            if k.startswith("lm_head.") or k.startswith("model.decoder.embed_tokens.")}
        del full
        out["weight_digest"] = state_dict_digest({k: v for k, v in pruned.items()})
        out["seeded_digest"] = state_dict_digest({k: sd_seed[k] for k in pruned if k in sd_seed})
        # the backbone config the export stores (base_cfg.to_dict() after untying)
        bcfg.tie_word_embeddings = False
        for side in ("encoder", "decoder"):
            sub = getattr(bcfg, side, None)
            if sub is not None:
                sub.tie_word_embeddings = False
        t5_dict = bcfg.to_dict()
    t5_dict.pop("_name_or_path", None)
    out["config_json"] = export_config_json(cfg, t5_dict, defaults)
    with open(os.path.join(HERE, "golden_export.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote golden_export.json:", len(out["state_dict"]), "tensors,",
          len(out["state_dict_unpruned_extra"]), "unpruned extras")


if __name__ == "__main__":
    main()
