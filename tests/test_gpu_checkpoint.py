"""The drop-in loaded from an export-shaped directory (config.json + sharded safetensors
under the reference export's names, tests/test_checkpoint_cpu.write_export) reproduces the
reference's tokens: ``T5GemmaVoiceForConditionalGeneration.from_pretrained(dir)`` then, per
golden case, ``torch.manual_seed(seed); inference_tts(...)`` exactly as the reference
generated the golden (tests/golden/make_golden.py run_case).

The export holds golden_tiny_eager's tensors (seed 8). Its config's ``attn_implementation``
decides the attention: "sdpa" is the path parity mode restates, so the export loaded that
way must match golden_tiny_s8_sdpa (the reference on the same weights with sdpa attention)
token for token; the reference default "eager" turns the 50.0 softcap on, which parity mode
does not restate -- inference_tts then runs the fast kernels (with a warning) and an
explicit ``parity=True`` is refused."""
import json
import os
import tempfile
import warnings

import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _load(td, **overrides):
    from t5gemma_tts_amd.engine import T5GemmaVoiceForConditionalGeneration
    from test_checkpoint_cpu import write_export
    write_export(td, shards=2, unpruned=True, config_overrides=overrides or None)
    return T5GemmaVoiceForConditionalGeneration.from_pretrained(td, device="cuda:0", max_batch=1, max_text=64,
                                                                max_audio=256, max_gen=200)


def _run(model, c, **kw):
    torch.manual_seed(c["seed"])
    return model.inference_tts(torch.tensor([c["x"]]), torch.tensor([len(c["x"])]),
                               torch.tensor(c["y"], dtype=torch.long).view(1, -1, 1),
                               tgt_y_lens=torch.tensor([c["tgt"]]), top_k=c["top_k"], top_p=c["top_p"],
                               min_p=c["min_p"], temperature=c["temperature"],
                               stop_repetition=c["stop_repetition"], silence_tokens=c["silence_tokens"],
                               prompt_frames=len(c["y"]), **kw)


def test_from_pretrained_export_reproduces_reference_tokens():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with open(os.path.join(GOLDEN, "golden_tiny_s8_sdpa.json")) as f:
        meta = json.load(f)
    with tempfile.TemporaryDirectory() as td:
        model = _load(td, attn_implementation="sdpa")
    assert model.config.backbone.softcap == 0.0
    exact = 0
    for c in meta["cases"]:
        res, gen = _run(model, c)
        exact += int(gen.view(-1).tolist() == c["gen"] and res.view(-1).tolist() == c["res"])
    assert exact == len(meta["cases"]), exact


def test_from_pretrained_eager_export_runs_fast_path():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with open(os.path.join(GOLDEN, "golden_tiny_eager.json")) as f:
        meta = json.load(f)
    with tempfile.TemporaryDirectory() as td:
        model = _load(td)
    assert model.config.backbone.softcap == 50.0   # the reference default attn_implementation
    c = meta["cases"][0]
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        res, gen = _run(model, c)
    assert any("eager (softcap)" in str(w.message) for w in rec)
    assert gen.numel() > 0 and res.numel() == len(c["y"]) + gen.numel()
    with pytest.raises(ValueError):
        _run(model, c, parity=True)
