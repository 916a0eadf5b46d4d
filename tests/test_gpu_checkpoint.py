"""The drop-in loaded from an export-shaped directory (config.json + sharded safetensors
under the reference export's names, tests/test_checkpoint_cpu.write_export) reproduces the
reference's tokens: ``T5GemmaVoiceForConditionalGeneration.from_pretrained(dir)`` then, per
golden_tiny_eager case, ``torch.manual_seed(seed); inference_tts(...)`` exactly as the
reference generated the golden (tests/golden/make_golden.py run_case). The config's
``attn_implementation`` is what turns the 50.0 softcap on -- the golden is the eager model."""
import json
import os
import tempfile

import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_from_pretrained_export_reproduces_reference_tokens():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd.engine import T5GemmaVoiceForConditionalGeneration
    from test_checkpoint_cpu import write_export
    with open(os.path.join(GOLDEN, "golden_tiny_eager.json")) as f:
        meta = json.load(f)
    with tempfile.TemporaryDirectory() as td:
        cfg, _ = write_export(td, shards=2, unpruned=True)
        model = T5GemmaVoiceForConditionalGeneration.from_pretrained(td, device="cuda:0", max_batch=1, max_text=64,
                                                                      max_audio=256, max_gen=200)
    assert model.config.backbone.softcap == 50.0
    exact = 0
    for c in meta["cases"]:
        torch.manual_seed(c["seed"])
        res, gen = model.inference_tts(torch.tensor([c["x"]]), torch.tensor([len(c["x"])]),
                                       torch.tensor(c["y"], dtype=torch.long).view(1, -1, 1),
                                       tgt_y_lens=torch.tensor([c["tgt"]]), top_k=c["top_k"], top_p=c["top_p"],
                                       min_p=c["min_p"], temperature=c["temperature"],
                                       stop_repetition=c["stop_repetition"], silence_tokens=c["silence_tokens"],
                                       prompt_frames=len(c["y"]))
        exact += int(gen.view(-1).tolist() == c["gen"] and res.view(-1).tolist() == c["res"])
    # golden_tiny_eager is free-running token-exact on every case (test_gpu_parity MIN_EXACT)
    assert exact == len(meta["cases"]), exact
