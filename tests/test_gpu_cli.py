"""The CLI entry on the GPU (synthetic tiny voice model + tiny codec): run_inference's
frames are the drop-in's own inference_tts tokens under seed_everything(seed) (the
reference's RNG contract), stripped of y_sep / EOS, and the wav is their decode."""
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_run_inference_synthetic_tiny_matches_drop_in():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd import cli
    from t5gemma_tts_amd.pipeline import strip_sep_and_eos
    model = cli.load_model(synthetic="tiny", max_text=64, max_audio=256)
    codec = cli.load_codec(codec="tiny", max_batch=1, max_frames=256)
    tok = cli.ByteTokenizer()
    with tempfile.TemporaryDirectory() as td:
        cli.run_inference(target_text="hello there", target_duration=0.6, seed=3, dump_tokens=True, output_dir=td,
                          model=model, audio_tokenizer=codec, text_tokenizer=tok)
        frames = np.load(os.path.join(td, "generated_frames.npy"))
        assert os.path.getsize(os.path.join(td, "generated.wav")) > 44
    cfg = model.config
    x = tok.encode("hello there")
    cli.seed_everything(3)
    _, gen = model.inference_tts(torch.tensor([x]), torch.tensor([len(x)]), torch.zeros(1, 0, 1, dtype=torch.long),
                                 tgt_y_lens=torch.tensor([int(50 * 0.6)]), top_k=30, top_p=0.9, min_p=0,
                                 temperature=0.8, stop_repetition=3, silence_tokens=[], prompt_frames=0)
    want = strip_sep_and_eos(gen, cfg.y_sep_token, cfg.eos)
    assert frames.reshape(-1).tolist() == want.reshape(-1).tolist()
