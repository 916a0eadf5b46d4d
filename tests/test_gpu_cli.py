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


def test_run_inference_transcribes_reference_speech_with_whisper(tmp_path, monkeypatch):
    """reference_speech without reference_text (inference_commandline_hf.py:144-150): the
    CLI loads a local openai-format Whisper checkpoint by name from the whisper cache
    directory (here a seeded tiny one plus a synthetic tiktoken vocabulary), transcribes
    the reference WAV on the GPU, and the transcript becomes the prompt text -- the same
    prompt run_inference builds when that text is passed as reference_text."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sys
    from t5gemma_tts_amd import cli, whisper_asr
    from t5gemma_tts_amd.audio import write_wav
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "oracle"))
    sys.path.insert(0, os.path.join(repo, "tests", "golden"))
    from make_golden_codec_enc import test_wave
    from whisper_oracle import write_synthetic_tiktoken
    cache = tmp_path / "whisper"
    cache.mkdir()
    d = whisper_asr.dims_tiny()
    torch.save({"dims": dict(d.__dict__), "model_state_dict": whisper_asr.synthetic_weights(d, 41)},
               str(cache / "tiny-test.pt"))
    write_synthetic_tiktoken(str(cache / "multilingual.tiktoken"), 50257, 0)
    monkeypatch.setenv("XDG_CACHE_HOME", str(tmp_path))
    ref = str(tmp_path / "ref.wav")
    write_wav(ref, test_wave(16000 * 2, 3), 16000)
    model = cli.load_model(synthetic="tiny", max_text=2048, max_audio=512)

    class TinyVocabCodec:
        """The tiny codec with its codes folded into the tiny voice model's 64 audio tokens
        (the two synthetic configs do not share a vocabulary)."""
        def __init__(self, c):
            self.c = c

        def __getattr__(self, k):
            return getattr(self.c, k)

        def encode(self, wav):
            return self.c.encode(wav) % 64
    codec = TinyVocabCodec(cli.load_codec(codec="tiny", max_batch=1, max_frames=512))
    tok = cli.ByteTokenizer()
    # run_inference seeds before it loads and runs Whisper, and random weights make the
    # transcription fall back to sampled temperatures: replay the same seeded sequence
    cli.seed_everything(3)
    asr = whisper_asr.load_model("tiny-test", device="cuda:0")
    text = asr.transcribe(ref)["text"]
    seen = []
    import t5gemma_tts_amd.pipeline as pl
    orig = pl.inference_one_sample

    def spy(**kw):
        seen.append(kw["prefix_transcript"])
        return orig(**kw)
    monkeypatch.setattr(pl, "inference_one_sample", spy)
    with tempfile.TemporaryDirectory() as td:
        cli.run_inference(reference_speech=ref, target_text="hi", target_duration=0.4, seed=3, output_dir=td,
                          model=model, audio_tokenizer=codec, text_tokenizer=tok, whisper_model="tiny-test")
        assert os.path.getsize(os.path.join(td, "generated.wav")) > 44
    from t5gemma_tts_amd.text import normalize_text_with_lang
    _, lang_code = normalize_text_with_lang("hi", None)
    assert seen and seen[0] == normalize_text_with_lang(text, lang_code)[0]


@pytest.mark.timeout(900)
def test_run_inference_accepts_reference_extremes(tmp_path):
    """the drop-in CLI path accepts the reference's extremes -- a 100 s
    reference clip (cut_off_sec = 100, inference_commandline_hf.py:91, 181: 5 001 codes, a
    5 003-token prefill) and a 90 s target (4 500 frames + the extra_cutoff budget) -- on
    the full-size 2b-2b model in parity mode (the default), through the XCodec2 encoder,
    the engine and the 44.1 kHz decoder, with the CLI's default sizing (cli.load_codec)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import sys
    from t5gemma_tts_amd import cli
    from t5gemma_tts_amd.audio import write_wav
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import MAX_AUDIO, T5GemmaVoiceForConditionalGeneration
    from t5gemma_tts_amd.weights import synthetic_weights
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "tests", "golden"))
    from make_golden_codec_enc import test_wave
    cfg = named_config("2b2b")
    model = T5GemmaVoiceForConditionalGeneration(cfg, synthetic_weights(cfg, 7, device="cuda"), device="cuda:0",
                                                 max_batch=1, max_text=512, max_audio=MAX_AUDIO)
    codec = cli.load_codec(codec="44k", max_batch=1)
    ref = str(tmp_path / "ref100s.wav")
    write_wav(ref, test_wave(16000 * 100, 5), 16000)
    out = cli.run_inference(reference_speech=ref, reference_text="a reference transcript of one hundred seconds",
                            target_text="the target sentence that should take about ninety seconds to speak",
                            target_duration=90.0, seed=1, dump_tokens=True, output_dir=str(tmp_path / "out"),
                            model=model, audio_tokenizer=codec, text_tokenizer=cli.ByteTokenizer())
    assert os.path.exists(out)
    concat = np.load(str(tmp_path / "out" / "concat_frames.npy")).reshape(-1)
    gen = np.load(str(tmp_path / "out" / "generated_frames.npy")).reshape(-1)
    print(f"100 s prompt + 90 s target: concat {concat.size} frames, generated {gen.size}")
    assert concat.size - gen.size == 16000 * 100 // 320 + 1        # the 5 001 prompt codes
    # random weights may sample EOS before the time budget (the reference's stop rule); the
    # budget of a 90 s target is the ceiling
    assert 1 <= gen.size <= 4500 + 50 * cfg.extra_cutoff + 2
