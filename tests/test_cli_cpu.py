"""The CLI surface (inference_commandline_hf.py:72-242) on CPU with recording fakes:
argument parsing, the reference's errors, duration estimation when ``target_duration`` is
absent, the prompt cut in samples of the reference file, and the outputs written
(generated.wav, the stats line, dumped frames)."""
import os
import tempfile
import wave

import numpy as np
import pytest
import torch

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd import cli
from t5gemma_tts_amd.config import named_config


class FakeModel:
    def __init__(self, gen):
        self.config = named_config("tiny")
        self.calls, self.gen = [], gen

    def inference_tts(self, x, x_lens, y, tgt_y_lens=None, **kw):
        self.calls.append({"x": x.tolist(), "y": y.tolist(), "tgt": tgt_y_lens.tolist(), "kw": kw})
        g = torch.tensor(self.gen, dtype=torch.long).view(1, 1, -1)
        return torch.cat([y.transpose(2, 1), g], dim=2), g


class FakeCodec:
    sample_rate = 44100
    encode_sample_rate = 16000

    def __init__(self):
        self.encoded = []

    def encode(self, wav):
        self.encoded.append(wav.shape[-1])
        return torch.arange(wav.shape[-1] // 320 + 1).view(1, 1, -1) % 60

    def decode(self, frames):
        return torch.full((frames.shape[0], 1, frames.shape[-1] * 882), 0.25)


def _run(td, **kw):
    model, codec = FakeModel([5, 6, 7, 67]), FakeCodec()
    out = cli.run_inference(model=model, audio_tokenizer=codec, text_tokenizer=cli.ByteTokenizer(), output_dir=td,
                            **kw)
    return out, model, codec


def test_writes_wav_stats_and_frames(capsys):
    with tempfile.TemporaryDirectory() as td:
        out, model, _ = _run(td, target_text="hello", target_duration=0.5, dump_tokens=True, seed=3)
        with wave.open(out) as w:
            assert w.getframerate() == 44100 and w.getnframes() == 3 * 882
        assert np.load(os.path.join(td, "generated_frames.npy")).tolist() == [[5, 6, 7]]
        text = capsys.readouterr().out
        assert "max_abs: 0.250000, rms: 0.250000" in text and "[Success]" in text
        c = model.calls[0]
        assert c["tgt"] == [25] and torch.tensor(c["y"]).numel() == 0
        assert c["x"][0] == [3 + b for b in b"hello"]
        assert c["kw"]["top_k"] == 30 and c["kw"]["top_p"] == 0.9 and c["kw"]["temperature"] == 0.8


def test_reference_text_without_speech_is_an_error():
    with tempfile.TemporaryDirectory() as td:
        with pytest.raises(ValueError):
            _run(td, target_text="hi", reference_text="ref", target_duration=1.0)


class FakeASR:
    def __init__(self):
        self.calls = []

    def transcribe(self, audio):
        self.calls.append(audio)
        return {"text": " whisper said this", "segments": [], "language": "en"}


def test_speech_without_transcript_is_transcribed_by_whisper(capsys):
    """:144-150: reference audio without reference_text -> Whisper's transcript becomes the
    prompt text (normalised like a given reference_text)."""
    from t5gemma_tts_amd.audio import write_wav
    with tempfile.TemporaryDirectory() as td:
        ref = os.path.join(td, "ref.wav")
        write_wav(ref, np.zeros(16000), 16000)
        asr = FakeASR()
        _, model, _ = _run(td, target_text="hi", reference_speech=ref, target_duration=1.0, asr_model=asr)
        assert asr.calls == [ref]
        assert "[Info] Whisper transcribed text:  whisper said this" in capsys.readouterr().out
        x = model.calls[0]["x"][0]
        with_text = _run(td, target_text="hi", reference_speech=ref, target_duration=1.0,
                         reference_text=" whisper said this")[1].calls[0]["x"][0]
        assert x == with_text


def test_whisper_checkpoint_is_never_downloaded(monkeypatch):
    with tempfile.TemporaryDirectory() as td:
        monkeypatch.setenv("XDG_CACHE_HOME", td)
        with pytest.raises(FileNotFoundError):
            _run(td, target_text="hi", reference_speech="a.wav", target_duration=1.0, whisper_model="large-v3-turbo")


def test_estimated_duration_and_sample_cut_of_reference_audio():
    from t5gemma_tts_amd.audio import write_wav
    from t5gemma_tts_amd.text import estimate_duration
    with tempfile.TemporaryDirectory() as td:
        ref = os.path.join(td, "ref.wav")
        write_wav(ref, np.zeros(44100 * 3), 44100)
        out, model, codec = _run(td, target_text="this is a test", reference_speech=ref, reference_text="a reference",
                                 cut_off_sec=1.5)
        dur = estimate_duration("this is a test", reference_speech=ref, reference_transcript="a reference",
                                target_lang=None, reference_lang=None)
        # 1.5 s of the 44.1 kHz file, resampled to 16 kHz, went to the encoder
        assert codec.encoded == [24000]
        T_p = 24000 // 320 + 1 + 1                    # codes + y_sep
        assert model.calls[0]["tgt"] == [T_p + int(50 * dur)]
        assert model.calls[0]["x"][0][-len("this is a test"):] == [3 + b for b in b"this is a test"]


def test_argparse_surface(monkeypatch):
    seen = {}
    monkeypatch.setattr(cli, "run_inference", lambda **kw: seen.update(kw))
    cli.main(["--target_text", "123", "--top_k", "5", "--silence_tokens", "[1, 2]", "--target_duration", "2.5",
              "--dump_tokens", "True", "--synthetic", "tiny"])
    assert seen["target_text"] == "123" and seen["top_k"] == 5 and seen["silence_tokens"] == [1, 2]
    assert seen["target_duration"] == 2.5 and seen["dump_tokens"] is True and seen["synthetic"] == "tiny"
    assert seen["seed"] == 1 and seen["temperature"] == 0.8 and seen["reference_speech"] is None
