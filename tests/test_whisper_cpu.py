"""Whisper recognizer host side on CPU (no GPU calls): tables and restated algorithms
against transformers' Whisper port (the in-container oracle), the BPE tokenizer, the
checkpoint formats, the logit filters, the C ABI exports, and the oracle's golden
transcription."""
import ctypes as C
import json
import os
import re
import sys

import numpy as np
import pytest
import torch

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd import whisper_asr as w
from conftest import GOLDEN, REPO

sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, GOLDEN)


def test_language_codes_match_transformers():
    from transformers.models.whisper.tokenization_whisper import LANGUAGES
    assert w.LANGUAGE_CODES == list(LANGUAGES.keys())


@pytest.mark.parametrize("n_mels", [80, 128])
def test_mel_filters_match_transformers(n_mels):
    from transformers.audio_utils import mel_filter_bank
    ref = mel_filter_bank(num_frequency_bins=201, num_mel_filters=n_mels, min_frequency=0.0, max_frequency=8000.0,
                          sampling_rate=16000, norm="slaney", mel_scale="slaney")
    got = w.mel_filters(n_mels)
    assert got.shape == (n_mels, 224) and float(got[:, 201:].abs().max()) == 0.0
    assert np.allclose(got[:, :201].numpy(), ref.T, atol=1e-7, rtol=1e-5)


def test_dft_basis_power_is_the_stft_power():
    g = torch.Generator().manual_seed(0)
    frames = torch.randn(5, 400, generator=g, dtype=torch.float64)
    B = w.dft_basis().double()[:, :400]
    spec = frames @ B.T
    pw = spec[:, 0::2] ** 2 + spec[:, 1::2] ** 2
    ref = torch.fft.rfft(frames, dim=1).abs() ** 2
    assert torch.allclose(pw, ref, rtol=1e-5, atol=1e-5)
    win = w.hann_window()
    assert torch.allclose(win, torch.hann_window(400), atol=1e-7)


def test_ref_log_mel_matches_feature_extractor():
    """oracle ref_log_mel (openai log_mel_spectrogram) == WhisperFeatureExtractor on the
    content frames (both pad with 30 s of zeros before the STFT)."""
    from transformers import WhisperFeatureExtractor
    from make_golden_codec_enc import test_wave
    from whisper_oracle import ref_log_mel
    a = test_wave(int(3.3 * 16000), 4)
    for n_mels in (80, 128):
        fe = WhisperFeatureExtractor(feature_size=n_mels)
        hf = fe(a.numpy(), sampling_rate=16000, return_tensors="np")["input_features"][0]
        got = ref_log_mel(a, n_mels)
        assert got.shape == (n_mels, a.numel() // 160 + 3000)
        content = a.numel() // 160
        err = np.abs(got[:, :content].numpy() - hf[:, :content]).max()
        assert err < 2e-4, err


def test_hf_names_map_to_openai_names():
    from whisper_oracle import hf_config
    from transformers import WhisperForConditionalGeneration
    d = w.dims_tiny()
    m = WhisperForConditionalGeneration(hf_config(d))
    mapped = w.hf_to_openai_names(m.state_dict())
    shapes = w.weight_shapes(d)
    assert set(mapped) == set(shapes), set(mapped) ^ set(shapes)
    for k, v in mapped.items():
        assert tuple(v.shape) == shapes[k], k


def test_checkpoint_formats_load_the_same_weights(tmp_path):
    from safetensors.torch import save_file
    from whisper_oracle import hf_config, hf_model
    d = w.dims_tiny()
    sd = w.synthetic_weights(d, 5)
    torch.save({"dims": dict(d.__dict__), "model_state_dict": sd}, str(tmp_path / "tiny.pt"))
    dims, got, where = w.load_checkpoint("tiny", download_root=str(tmp_path))
    assert dims == d and where == str(tmp_path) and all(torch.equal(got[k], sd[k]) for k in sd)
    hf_dir = tmp_path / "hf"
    hf_dir.mkdir()
    m = hf_model(d, sd)
    with open(hf_dir / "config.json", "w") as f:
        json.dump(hf_config(d).to_dict(), f)
    save_file({k: v.contiguous() for k, v in m.state_dict().items() if k != "proj_out.weight"},
              str(hf_dir / "model.safetensors"))
    dims2, got2, _ = w.load_checkpoint(str(hf_dir))
    assert dims2 == d and set(got2) == set(sd)
    assert all(torch.allclose(got2[k], sd[k].float()) for k in sd)
    with pytest.raises(FileNotFoundError):
        w.load_checkpoint("large-v3-turbo", download_root=str(tmp_path))


def _tok(tmp_path, seed=0):
    from whisper_oracle import write_synthetic_tiktoken
    p = str(tmp_path / "v.tiktoken")
    write_synthetic_tiktoken(p, 50257, seed)
    return w.WhisperTokenizer.from_tiktoken(p, 100)


def test_tokenizer_specials_and_round_trip(tmp_path):
    tok = _tok(tmp_path)
    assert tok.n_vocab == 51866 and tok.eot == 50257 and tok.sot == 50258
    assert tok.transcribe == 50360 and tok.no_timestamps == 50364 and tok.timestamp_begin == 50365
    assert tok.with_language("ja").sot_sequence == (50258, 50259 + w.LANGUAGE_CODES.index("ja"), 50360)
    for text in ["hello world", " こんにちは、世界", "a  b\n\tc", "Ünïcödé 123 !?"]:
        ids = tok.encode(text)
        assert all(0 <= i < 50257 for i in ids)
        assert tok.decode(ids) == text
    # timestamps are dropped, specials decode to their text
    assert tok.decode([tok.sot, tok.timestamp_begin] + tok.encode("x")) == "<|startoftranscript|>x"
    ns = tok.non_speech_tokens
    assert len(ns) > 5 and all(i < 50257 for i in ns) and list(ns) == sorted(set(ns))


def test_bpe_merges_lowest_rank_first(tmp_path):
    import base64
    p = tmp_path / "small.tiktoken"
    toks = [bytes([b]) for b in range(256)] + [b"ll", b"he", b"hell", b"llo", b"hello", b" w"]
    p.write_text("".join(f"{base64.b64encode(t).decode()} {i}\n" for i, t in enumerate(toks)))
    bpe = w._BPE(w.load_tiktoken_ranks(str(p)))
    # "hello": ll (256) merges first, then he (257), then hell (258) -> [hell, o]; "hello"
    # itself is a vocabulary entry, so the whole piece maps to it directly
    assert bpe.encode("hello") == [260]
    assert bpe.encode("helo") == [257, ord("l"), ord("o")]
    assert bpe.encode("hellx") == [258, ord("x")]
    assert bpe.encode(" world") == [261, ord("o"), ord("r"), ord("l"), ord("d")]


class _GenCfg:
    def __init__(self, no_ts, eot):
        self.no_timestamps_token_id = no_ts
        self.eos_token_id = eot
        self.bos_token_id = eot
        self.max_initial_timestamp_index = 50


def test_timestamp_rules_match_transformers(tmp_path):
    from transformers.generation.logits_process import WhisperTimeStampLogitsProcessor
    tok = _tok(tmp_path)
    tb, eot = tok.timestamp_begin, tok.eot
    g = torch.Generator().manual_seed(3)
    rng = np.random.default_rng(3)
    begin = 3
    proc = WhisperTimeStampLogitsProcessor(_GenCfg(tok.no_timestamps, eot), begin_index=begin)
    n_cases = 0
    for case in range(200):
        L = int(rng.integers(0, 8))
        seq = [tok.sot, 50259, tok.transcribe]
        for _ in range(L):
            r = rng.random()
            seq.append(int(rng.integers(tb, tb + 300)) if r < 0.4 else (eot if r < 0.45 else int(rng.integers(0, 50257))))
        logits = torch.randn(tok.n_vocab, generator=g) * 3
        if case % 3 == 0:
            logits[tb:] += 4.0            # timestamp mass beats text in some cases
        ref = proc(torch.tensor([seq]), logits[None].clone())[0]
        got = logits.clone()
        w.apply_timestamp_rules(got, seq, begin, tok, 50)
        assert torch.equal(torch.isinf(got), torch.isinf(ref)), case
        assert torch.equal(got[~torch.isinf(got)], ref[~torch.isinf(ref)]), case
        n_cases += 1
    assert n_cases == 200


def test_suppress_lists(tmp_path):
    tok = _tok(tmp_path)
    st = w.suppress_token_list(tok, "-1")
    for t in (tok.transcribe, tok.translate, tok.sot, tok.sot_prev, tok.sot_lm, tok.no_speech):
        assert t in st
    assert set(tok.non_speech_tokens) <= set(st)
    logits = torch.zeros(tok.n_vocab)
    w.suppress_blank(logits, [1, 2, 3], 3, tok)
    assert torch.isinf(logits[tok.eot]) and all(torch.isinf(logits[i]) for i in tok.encode(" "))
    logits = torch.zeros(tok.n_vocab)
    w.suppress_blank(logits, [1, 2, 3, 4], 3, tok)
    assert not torch.isinf(logits).any()


def _header_symbols():
    src = open(os.path.join(REPO, "include", "whisper.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(whs_[a-z_0-9]+)\s*\(", src)))


def test_whs_exports_and_struct_sizes():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    syms = _header_symbols()
    assert set(syms) == set(w.WHS_SIGNATURES), set(syms) ^ set(w.WHS_SIGNATURES)
    for s in syms:
        assert hasattr(L, s), s
    assert C.sizeof(w.WHSConfig) == 11 * 4
    assert C.sizeof(w.WHSAttn) == 7 * 8
    assert C.sizeof(w.WHSBlock) == 24 * 8
    assert C.sizeof(w.WHSWeights) == 7 * 8 + 8 + 8 + 64 * 192 + 4 * 8 + 64 * 192 + 2 * 8


def test_whs_create_rejects_bad_config():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    fn = L.whs_create
    fn.restype, fn.argtypes = w.WHS_SIGNATURES["whs_create"]
    h = C.c_void_p()
    bad = w.WHSConfig(n_mels=80, n_audio_ctx=1500, n_audio_state=1000, n_audio_head=16, n_audio_layer=2,
                      n_vocab=51866, n_text_ctx=448, n_text_state=1000, n_text_head=16, n_text_layer=2,
                      max_samples=16000)
    assert fn(C.byref(bad), C.byref(w.WHSWeights()), C.byref(h)) == -1
    bad2 = w.WHSConfig(n_mels=80, n_audio_ctx=1000, n_audio_state=128, n_audio_head=2, n_audio_layer=2,
                       n_vocab=51866, n_text_ctx=448, n_text_state=128, n_text_head=2, n_text_layer=2,
                       max_samples=16000)
    assert fn(C.byref(bad2), C.byref(w.WHSWeights()), C.byref(h)) == -1


def test_oracle_transcription_reproduces_golden(tmp_path):
    """The golden generator is deterministic: HFWhisper + the host control flow give the
    committed tiny transcription and teacher-forced argmaxes again."""
    from make_golden_codec_enc import test_wave
    from whisper_oracle import HFWhisper
    with open(os.path.join(GOLDEN, "golden_whisper_tiny.json")) as f:
        meta = json.load(f)
    tok = _tok(tmp_path, meta["tok_seed"])
    d = w.dims_tiny()
    m = HFWhisper(d, w.synthetic_weights(d, meta["weight_seed"]), tok)
    audio = test_wave(int(meta["audio_seconds"] * 16000), meta["audio_seed"])
    m.log_mel(audio)
    m.encode(0, meta["content_frames"])
    lg = m.logits(meta["teacher_tokens"], 0)
    assert lg.argmax(-1).tolist() == meta["logit_argmax"]
    r = m.transcribe(audio, temperature=0.0)
    assert r["language"] == meta["transcribe_language"]
    assert [s["tokens"] for s in r["segments"]] == [s["tokens"] for s in meta["segments"]]
