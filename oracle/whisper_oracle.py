"""CPU oracle for the Whisper recognizer (TEST INFRASTRUCTURE ONLY).

* ``ref_log_mel`` -- openai-whisper's log_mel_spectrogram (whisper/audio.py) restated with
  torch.stft: audio + 30 s of zeros, STFT 400 / 160 with the periodic Hann window
  (center, reflect), last frame dropped, |X|^2, slaney mel filters, log10 clamped at 1e-10,
  max - 8 floor, (x + 4) / 4. Pinned in tests/test_whisper_cpu.py against transformers'
  WhisperFeatureExtractor on the content frames.
* ``HFWhisper`` -- transformers WhisperForConditionalGeneration (fp32, eager attention) on
  the same openai-named weights, behind the interface t5gemma_tts_amd.whisper_asr.decode /
  transcribe drive (log_mel, encode, logits, detect_language), so the goldens run the
  product's host control flow over the architecture oracle's logits.
Parity against the openai-whisper package itself is UNPINNED (package and checkpoints
absent).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this file.
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch

N_SAMPLES, N_FRAMES = 480000, 3000


def ref_log_mel(audio: torch.Tensor, n_mels: int) -> torch.Tensor:
    """[n_mels][n // 160 + 3000] fp32 (whisper/audio.py log_mel_spectrogram(padding=N_SAMPLES))."""
    from t5gemma_tts_amd.whisper_asr import mel_filters
    audio = torch.nn.functional.pad(audio.reshape(-1).float(), (0, N_SAMPLES))
    window = torch.hann_window(400)
    stft = torch.stft(audio, 400, 160, window=window, return_complex=True)
    mag = stft[..., :-1].abs() ** 2
    mel = mel_filters(n_mels)[:, :201] @ mag
    log_spec = torch.clamp(mel, min=1e-10).log10()
    log_spec = torch.maximum(log_spec, log_spec.max() - 8.0)
    return (log_spec + 4.0) / 4.0


def hf_config(dims):
    from transformers import WhisperConfig
    return WhisperConfig(vocab_size=dims.n_vocab, num_mel_bins=dims.n_mels, encoder_layers=dims.n_audio_layer,
                         encoder_attention_heads=dims.n_audio_head, decoder_layers=dims.n_text_layer,
                         decoder_attention_heads=dims.n_text_head, d_model=dims.n_audio_state,
                         encoder_ffn_dim=4 * dims.n_audio_state, decoder_ffn_dim=4 * dims.n_text_state,
                         max_source_positions=dims.n_audio_ctx, max_target_positions=dims.n_text_ctx,
                         activation_function="gelu", scale_embedding=False, attn_implementation="eager")


def hf_model(dims, sd: Dict[str, torch.Tensor]):
    """WhisperForConditionalGeneration carrying the openai-named weights sd."""
    from transformers import WhisperForConditionalGeneration
    from t5gemma_tts_amd.whisper_asr import hf_to_openai_names
    m = WhisperForConditionalGeneration(hf_config(dims)).eval()
    state = m.state_dict()
    new = {}
    for k in state:
        if k == "proj_out.weight":
            new[k] = sd["decoder.token_embedding.weight"]
            continue
        (name,) = hf_to_openai_names({k: None}).keys()
        new[k] = sd[name].reshape(state[k].shape).float()
    m.load_state_dict(new)
    return m


class HFWhisper:
    """transformers Whisper behind the WhisperModel interface (batch 1, fp32 CPU)."""

    def __init__(self, dims, sd, tokenizer=None):
        self.dims, self.tokenizer = dims, tokenizer
        self.model = hf_model(dims, sd)
        self.mel = None
        self.mel_frames = 0
        self.feat = None
        self.pkv = None

    is_multilingual = property(lambda self: self.dims.is_multilingual)
    num_languages = property(lambda self: self.dims.num_languages)

    @torch.no_grad()
    def log_mel(self, audio, out=False):
        self.mel = ref_log_mel(torch.as_tensor(audio), self.dims.n_mels)
        self.mel_frames = self.mel.shape[-1]
        return self.mel.T.contiguous() if out else None

    @torch.no_grad()
    def encode(self, seek, seg_frames, out=False):
        win = torch.zeros(self.dims.n_mels, N_FRAMES)
        win[:, :seg_frames] = self.mel[:, seek:seek + seg_frames]
        self.feat = self.model.model.encoder(win[None]).last_hidden_state
        self.pkv = None
        return self.feat[0] if out else None

    @torch.no_grad()
    def logits(self, tokens: Sequence[int], offset: int) -> torch.Tensor:
        if offset == 0:
            self.pkv = None
        ids = torch.tensor([list(tokens)], dtype=torch.long)
        o = self.model(encoder_outputs=(self.feat,), decoder_input_ids=ids, past_key_values=self.pkv,
                       use_cache=True)
        self.pkv = o.past_key_values
        return o.logits[0]

    def detect_language(self, tokenizer):
        from t5gemma_tts_amd.whisper_asr import WhisperModel
        return WhisperModel.detect_language(self, tokenizer)

    def transcribe(self, audio, **kw):
        from t5gemma_tts_amd.whisper_asr import transcribe
        return transcribe(self, audio, **kw)


def write_synthetic_tiktoken(path: str, n_ordinary: int = 50257, seed: int = 0) -> None:
    """A tiktoken-format vocabulary of n_ordinary byte strings: the 256 single bytes, then
    seeded concatenations of two earlier entries (so every entry is reachable by BPE
    merges). Stands in for openai's multilingual.tiktoken asset, which is absent."""
    import base64
    import random
    rng = random.Random(seed)
    toks = [bytes([b]) for b in range(256)]
    seen = set(toks)
    while len(toks) < n_ordinary:
        a = toks[rng.randrange(min(len(toks), 4096))]
        b = toks[rng.randrange(min(len(toks), 4096))]
        t = a + b
        if len(t) <= 8 and t not in seen:
            seen.add(t)
            toks.append(t)
    with open(path, "w") as f:
        for i, t in enumerate(toks):
            f.write(f"{base64.b64encode(t).decode()} {i}\n")
