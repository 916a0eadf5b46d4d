"""Goldens for the Whisper recognizer from transformers' WhisperForConditionalGeneration
(oracle/whisper_oracle.py HFWhisper: fp32 CPU, eager attention) on seeded openai-named
weights, a seeded synthetic tiktoken vocabulary and a seeded speech-like 16 kHz signal.

Per config (tiny test dims; large-v3-turbo dims) it stores:
* the encoder output of the first window (seek 0, content frames), every 25th row;
* teacher-forced decoder logits of a fixed token sequence (sot, en, transcribe,
  timestamps and text ids) at every 53rd vocabulary id, plus each row's argmax / max;
* detect_language's language and top-5 probabilities;
* the tokens of transcribe(audio, temperature=0.0) -- the product's host control flow
  (t5gemma_tts_amd.whisper_asr) over the oracle's logits.
Run: python tests/golden/make_golden_whisper.py [tiny|turbo]
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, HERE)

CONFIGS = {
    "tiny": dict(dims="dims_tiny", weight_seed=41, audio_seconds=6.5, audio_seed=3, tok_seed=0),
    "turbo": dict(dims="dims_large_v3_turbo", weight_seed=42, audio_seconds=4.0, audio_seed=5, tok_seed=0),
}


def teacher_tokens(tok):
    tb = tok.timestamp_begin
    return list(tok.with_language("en").sot_sequence) + [tb, 1000, 2000, 30000, tb + 50, tok.eot]


def main(name):
    import t5gemma_tts_amd.whisper_asr as w
    from make_golden_codec_enc import test_wave
    from whisper_oracle import HFWhisper, write_synthetic_tiktoken
    torch.set_num_threads(8)
    c = CONFIGS[name]
    dims = getattr(w, c["dims"])()
    sd = w.synthetic_weights(dims, c["weight_seed"])
    tpath = "/tmp/golden_whisper.tiktoken"
    write_synthetic_tiktoken(tpath, 50257, c["tok_seed"])
    tok = w.WhisperTokenizer.from_tiktoken(tpath, dims.num_languages)
    m = HFWhisper(dims, sd, tok)
    audio = test_wave(int(c["audio_seconds"] * 16000), c["audio_seed"])
    m.log_mel(audio)
    content = m.mel_frames - 3000
    feat = m.encode(0, content, out=True)
    toks = teacher_tokens(tok)
    lg = m.logits(toks, 0)
    sub = np.arange(0, dims.n_vocab, 53)
    lang, probs = m.detect_language(tok.with_language("en"))
    top5 = sorted(probs.items(), key=lambda kv: -kv[1])[:5]
    r = m.transcribe(audio, temperature=0.0)
    meta = {"config": name, **c, "model_dims": dims.__dict__, "content_frames": content, "teacher_tokens": toks,
            "logit_argmax": lg.argmax(-1).tolist(), "logit_max": lg.max(-1).values.tolist(),
            "language": lang, "language_top5": top5, "transcribe_language": r["language"],
            "segments": [{"start": s["start"], "end": s["end"], "tokens": s["tokens"]} for s in r["segments"]],
            "torch": torch.__version__}
    with open(os.path.join(HERE, f"golden_whisper_{name}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(HERE, f"golden_whisper_{name}.npz"), feat_rows=feat[::25].numpy(),
                        logits_sub=lg[:, sub].numpy(), sub=sub)
    print(name, "language", lang, "segments", len(r["segments"]),
          "tokens", sum(len(s["tokens"]) for s in r["segments"]))


if __name__ == "__main__":
    for n in (sys.argv[1:] or ["tiny", "turbo"]):
        main(n)
