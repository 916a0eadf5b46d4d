"""XCodec2 encoder on the GPU (xc2e_* C ABI) against the transformers port's
``Xcodec2Model.encode`` goldens (tests/golden/make_golden_codec_enc.py), at a reduced width
and at the real 16 kHz dims (w2v-BERT 16 x 1024, acoustic 48 -> 1536 channels):

* the fbank front end against SeamlessM4TFeatureExtractor's features (fp32 vs the
  extractor's fp64: <= 2e-3 absolute on unit-variance features);
* the project_in latents within 1e-2 x their RMS (fp32 GEMM-order differences through
  ~40 layers);
* the codec ids equal, except where the golden latent sits within 2e-3 of an FSQ rounding
  boundary (a tie the fp32 order could flip; measured on MI355X: every id equal, 42/42
  and 63/63, features within 1.3e-5, latents within 1.5e-5 x RMS).
Parity against the pip ``xcodec2`` package the reference imports is unpinned (absent)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _load(name):
    with open(os.path.join(GOLDEN, f"golden_codec_enc_{name}.json")) as f:
        meta = json.load(f)
    return meta, dict(np.load(os.path.join(GOLDEN, f"golden_codec_enc_{name}.npz")))


def _bounded(p, level=4):
    half_range = (level - 1) * (1 + 1e-3) / 2
    offset = 0.5 if level % 2 == 0 else 0.0
    shift = np.arctanh(offset / half_range)
    b = np.tanh(p + shift) * half_range - offset
    return np.tanh(b + shift) * half_range - offset


@pytest.mark.parametrize("name", ["tiny", "full16k"])
def test_encoder_vs_transformers_golden(name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd.codec_enc import EncoderConfig, XCodec2Encoder, synthetic_encoder_weights
    meta, z = _load(name)
    c = dict(meta["config"])
    c["strides"], c["levels"] = tuple(c["strides"]), tuple(c["levels"])
    cfg = EncoderConfig(**c)
    enc = XCodec2Encoder(cfg, synthetic_encoder_weights(cfg, meta["weight_seed"]), device="cuda:0", max_seconds=2.0)
    wav = torch.from_numpy(z["wav"])
    feat = enc.features(wav).cpu()
    ferr = (feat - torch.from_numpy(z["features"])).abs().max().item()
    codes, lat = enc.encode(wav, return_latent=True)
    torch.cuda.synchronize()
    codes = codes.view(-1).cpu().numpy()
    lat = lat.cpu().numpy()
    ref_lat = z["latent"]
    rms = float(np.sqrt((ref_lat ** 2).mean()))
    lerr = float(np.abs(lat - ref_lat).max()) / rms
    b = _bounded(ref_lat)
    near = (np.abs(b - np.floor(b) - 0.5) < 2e-3).any(axis=1)
    same = codes == z["codes"]
    print(f"{name}: features max |err| {ferr:.2e}, latent max err / rms {lerr:.2e}, codes equal "
          f"{int(same.sum())}/{same.size} ({int(near.sum())} near a rounding boundary)")
    assert ferr <= 2e-3, ferr
    assert lerr <= 1e-2, lerr
    assert np.all(same | near), np.nonzero(~same)[0]


def test_audio_tokenizer_encode_and_prompt_from_wav_file(tmp_path):
    """AudioTokenizer.encode (data/tokenizer.py:105-115 shape contract) and the prompt path
    of inference_one_sample from a reference WAV file: cut to prompt_end_frame samples of
    the file's rate, resampled to 16 kHz, encoded -- the codes the engine receives."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd.audio import load_audio, resample, write_wav
    from t5gemma_tts_amd.codec import AudioTokenizer, codec_tiny, synthetic_codec_weights
    from t5gemma_tts_amd.codec_enc import encoder_tiny, num_codes, synthetic_encoder_weights
    from t5gemma_tts_amd.pipeline import prompt_codes_from, prompt_frames_for_samples
    ecfg = encoder_tiny()
    tok = AudioTokenizer(device="cuda:0", cfg=codec_tiny(), state_dict=synthetic_codec_weights(codec_tiny(), 22),
                         encoder_cfg=ecfg, encoder_state_dict=synthetic_encoder_weights(ecfg, 31), max_batch=2,
                         max_frames=256, max_encode_seconds=3.0)
    _, z = _load("tiny")
    wav = torch.from_numpy(z["wav"])
    codes = tok.encode(wav.view(1, 1, -1))
    assert codes.shape == (1, 1, num_codes(wav.numel())) and codes.dtype == torch.long
    assert torch.equal(codes, tok.encoder.encode(wav))     # deterministic, batch row == single call
    # a 44.1 kHz reference file, cut at 0.5 s of its own samples
    w44 = resample(wav[None], 16000, 44100)[0]
    path = str(tmp_path / "ref.wav")
    write_wav(path, w44, 44100)
    cut = int(0.5 * 44100)
    got = prompt_codes_from(path, tok, cut, 44100)
    x, sr = load_audio(path, num_frames=cut)
    want = tok.encode(resample(x, sr, 16000).unsqueeze(0))
    assert got.shape[-1] == prompt_frames_for_samples(cut, 44100)
    assert torch.equal(got.cpu(), want.cpu())
