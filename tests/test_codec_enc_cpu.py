"""XCodec2 encoder host side on CPU: the constant tables the kernels use against the
transformers functions they restate (Kaldi mel filters, povey window, Kaiser-sinc
anti-aliasing filter), the weight-name table against transformers ``Xcodec2Model``, and
the fbank front end's GPU algorithm (frame -> DC removal -> pre-emphasis -> window ->
DFT-as-GEMM -> power -> mel GEMM -> log -> per-bin normalisation), run here in fp32
torch, against the SeamlessM4T features of the committed golden."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

import t5gemma_tts_amd  # noqa: F401
from t5gemma_tts_amd import codec_enc as E


def test_tables_match_transformers():
    from transformers.audio_utils import mel_filter_bank, window_function
    from transformers.models.xcodec2.modeling_xcodec2 import kaiser_sinc_filter1d
    ref = mel_filter_bank(num_frequency_bins=257, num_mel_filters=80, min_frequency=20, max_frequency=8000,
                          sampling_rate=16000, norm=None, mel_scale="kaldi", triangularize_in_mel_space=True)
    got = E.kaldi_mel_filters()
    assert got.shape == (80, 288) and torch.all(got[:, 257:] == 0)
    assert np.abs(got[:, :257].numpy().T - ref).max() < 1e-6
    assert np.abs(E.povey_window().numpy() - window_function(400, "povey", periodic=False)).max() < 1e-6
    assert torch.allclose(E.kaiser_sinc_filter(), kaiser_sinc_filter1d(0.25, 0.3, 12).view(-1), atol=1e-7)
    B = E.fbank_dft_basis().double()
    x = torch.randn(512, dtype=torch.float64)
    X = torch.fft.rfft(x)
    assert torch.allclose(B[0:514:2] @ x, X.real, atol=1e-4) and torch.allclose(B[1:514:2] @ x, X.imag, atol=1e-4)


def test_weight_names_match_transformers_model():
    from transformers import Xcodec2Config, Xcodec2Model
    cfg = E.encoder_tiny()
    sem = dict(hidden_size=cfg.sem_hidden, num_attention_heads=cfg.sem_heads, intermediate_size=cfg.sem_intermediate,
               num_hidden_layers=cfg.sem_layers)
    with torch.device("meta"):
        m = Xcodec2Model(Xcodec2Config(hidden_size=cfg.hidden, num_attention_heads=cfg.hidden // 64,
                                       encoder_hidden_size=cfg.ac_channels0, quantization_dim=cfg.fc_dim,
                                       semantic_model_config=sem))
    ref = {k: tuple(v.shape) for k, v in m.state_dict().items()
           if not (k.startswith("acoustic_decoder.") or k.startswith("quantizer.project_out")
                   or k == "semantic_encoder.masked_spec_embed")}
    assert E.encoder_weight_shapes(cfg) == ref


def _fbank_like_gpu(wav: torch.Tensor) -> torch.Tensor:
    """xc2enc.hip's front end step by step, fp32."""
    n = wav.numel()
    T = E.num_codes(n)
    F = 2 * T
    sig = torch.zeros(T * E.HOP + 320 + 400)
    sig[160:160 + n] = wav * 32768.0
    idx = torch.arange(F)[:, None] * 160 + torch.arange(400)[None, :]
    fr = sig[idx]
    fr = fr - fr.mean(1, keepdim=True)
    y = fr.clone()
    y[:, 1:] = fr[:, 1:] - 0.97 * fr[:, :-1]
    y[:, 0] = fr[:, 0] * (1.0 - 0.97)
    y = y * E.povey_window()
    frames = torch.zeros(F, 512)
    frames[:, :400] = y
    spec = frames @ E.fbank_dft_basis().T
    pw = torch.zeros(F, 288)
    pw[:, :257] = spec[:, 0:514:2] ** 2 + spec[:, 1:514:2] ** 2
    lm = torch.log(torch.clamp(pw @ E.kaldi_mel_filters().T, min=1.1920929e-7))
    lm = (lm - lm.mean(0)) / torch.sqrt(lm.var(0, unbiased=True) + 1e-7)
    return lm.reshape(T, 160)


@pytest.mark.parametrize("name", ["tiny", "full16k"])
def test_fbank_algorithm_vs_seamless_features(name):
    z = np.load(os.path.join(GOLDEN, f"golden_codec_enc_{name}.npz"))
    got = _fbank_like_gpu(torch.from_numpy(z["wav"]))
    ref = torch.from_numpy(z["features"])
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err < 2e-3, err


def test_golden_meta_consistent():
    for name in ("tiny", "full16k"):
        with open(os.path.join(GOLDEN, f"golden_codec_enc_{name}.json")) as f:
            meta = json.load(f)
        z = np.load(os.path.join(GOLDEN, f"golden_codec_enc_{name}.npz"))
        assert z["codes"].shape == (E.num_codes(meta["n_samples"]),) == (meta["n_codes"],)
        assert z["latent"].shape == (meta["n_codes"], 8)
        assert z["codes"].min() >= 0 and z["codes"].max() < 4 ** 8
