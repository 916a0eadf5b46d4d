"""Pin the CPU oracle against golden vectors captured from the reference itself
(tests/golden/make_golden.py). CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle.t5g_oracle import SamplerParams, T5GemmaTTSOracle, draw_noise, sample_helper, \
    top_k_top_p_filtering, RowState
from t5gemma_tts_amd.config import named_config
from t5gemma_tts_amd.weights import state_dict_digest, synthetic_weights


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    npz = os.path.join(GOLDEN, name + ".npz")
    arrs = dict(np.load(npz)) if os.path.exists(npz) else {}
    return meta, arrs


def _params(c):
    return SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"],
                         temperature=c["temperature"], stop_repetition=c["stop_repetition"],
                         silence_tokens=tuple(c["silence_tokens"]))


def _bits(t):
    return t.contiguous().view(torch.int16).numpy()


@pytest.mark.parametrize("name", ["golden_tiny", "golden_tiny_eager", "golden_tiny_window"])
def test_oracle_matches_reference_tokens(name):
    if not os.path.exists(os.path.join(GOLDEN, name + ".json")):
        pytest.skip("fixture not generated")
    meta, arrs = _load(name)
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    assert state_dict_digest(sd) == meta["weight_sha256"], "weight generator drifted"
    orc = T5GemmaTTSOracle(cfg, sd)
    for ci, c in enumerate(meta["cases"]):
        out = orc.generate(c["x"], c["y"], c["tgt"], _params(c), seed=c["seed"], record_logits=True)
        ref = arrs[f"logits_{ci}"]
        got = _bits(out["logits"])
        assert got.shape == ref.shape, (ci, got.shape, ref.shape)
        assert np.array_equal(got, ref), f"case {ci}: logits differ at steps {np.nonzero((got != ref).any(1))[0][:5]}"
        assert out["gen"].view(-1).tolist() == c["gen"], ci
        assert out["res"].view(-1).tolist() == c["res"], ci


def test_sampler_matches_reference():
    from tests.golden.make_golden import make_sampler_logits
    meta, _ = _load("golden_sampler")
    for c in meta["cases"]:
        logits = make_sampler_logits(c["logit_seed"], c["V"], c["scale"], c["quant"])
        g = torch.Generator().manual_seed(c["noise_seed"])
        noise = draw_noise(g, c["V"])
        x = logits.clone()
        if c["temperature"] != 1.0:
            x = x / c["temperature"]
        filt = top_k_top_p_filtering(x, top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"])
        surv = torch.nonzero(torch.isfinite(filt)).view(-1)
        assert surv.numel() == c["n_survivors"]
        assert surv[:64].tolist() == c["survivors_head"]
        probs = torch.softmax(filt, -1)
        tok = int(torch.argmax(probs / noise))
        assert tok == c["token"]


def test_oracle_matches_reference_mid():
    """True 2b-2b widths (reduced depth): token ids, per-step logit sha and top-64."""
    import hashlib
    name = "golden_mid"
    if not os.path.exists(os.path.join(GOLDEN, name + ".json")):
        pytest.skip("fixture not generated")
    meta, arrs = _load(name)
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    assert state_dict_digest(sd) == meta["weight_sha256"]
    orc = T5GemmaTTSOracle(cfg, sd)
    for ci, c in enumerate(meta["cases"]):
        out = orc.generate(c["x"], c["y"], c["tgt"], _params(c), seed=c["seed"], record_logits=True)
        assert out["gen"].view(-1).tolist() == c["gen"], ci
        bits = _bits(out["logits"])
        shas = [hashlib.sha256(r.astype(np.int16).tobytes()).hexdigest()[:16] for r in bits]
        assert shas == c["logit_sha"], ci


def test_oracle_matches_reference_full_depth():
    """Full 26+26-layer 2b-2b at the C3 shapes (T_x 60, T_p 151), 16 steps per case: token
    ids and every step's full logit-row sha equal the reference's own run (same host,
    same thread count as the fixture)."""
    import hashlib
    name = "golden_full"
    if not os.path.exists(os.path.join(GOLDEN, name + ".json")):
        pytest.skip("fixture not generated")
    meta, arrs = _load(name)
    torch.set_num_threads(meta["threads"])
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    assert state_dict_digest(sd) == meta["weight_sha256"]
    orc = T5GemmaTTSOracle(cfg, sd)
    for ci, c in enumerate(meta["cases"]):
        out = orc.generate(c["x"], c["y"], c["tgt"], _params(c), seed=c["seed"], record_logits=True)
        assert out["gen"].view(-1).tolist() == c["gen"], ci
        bits = _bits(out["logits"])
        shas = [hashlib.sha256(r.astype(np.int16).tobytes()).hexdigest()[:16] for r in bits]
        assert shas == c["logit_sha"], ci
        top = torch.topk(out["logits"].float(), 64, dim=-1)
        assert np.array_equal(top.indices.numpy().astype(np.int32), arrs[f"top_idx_{ci}"]), ci


def test_oracle_fp64_restatement_tracks_bf16():
    """The fp64 restatement (noise-floor yardstick of test_gpu_noise_floor.py) runs the same
    graph: on the tiny golden case its logits stay within bf16 rounding noise of the bf16
    oracle's, and the bf16 oracle itself is unchanged (pinned by the goldens above)."""
    meta, _ = _load("golden_tiny")
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    c = meta["cases"][0]
    o16, o64 = T5GemmaTTSOracle(cfg, sd), T5GemmaTTSOracle(cfg, sd, dtype=torch.float64)
    a, b = o16.prepare(c["x"], c["y"], c["tgt"]), o64.prepare(c["x"], c["y"], c["tgt"])
    b["state"] = a["state"]
    for tok in c["gen"][:8]:
        l16, l64 = o16.step_logits(a), o64.step_logits(b)
        assert l64.dtype == torch.float64
        err = (l16.double() - l64).abs().max().item() / l64.abs().max().item()
        assert 0.0 < err < 0.05, err
        a["state"].current_length += 1
        o16.advance(a, tok)
        o64.advance(b, tok)
