"""Parity mode's decode layer after the self attention as one persistent launch
(csrc/xlayer.hip: self o-proj, norm, cross-q, PM cross attention, cross-o, norm, gate/up
GeGLU, down in the reference's two K parts, norm, the next layer's q|k|v) against the same
step as parity mode's per-op launches (xmm.hip / norm.hip / xattn.hip): tokens and every
logit row bitwise equal, at the true 2b-2b widths (d 2304, FFN 9216, 8 x 256 q heads over 4
kv heads; 2 + 2 layers), for 1-8 rows, across repeated calls (the launch's counter sets
reset themselves), and after a hand-off timeout (the call reruns on the per-op launches).
Reference: hf_export/modeling_t5gemma_voice.py:256-323 (PMDecoderLayer), [tf]
modeling_t5gemma.py:81-97; the parity goldens (tests/test_gpu_parity_full.py) run the
persistent layer against the reference's own outputs."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN  # noqa: F401  (sys.path set-up)

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def _mid_engine(max_batch):
    import json
    import os
    from conftest import GOLDEN as G
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    from t5gemma_tts_amd.weights import synthetic_weights
    meta = json.load(open(os.path.join(G, "golden_mid.json")))
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=max_batch, max_text=64, max_audio=128, max_gen=40)
    return cfg, eng


def _utts(cfg, n, seed, max_text=40):
    from t5gemma_tts_amd.engine import Utterance
    rng = np.random.default_rng(seed)
    utts = []
    for _ in range(n):
        x = rng.integers(3, 4000, size=int(rng.integers(4, max_text))).tolist()
        tp = int(rng.integers(0, 40))
        y = rng.integers(0, 65536, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(8, 30))))
    return utts


def _run(eng, utts, p, seeds, fused):
    eng.set_fused(fused)
    before = eng.xlayer_launches()
    out = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
    return out, eng.xlayer_launches() - before


def _assert_same(a, b, B, tag):
    for r in range(B):
        assert a["gen"][r].tolist() == b["gen"][r].tolist(), (tag, r)
    assert len(a["logits"]) == len(b["logits"]), tag
    for s, (la, lb) in enumerate(zip(a["logits"], b["logits"])):
        assert torch.equal(la.view(torch.int16), lb.view(torch.int16)), (tag, s)


@pytest.mark.parametrize("B", [1, 3, 8])
def test_xlayer_bitwise_equal_to_per_op_exact_launches(B):
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(16)
    utts = _utts(cfg, B, 90 + B, max_text=64)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(700, 700 + B))
    on0, n_on0 = _run(eng, utts, p, seeds, True)
    off, n_off = _run(eng, utts, p, seeds, False)
    on1, n_on1 = _run(eng, utts, p, seeds, True)
    assert n_off == 0
    assert n_on0 >= cfg.backbone.num_decoder_layers and n_on1 >= cfg.backbone.num_decoder_layers   # the persistent layer ran
    _assert_same(on0, off, B, "on/off")
    _assert_same(on0, on1, B, "on/on")
    assert sum(len(g) for g in on0["gen"]) > B


def test_xlayer_not_used_past_its_shape():
    """More than 8 rows: parity mode keeps the per-op launches (no persistent layer)."""
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(16)
    utts = _utts(cfg, 9, 33)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    out, n = _run(eng, utts, p, list(range(9)), True)
    assert n == 0
    assert sum(len(g) for g in out["gen"]) > 9


def test_xlayer_handoff_timeout_reruns_on_per_op_launches():
    """The sticky timeout word set through the test hook: every in-launch wait of the
    persistent layer gives up at once (no hang), the call reports T5G_EHANDOFF and reruns on
    the per-op launches -- the tokens of a per-op run; the next call uses the launch again."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(8)
    utts = _utts(cfg, 4, 55)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(40, 44))
    ref, _ = _run(eng, utts, p, seeds, False)
    eng.set_fused(True)
    _lib.check(_lib.lib().t5g_engine_poison_handoff(eng.h, 77), "poison_handoff")
    with pytest.warns(UserWarning):
        out = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
    _assert_same(out, ref, 4, "rerun")
    again, n = _run(eng, utts, p, seeds, True)
    assert n > 0
    _assert_same(again, ref, 4, "again")
