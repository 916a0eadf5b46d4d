"""The decode MLP half as one persistent launch (csrc/fused.hip: cross-attention residual
norm -> gate/up GeGLU -> down, with in-launch hand-offs) against the same step as three
launches (resid_norm + the two register-X GEMVs): tokens and every logit row bitwise equal,
at the true 2b-2b widths (d 2304, FFN 9216; 2 + 2 layers), for 1, 8, 12 and 16 rows (the
whole-layer launch, one 16-row MFMA tile: 16 rows = 128 attention workers, the most it takes)
and 32 rows (the MLP-half launch, two tiles), and across repeated calls (the hand-off
counters reset themselves)."""
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


def _utts(cfg, n, seed):
    from t5gemma_tts_amd.engine import Utterance
    rng = np.random.default_rng(seed)
    utts = []
    for _ in range(n):
        x = rng.integers(3, 4000, size=int(rng.integers(4, 40))).tolist()
        tp = int(rng.integers(0, 40))
        y = rng.integers(0, 65536, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(8, 30))))
    return utts


@pytest.mark.parametrize("B", [1, 8, 12, 16, 32])
def test_fused_mlp_bitwise_equal_to_three_launches(B):
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(32)
    utts = _utts(cfg, B, 40 + B)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(300, 300 + B))
    runs, fast = [], []
    for fused in (True, False, True):
        eng.set_fused(fused)
        # the fast kernels step by step from the host loop (logits of every step recorded),
        # and the on-device graph-replayed loop (tokens)
        runs.append(eng.generate(utts, p, seeds=seeds, parity=True, exact=False, record_logits=True))
        fast.append(eng.generate(utts, p, seeds=seeds))
    for k in (1, 2):
        for b in range(B):
            assert fast[0]["gen"][b].tolist() == fast[k]["gen"][b].tolist(), (k, b)
    for k in (1, 2):
        for b in range(B):
            assert runs[0]["gen"][b].tolist() == runs[k]["gen"][b].tolist(), (k, b)
        assert len(runs[0]["logits"]) == len(runs[k]["logits"])
        for s, (l0, lk) in enumerate(zip(runs[0]["logits"], runs[k]["logits"])):
            assert torch.equal(l0.view(torch.int16), lk.view(torch.int16)), (k, s)
    assert sum(len(g) for g in runs[0]["gen"]) > B


def test_handoff_timeout_falls_back_to_per_op_launches():
    """A fused launch whose hand-offs give up (as when another process holds CUs): the
    sticky timeout word is set through the test hook, every in-launch wait then gives up at
    once (no hang), t5g_read_tokens reports T5G_EHANDOFF and clears the counters, and
    engine.generate reruns the call on the per-op launches -- the same tokens as a per-op
    run. Re-enabling the fused launch afterwards gives those tokens again."""
    _need_gpu()
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _mid_engine(8)
    utts = _utts(cfg, 8, 77)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(500, 508))
    eng.set_fused(False)
    ref = eng.generate(utts, p, seeds=seeds)
    eng.set_fused(True)
    _lib.check(_lib.lib().t5g_engine_poison_handoff(eng.h, 99), "poison_handoff")
    out = eng.generate(utts, p, seeds=seeds)
    for b in range(8):
        assert out["gen"][b].tolist() == ref["gen"][b].tolist(), b
    eng.set_fused(True)
    again = eng.generate(utts, p, seeds=seeds)
    for b in range(8):
        assert again["gen"][b].tolist() == ref["gen"][b].tolist(), b
