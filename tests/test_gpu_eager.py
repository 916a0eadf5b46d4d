"""Parity mode for eager-attention checkpoints (attn_implementation="eager", the reference
default: hf_export/configuration_t5gemma_voice.py:59, config.py:87; [tf]
eager_attention_forward modeling_t5gemma.py:199-230).

* t5g_eager_attention (csrc/eager.hip) == oracle.cpu_order.eager_attention -- the CPU
  restatement pinned bitwise on the reference's own eager run (tests/test_cpu_order_cpu.py)
  -- over decode, prefill, cross and encoder call shapes, including the regime edges of the
  measured matmul selection (1, 2, 3 keys; pair chain below 64 keys; the E/O chunks above).
* The engine in parity mode on an eager 2b-2b checkpoint reproduces golden_2b2b_eager (the
  reference's 26+26-layer eager run, tests/golden/make_golden.py --only eager2b): tokens and
  every logit row, each case alone and the three in one batch."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _st():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("Tq,Tk,causal,qscale", [
    (1, 1, 1, 1.0), (1, 2, 1, 1.0), (1, 3, 1, 1.0), (1, 15, 1, 1.0), (1, 17, 1, 1.0), (1, 60, 0, 1.0),
    (1, 63, 1, 1.0), (1, 64, 1, 1.0), (1, 65, 1, 1.0), (1, 152, 1, 4.0), (1, 527, 1, 1.0), (1, 903, 1, 4.0),
    (6, 6, 1, 1.0), (7, 7, 1, 1.0), (6, 7, 0, 1.0), (16, 16, 1, 4.0), (60, 60, 0, 1.0), (152, 152, 1, 1.0),
    (152, 60, 0, 4.0),
])
def test_eager_attention_bitwise_vs_oracle(Tq, Tk, causal, qscale):
    _need_gpu()
    from oracle import cpu_order
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    Hq, Hkv, D = 8, 4, 256
    cap = max(Tk, 64)
    g = torch.Generator().manual_seed(Tq * 1009 + Tk * 31 + causal)
    q = (torch.randn(Tq, Hq, D, generator=g) * qscale).to(BF16)
    kc = torch.randn(1, Hkv, cap, D, generator=g).to(BF16)
    vc = torch.randn(1, Hkv, cap, D, generator=g).to(BF16)
    dev = "cuda"
    i32 = dict(dtype=torch.int32, device=dev)
    kv_len = torch.tensor([Tk], **i32)
    lut = torch.from_numpy(np.frombuffer(bytes(_lib.tanh_table()), dtype=np.int16).copy()).to(dev)
    qd, kd, vd = q.reshape(Tq, Hq * D).to(dev), kc.to(dev), vc.to(dev)
    o = torch.zeros(Tq, Hq * D, dtype=BF16, device=dev)
    if Tq == 1:
        q_row = q_pos = q_len = None
    else:
        q_row = torch.zeros(Tq, **i32)
        q_pos = torch.arange(Tq, **i32)
        q_len = torch.tensor([Tq], **i32)
    p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
    rc = L.t5g_eager_attention(C.c_void_p(qd.data_ptr()), Tq, p(q_row), p(q_pos), p(q_len), C.c_void_p(kd.data_ptr()),
                               C.c_void_p(vd.data_ptr()), cap, C.c_void_p(kv_len.data_ptr()), Hq, Hkv, D, causal, 0,
                               1.0 / 16, 50.0, C.c_void_p(lut.data_ptr()), C.c_void_p(o.data_ptr()), _st())
    assert rc == 0
    torch.cuda.synchronize()
    got = o.cpu().view(Tq, Hq, D).transpose(0, 1)
    k = kc[0, :, :Tk].repeat_interleave(Hq // Hkv, 0)
    v = vc[0, :, :Tk].repeat_interleave(Hq // Hkv, 0)
    mask = (torch.arange(Tq)[:, None] + (Tk - Tq) >= torch.arange(Tk)[None, :]) if (causal and Tq > 1) else None
    ref = cpu_order.eager_attention(q.transpose(0, 1), k, v, 1.0 / 16, 50.0, mask)
    bad = (got.view(torch.int16) != ref.view(torch.int16))
    assert not bad.any(), f"{int(bad.sum())} of {bad.numel()} outputs differ"


@pytest.fixture(scope="module")
def eager_engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine
    from t5gemma_tts_amd.weights import state_dict_digest, synthetic_weights
    with open(os.path.join(GOLDEN, "golden_2b2b_eager.json")) as f:
        meta = json.load(f)
    cfg = named_config(meta["config"], **meta["config_kw"])
    assert cfg.backbone.softcap == 50.0
    sd = synthetic_weights(cfg, meta["weight_seed"])
    assert state_dict_digest(sd) == meta["weight_sha256"]
    c0 = meta["cases"][0]
    p = SamplingParams(top_k=c0["top_k"], top_p=c0["top_p"], min_p=c0["min_p"], temperature=c0["temperature"],
                       stop_repetition=c0["stop_repetition"])
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=len(meta["cases"]), max_text=64, max_audio=1024,
                           max_gen=200)
    return meta, p, eng


def test_eager_golden_exact(eager_engine):
    """Parity mode on the eager 2b-2b checkpoint == the reference's own eager runs."""
    from t5gemma_tts_amd.engine import Utterance
    meta, p, eng = eager_engine
    cases = meta["cases"]
    report = {}
    for sel in ([0], [1], [2], [0, 1, 2]):
        utts = [Utterance(x=cases[i]["x"], y=cases[i]["y"], tgt_y_len=cases[i]["tgt"]) for i in sel]
        out = eng.generate(utts, p, seeds=[cases[i]["seed"] for i in sel], parity=True, record_logits=True)
        for slot, i in enumerate(sel):
            c = cases[i]
            n = len(c["gen"])
            shas = [hashlib.sha256(lg[slot].cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]
                    for lg in out["logits"][:n]]
            eq = [a == b for a, b in zip(shas, c["logit_sha"])]
            report[f"{sel}:{i}"] = {"tokens_equal": out["gen"][slot].tolist() == c["gen"], "rows": sum(eq),
                                    "of": n, "first_bad": eq.index(False) if not all(eq) else None}
    print(json.dumps(report))
    for r in report.values():
        assert r["tokens_equal"] and r["rows"] == r["of"], report


def test_eager_fast_path(eager_engine):
    """The fast path on the eager checkpoint (the kernels apply the tanh softcap in the
    score, common.h fast_score): the persistent layer launch equals the per-op launches bit
    for bit (tokens and every logit row), and its step-0 logits stay within fast-mode
    tolerance of the parity path's, which are the reference's bits: |diff| <= 3 % of
    max |logit|, >= 25 of the top-30 ids shared."""
    from t5gemma_tts_amd.engine import Utterance
    meta, p, eng = eager_engine
    cases = meta["cases"]
    utts = [Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"]) for c in cases]
    seeds = [c["seed"] for c in cases]
    runs = []
    for fused in (True, False):
        eng.set_fused(fused)
        runs.append(eng.generate(utts, p, seeds=seeds, parity=True, exact=False, record_logits=True))
    eng.set_fused(True)
    for b in range(len(cases)):
        assert runs[0]["gen"][b].tolist() == runs[1]["gen"][b].tolist(), b
    for s_, (l0, l1) in enumerate(zip(runs[0]["logits"], runs[1]["logits"])):
        assert torch.equal(l0.view(torch.int16), l1.view(torch.int16)), s_
    ex = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
    for b in range(len(cases)):
        fa, xa = runs[0]["logits"][0][b].float().cpu(), ex["logits"][0][b].float().cpu()
        assert (fa - xa).abs().max().item() <= 0.03 * xa.abs().max().item(), b
        shared = len(set(torch.topk(fa, 30).indices.tolist()) & set(torch.topk(xa, 30).indices.tolist()))
        assert shared >= 25, (b, shared)


def test_eager_long_prompt_golden_exact(eager_engine):
    """A 601-code prompt (a 602-token eager prefill: q.k^T / P.V at 602 x 602, E/O-32 with
    no K split) then 16 decode steps == the reference's own eager run
    (golden_2b2b_eager_long), alone and as row 1 of a batch with a short eager row."""
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    meta, p, _ = eager_engine
    with open(os.path.join(GOLDEN, "golden_2b2b_eager_long.json")) as f:
        lm = json.load(f)
    assert lm["weight_sha256"] == meta["weight_sha256"] and lm["config_kw"]["attn_implementation"] == "eager"
    cfg = named_config(lm["config"], **lm["config_kw"])   # its own generation budget
    eng = T5GemmaTTSEngine(cfg, synthetic_weights(cfg, lm["weight_seed"]), device="cuda:0", max_batch=2,
                           max_text=64, max_audio=1024, max_gen=200)
    c = lm["cases"][0]
    short = meta["cases"][1]
    for utts, seeds, slot in (([Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], [c["seed"]], 0),
                              ([Utterance(x=short["x"], y=short["y"], tgt_y_len=short["tgt"]),
                                Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], [short["seed"], c["seed"]], 1)):
        out = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
        n = len(c["gen"])
        shas = [hashlib.sha256(lg[slot].cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]
                for lg in out["logits"][:n]]
        assert out["gen"][slot].tolist() == c["gen"], slot
        assert shas == c["logit_sha"], (slot, sum(a == b for a, b in zip(shas, c["logit_sha"])))
