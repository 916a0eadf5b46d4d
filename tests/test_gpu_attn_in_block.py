"""The fast path's decode self attention as stage S of the persistent layer launch
(csrc/fused.hip fb_self_attn: the flash launch's arithmetic, one 64-key chunk per 4-wave
group spread over every workgroup, the holder of a (row, kv head)'s last chunk combining, att_self handed to the o-projection
in-launch) against the same step with the attention as its own flash launch
(attn.hip attn_decode_kernel<256, 2, true, true>): tokens and every logit row bitwise equal,
at the true 2b-2b widths (2 + 2 layers), for 1-16 rows with rows of one chunk (the aten-order
single-block path), of several chunks and of partial chunk triples; on a sliding-window layer
past its window; and a call whose rows need more tasks than workgroups keeps the separate
launch (same bits). Reference: [tf] modeling_t5gemma.py:264-304 (self attention in
PMDecoderLayer, hf_export/modeling_t5gemma_voice.py:256-323)."""
import dataclasses

import numpy as np
import pytest
import torch

from conftest import GOLDEN  # noqa: F401  (sys.path set-up)

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs the MI355X")


def _engine(max_batch, max_audio, window=None):
    import json
    import os
    from conftest import GOLDEN as G
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    from t5gemma_tts_amd.weights import synthetic_weights
    meta = json.load(open(os.path.join(G, "golden_mid.json")))
    cfg = named_config(meta["config"], **meta["config_kw"])
    if window is not None:
        cfg = dataclasses.replace(cfg, backbone=dataclasses.replace(cfg.backbone, sliding_window=window))
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=max_batch, max_text=64, max_audio=max_audio,
                           max_gen=40)
    return cfg, eng


def _utts(cfg, n, seed, tp_max):
    from t5gemma_tts_amd.engine import Utterance
    rng = np.random.default_rng(seed)
    utts = []
    for i in range(n):
        x = rng.integers(3, 4000, size=int(rng.integers(4, 40))).tolist()
        tp = 0 if i == 0 else int(rng.integers(0, tp_max))   # row 0: one-chunk rows throughout
        y = rng.integers(0, 65536, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(8, 30))))
    return utts


def _run(eng, utts, p, seeds, on):
    eng.set_attn_in_block(on)   # 0 the separate flash launch, 1 stage S in front, 2 at the end
    before = eng.attn_in_block_launches()
    # host loop (every step's logits) and the graph-replayed on-device loop (tokens)
    out = eng.generate(utts, p, seeds=seeds, parity=True, exact=False, record_logits=True)
    fast = eng.generate(utts, p, seeds=seeds)
    return out, fast, eng.attn_in_block_launches() - before


def _assert_same(a, b, B, tag):
    for r in range(B):
        assert a["gen"][r].tolist() == b["gen"][r].tolist(), (tag, r)
    if "logits" not in a:   # the graph-replayed loop: tokens only
        return
    assert len(a["logits"]) == len(b["logits"]), tag
    for s, (la, lb) in enumerate(zip(a["logits"], b["logits"])):
        assert torch.equal(la.view(torch.int16), lb.view(torch.int16)), (tag, s)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("B,tp_max", [(1, 1), (3, 300), (8, 400), (16, 300)])
def test_attention_in_block_bitwise_equal_to_flash_launch(B, tp_max, mode):
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _engine(16, 448)
    utts = _utts(cfg, B, 60 + B, tp_max)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(900, 900 + B))
    on0, fon0, n_on0 = _run(eng, utts, p, seeds, mode)
    assert eng.attn_in_block_mode() == mode   # short rows: each mode takes its own placement
    off, foff, n_off = _run(eng, utts, p, seeds, 0)
    on1, fon1, n_on1 = _run(eng, utts, p, seeds, mode)
    assert n_off == 0 and n_on0 > 0 and n_on1 > 0   # stage S ran, and only when enabled
    _assert_same(on0, off, B, "on/off")
    _assert_same(on0, on1, B, "on/on")
    _assert_same(fon0, foff, B, "graph on/off")
    _assert_same(fon0, fon1, B, "graph on/on")
    assert sum(len(g) for g in on0["gen"]) > B


@pytest.mark.parametrize("mode", [1, 2])
def test_attention_in_block_sliding_window(mode):
    """Layer 0 slides over a 100-key window: rows past it start their chunks at t - 99."""
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _engine(8, 448, window=100)
    utts = _utts(cfg, 6, 17, 350)
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(6))
    on, fon, n_on = _run(eng, utts, p, seeds, mode)
    off, foff, _ = _run(eng, utts, p, seeds, 0)
    assert n_on > 0
    _assert_same(on, off, 6, "window")
    _assert_same(fon, foff, 6, "window graph")


def test_attention_in_block_falls_back_past_two_passes():
    """16 rows of up to ~1 650 keys: 16 x 4 kv heads x 26 chunks = 1 664 chunk slots > two
    passes of 3 per workgroup (1 536), so the call keeps the separate flash launch -- the same
    bits either way."""
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams
    cfg, eng = _engine(16, 1700)
    from t5gemma_tts_amd.engine import Utterance
    rng = np.random.default_rng(3)
    utts = [Utterance(x=rng.integers(3, 4000, size=20).tolist(),
                      y=rng.integers(0, 65536, size=1630).tolist() + [cfg.y_sep_token], tgt_y_len=1631 + 10)
            for _ in range(16)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(16))
    on, fon, n_on = _run(eng, utts, p, seeds, 2)
    on1, fon1, n_on1 = _run(eng, utts, p, seeds, 1)
    off, foff, _ = _run(eng, utts, p, seeds, 0)
    assert n_on == 0 and n_on1 == 0
    _assert_same(on, off, 16, "fallback")
    _assert_same(on1, off, 16, "fallback 1")
    _assert_same(fon, foff, 16, "fallback graph")


def test_tail_mode_falls_back_to_front_past_two_slots_per_worker():
    """16 rows of ~600 keys: 16 x 4 kv heads x 10 chunks = 640 > 2 slots per worker (480), so
    mode 2 runs stage S in front of each layer's o-projection (<= 3 per workgroup) -- still no
    separate attention launch, the same bits."""
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    cfg, eng = _engine(16, 640)
    rng = np.random.default_rng(4)
    utts = [Utterance(x=rng.integers(3, 4000, size=20).tolist(),
                      y=rng.integers(0, 65536, size=590).tolist() + [cfg.y_sep_token], tgt_y_len=591 + 10)
            for _ in range(16)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(16))
    on, fon, n_on = _run(eng, utts, p, seeds, 2)
    assert eng.attn_in_block_mode() == 1   # the placement the decode launches took: in front
    off, foff, _ = _run(eng, utts, p, seeds, 0)
    assert eng.attn_in_block_mode() == 0
    assert n_on > 0
    _assert_same(on, off, 16, "front fallback")
    _assert_same(fon, foff, 16, "front fallback graph")


@pytest.mark.parametrize("tp,max_audio", [(1240, 1300), (2480, 2560)])
def test_attention_in_block_long_rows(tp, max_audio):
    """Rows past 1 024 keys in the launch (round 6): 8 rows of ~1 250 keys (20 chunks: the
    combine reads its records in two batches of 16, as the flash launch does; one pass of 3
    slots per workgroup, front mode) and of ~2 500 keys (40 chunks: two passes of 3 nb slots).
    Bitwise equal to the separate flash launch, stage S in every decode launch. Reference: the
    reference serves 100 s prompts (inference_commandline_hf.py:91, 181)."""
    _need_gpu()
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    cfg, eng = _engine(8, max_audio)
    rng = np.random.default_rng(tp)
    utts = [Utterance(x=rng.integers(3, 4000, size=20).tolist(),
                      y=rng.integers(0, 65536, size=tp - 8 * i).tolist() + [cfg.y_sep_token],
                      tgt_y_len=tp - 8 * i + 1 + 12)
            for i in range(8)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(8))
    on, fon, n_on = _run(eng, utts, p, seeds, 2)
    assert eng.attn_in_block_mode() == 1   # past the tail's 2 slots per worker: front mode
    off, foff, n_off = _run(eng, utts, p, seeds, 0)
    assert n_off == 0 and n_on >= 2 * 12   # stage S ran in the decode launches
    _assert_same(on, off, 8, "long")
    _assert_same(fon, foff, 8, "long graph")
