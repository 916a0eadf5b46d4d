"""GPU parity: libt5gtts.so kernels / engine vs the CPU oracle and the reference's
golden vectors. Run on an MI355X (``pytest -m gpu``)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu

BF16 = torch.bfloat16


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    npz = os.path.join(GOLDEN, name + ".npz")
    return meta, (dict(np.load(npz)) if os.path.exists(npz) else {})


def _bf16_from_bits(a):
    return torch.from_numpy(a.astype(np.int16)).view(BF16)


# --------------------------------------------------------------------------- GEMM
PREFILL = 0x100   # include/t5gtts.h T5G_GEMM_PREFILL: the encoder / prefill kernel


@pytest.mark.parametrize("M,N,K,epi,splits", [
    (1, 4096, 2304, 0, 1), (8, 4096, 2304, 0, 1), (8, 2304, 2048, 4, 4), (16, 2304, 9216, 4, 8),
    # 17..32 rows, K = 2304 k-sliced: X staged in LDS and shared by 2 row groups (gemm_dx_kernel)
    (32, 4096, 2304, 4, 2), (20, 2048, 2304, 4, 4), (32, 2304, 9216, 4, 8),
    (8, 18432, 2304, 3, 1), (8, 2304, 2304, 2, 1), (8, 65541, 2304, 1, 1), (40, 4096, 2304, 0, 1),
    (200, 2304, 2048, 0, 1), (300, 18432, 2304, 3, 1), (5, 300, 128, 0, 1),
    # many-token kernel: encoder (B*T_x) / prefill (B*(T_p+1)) shapes, ragged tails, tiny widths
    (1216, 4096, 2304, PREFILL, 1), (480, 18432, 2304, 3 | PREFILL, 1), (300, 2304, 9216, PREFILL, 1),
    (37, 300, 128, 1 | PREFILL, 1), (130, 2304, 2304, 2 | PREFILL, 1), (5, 200, 96, PREFILL, 1),
])
def test_gemm_p16_vs_fp32(M, N, K, epi, splits):
    _need_gpu()
    flags, epi = epi & ~0xff, epi & 0xff
    import ctypes as C
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    X = (torch.randn(M, K, generator=g)).to(BF16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    bias = (torch.randn(N, generator=g) * 0.02).to(BF16)
    dev = "cuda"
    Xd, Wd, bd = X.to(dev), W.to(dev), bias.to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(Wd.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
    n_out = N // 2 if epi == 3 else N
    if epi == 4:
        Y = torch.zeros(splits, M, N, dtype=torch.float32, device=dev)
    else:
        Y = torch.zeros(M, n_out, dtype=BF16, device=dev)
    rc = L.t5g_gemm(C.c_void_p(Xd.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, splits,
                    C.c_void_p(bd.data_ptr()), C.c_void_p(Y.data_ptr()), Y.shape[-1], epi | flags, st)
    assert rc == 0
    torch.cuda.synchronize()
    # exact (fp64) products and sums: the kernel must land within rounding of this
    acc64 = X.double() @ W.double().t()
    acc = acc64.float()
    if epi == 4:
        got = Y.sum(0).cpu()
        assert torch.allclose(got, acc, rtol=1e-5, atol=1e-3 * acc.abs().max().item())
        return
    got = Y.float().cpu()
    if epi == 0:
        ref = acc64.to(BF16).float()
    elif epi == 1:
        ref = (acc64 + bias.double()).to(BF16).float()
    elif epi == 2:
        ref = torch.nn.functional.gelu((acc64 + bias.double()).to(BF16).float()).to(BF16).float()
    else:  # GeGLU over interleaved 8-row groups (gate, up, gate, up, ...)
        a3 = acc.view(M, N // 16, 2, 8)
        gate, up = a3[:, :, 0].reshape(M, -1), a3[:, :, 1].reshape(M, -1)
        act = torch.nn.functional.gelu(gate.to(BF16).float(), approximate="tanh").to(BF16).float()
        ref = (act * up.to(BF16).float()).to(BF16).float()
    # Against the exact value the kernel's fp32 sum rounds to bf16 correctly except where
    # the exact value sits on a bf16 rounding tie (bf16 x bf16 products make ties common)
    # and the fp32 sum lands on its other side: <= 1 spacing (at the larger magnitude of
    # the pair). Bias+GELU rounds twice (pre-activation, slope <= 1.13, then output): <= 4.
    # GeGLU chains three roundings, so a flipped gate/up ulp can move the output a few
    # ulps. Outputs near zero come from cancelling sums, where the fp32 accumulation error
    # (~2^-24 sqrt(K) sum_k |x_k w_k|) exceeds the bf16 spacing: added as an absolute floor.
    diff = (got - ref).abs()
    mag = torch.maximum(got.abs(), ref.abs()).clamp(min=2.0 ** -126)
    ulp = torch.exp2(torch.floor(torch.log2(mag)) - 7)
    if epi == 3:
        assert diff.max() <= 2 ** -6 * ref.abs().max(), diff.max()
    else:
        k = 4.0 if epi == 2 else 1.0
        floor32 = 2.0 ** -24 * K ** 0.5 * (X.float().abs() @ W.float().abs().t())
        bad = diff > ulp * k * 1.01 + floor32 + 1e-7
        assert not bad.any(), (int(bad.sum()), diff[bad].max(), ref[bad][:4], got[bad][:4])
    assert (diff == 0).float().mean() > 0.97


def test_gemm_decode_rows_bitwise_across_kernels():
    """The 17..32-row decode GEMM (X staged in LDS, gemm_dx_kernel) keeps the k-slice order
    of the 1..16-row kernel: rows 0..7 of a 32-row launch equal an 8-row launch bitwise."""
    _need_gpu()
    import ctypes as C
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    for N, K, splits in ((4096, 2304, 2), (2048, 2304, 4)):
        g = torch.Generator(device="cpu").manual_seed(N + splits)
        X = torch.randn(32, K, generator=g).to(BF16).cuda()
        W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).cuda()
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device="cuda")
        assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
        outs = []
        for M in (32, 8):
            Y = torch.zeros(splits, M, N, dtype=torch.float32, device="cuda")
            assert L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, splits, None,
                              C.c_void_p(Y.data_ptr()), N, 4, st) == 0
            outs.append(Y)
        torch.cuda.synchronize()
        assert torch.equal(outs[0][:, :8], outs[1])


def test_gemm_prefill_batch_invariant():
    """Many-token kernel: a token's outputs do not depend on the other tokens of the launch
    (bitwise) -- rows 37..73 of a 300-token launch equal the same rows launched alone."""
    _need_gpu()
    import ctypes as C
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    M, N, K = 300, 18432, 2304
    g = torch.Generator(device="cpu").manual_seed(11)
    dev = "cuda"
    X = torch.randn(M, K, generator=g).to(BF16).to(dev)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).to(dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0

    def run(x):
        Y = torch.zeros(x.shape[0], N // 2, dtype=BF16, device=dev)
        assert L.t5g_gemm(C.c_void_p(x.data_ptr()), K, x.shape[0], C.c_void_p(Wp.data_ptr()), N, K, 1, None,
                          C.c_void_p(Y.data_ptr()), N // 2, 3 | PREFILL, st) == 0
        torch.cuda.synchronize()
        return Y.cpu()

    full = run(X)
    part = run(X[37:74].contiguous())
    assert torch.equal(full[37:74], part)


# --------------------------------------------------------------------------- engine
def _engine(cfg, sd, **kw):
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    return T5GemmaTTSEngine(cfg, sd, device="cuda:0", **kw)


def _params(c):
    from t5gemma_tts_amd.engine import SamplingParams
    return SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                          stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))


def teacher_forced_check(cfg, sd, utt, params_o, seed, gpu_out, rtol):
    """Replay the GPU's token sequence through the CPU oracle. At every step:
    (a) the reference sampler fed the GPU's logits + the same noise returns the GPU's
        token (sampler exactness, incl. tie order and stop rules);
    (b) the GPU logits match the oracle logits under the identical history
        (bf16 GEMM accumulation order => within a few bf16 ulps, rtol of max |logit|).
    Returns (max relative logit error, number of exactly equal logit rows)."""
    import copy
    from oracle.t5g_oracle import T5GemmaTTSOracle, draw_noise, sample_helper
    orc = T5GemmaTTSOracle(cfg, sd)
    ctx = orc.prepare(utt.x, utt.y, utt.tgt_y_len)
    st = ctx["state"]
    gen = torch.Generator().manual_seed(int(seed))
    toks = gpu_out["gen"][0].tolist()
    worst, exact_rows = 0.0, 0
    for t, tok in enumerate(toks):
        lo = orc.step_logits(ctx)
        lg = gpu_out["logits"][t][0].cpu()
        noise = draw_noise(gen, lo.shape[-1])
        scale = lo.float().abs().max().item()
        err = (lg.float() - lo.float()).abs().max().item() / max(scale, 1e-6)
        worst = max(worst, err)
        exact_rows += int(torch.equal(lg, lo))
        st_g = copy.deepcopy(st)
        tok_g, _ = sample_helper(lg.clone(), params_o, st_g, noise, eos=cfg.eog_inference,
                                 encodec_sr=cfg.encodec_sr, extra_cutoff=cfg.extra_cutoff,
                                 text_guard_frames_per_token=cfg.text_guard_frames_per_token)
        assert tok_g == tok, f"step {t}: reference sampler on GPU logits -> {tok_g}, GPU sampled {tok}"
        ctx["state"] = st = st_g
        st.cur_num_gen += 1
        st.current_length += 1
        if tok == cfg.eog_inference:
            assert t == len(toks) - 1
            break
        orc.advance(ctx, tok)
    assert worst <= rtol, worst
    return worst, exact_rows


def _oparams(c):
    from oracle.t5g_oracle import SamplerParams
    return SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                         stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))


# free-running token-exact cases each golden set must keep (measured on MI355X, see
# profiles/r02_parity_rates.json); every other case must diverge only at an explained
# sampling-boundary flip (see _explain_divergence)
# golden_tiny_eager runs the FAST kernels (parity mode restates eager attention for the
# reference model's call shape only, 8 query heads of 256 -- tests/test_gpu_eager.py): since
# round 4 their decode attention applies the softcap inside the aten-order / flash softmax
# (common.h fast_score) instead of the separate eager-rounding launch, so 2 of the 4 cases
# now flip at a sampling boundary -- each flip explained and asserted below (sampler on the
# GPU's logits picks the GPU's token, on the reference's the reference's, logits within 2 %)
MIN_EXACT = {"golden_tiny": 12, "golden_tiny_eager": 2, "golden_tiny_window": 4}
# teacher-forced max |logit error| / max |logit| allowed per golden: 2 %, and for
# the eager case -- where the token-flip count above was relaxed -- a bound just above its
# measured 1.36 % (round 4-5), so a further drift of the fast kernels' softcap path fails here
# rather than only through token flips
TF_RTOL = {"golden_tiny": 0.02, "golden_tiny_eager": 0.016, "golden_tiny_window": 0.02}


def _topk_agree(g, r, k, tol):
    gv, gi = torch.topk(g.float(), k)
    rv, ri = torch.topk(r.float(), k)
    cut = min(gv[-1].item(), rv[-1].item())
    sg = {int(i) for i, v in zip(gi, gv) if v.item() > cut + tol}
    sr = {int(i) for i, v in zip(ri, rv) if v.item() > cut + tol}
    return sg <= set(ri.tolist()) and sr <= set(gi.tolist())


def _explain_divergence(cfg, c, gpu_logits, ref_logits, t, gpu_tok, oparams):
    """First divergent step t of a free-running run (histories identical before t): the
    GPU and reference logits agree within tolerance, and the reference sampler -- fed the
    same noise and state -- returns the reference's token on the reference logits and
    the GPU's token on the GPU logits. The divergence is then a draw landing on a
    bf16-level logit difference, not a different model or sampler."""
    import copy
    from oracle.t5g_oracle import RowState, draw_noise, sample_helper
    gen = torch.Generator().manual_seed(int(c["seed"]))
    V = ref_logits.shape[-1]
    for _ in range(t + 1):
        noise = draw_noise(gen, V)
    y = c["y"]
    st = RowState(cur_num_gen=t, current_length=len(y) + 1 + t, prompt_offset=len(y) + 1, target_total=c["tgt"],
                  first_input_len=len(c["x"]))
    st.est_total = c["tgt"] + 1
    for tok in c["gen"][:t]:   # the silence-run state of the shared history (:781-786)
        st.consec_silence = st.consec_silence + 1 if (tok in c["silence_tokens"] and tok == st.prev_token) else 0
        st.prev_token = tok
    kw = dict(eos=cfg.eog_inference, encodec_sr=cfg.encodec_sr, extra_cutoff=cfg.extra_cutoff)
    tg, _ = sample_helper(gpu_logits.clone(), oparams, copy.deepcopy(st), noise, **kw)
    tr, _ = sample_helper(ref_logits.clone(), oparams, copy.deepcopy(st), noise, **kw)
    scale = ref_logits.float().abs().max().item()
    err = (gpu_logits.float() - ref_logits.float()).abs().max().item() / scale
    ok = tg == gpu_tok and tr == c["gen"][t] and err <= 0.02
    return ok, {"step": t, "gpu_token": gpu_tok, "ref_token": c["gen"][t], "sampler_on_gpu_logits": tg,
                "sampler_on_ref_logits": tr, "rel_err": err}


@pytest.mark.parametrize("name", ["golden_tiny", "golden_tiny_eager", "golden_tiny_window"])
def test_tiny_engine_vs_reference_golden(name):
    """Parity mode on the reference's golden cases (SURVEY §7 acceptance criteria):
    (a) teacher-forced, the reference sampler on the GPU's logits returns the GPU's token
        at every step, and the logits stay within 2 % of max |logit| of the oracle's;
    (b) per-step top-k candidate sets agree with the reference's (ties within tolerance);
    (c) free-running token equality with the reference on >= MIN_EXACT[name] cases, and
        every other case diverges only at an explained sampling-boundary flip."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    if not os.path.exists(os.path.join(GOLDEN, name + ".json")):
        pytest.skip("fixture missing")
    meta, arrs = _load(name)
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = _engine(cfg, sd, max_batch=8, max_text=64, max_audio=256, max_gen=200)
    exact_tokens, worst, rows_exact, rows, topk_ok, topk_n = 0, 0.0, 0, 0, 0, 0
    divergences = []
    for ci, c in enumerate(meta["cases"]):
        u = Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])
        # the tiny eager (softcap) configuration: the reference RNG and sampler with the fast
        # kernels (parity mode restates eager attention for the 2b-2b call shape only)
        out = eng.generate([u], _params(c), seeds=[c["seed"]], parity=True, record_logits=True,
                           exact=False if name == "golden_tiny_eager" else None)
        w, ex = teacher_forced_check(cfg, sd, u, _oparams(c), c["seed"], out, rtol=TF_RTOL[name])
        worst = max(worst, w)
        rows_exact += ex
        rows += len(out["gen"][0])
        g = out["gen"][0].tolist()
        ref = _bf16_from_bits(arrs[f"logits_{ci}"])
        got = [l[0].cpu() for l in out["logits"]]
        t_div = next((t for t in range(min(len(g), len(c["gen"]))) if g[t] != c["gen"][t]), None)
        if t_div is None and len(g) != len(c["gen"]):
            t_div = min(len(g), len(c["gen"]))
        n_cmp = len(g) if t_div is None else t_div + 1
        for t in range(min(n_cmp, ref.shape[0], len(got))):
            topk_n += 1
            topk_ok += int(_topk_agree(got[t], ref[t], 30, 0.02 * ref[t].float().abs().max().item()))
        if t_div is None:
            exact_tokens += 1
            assert len(got) == ref.shape[0]
        else:
            ok, info = _explain_divergence(cfg, c, got[t_div], ref[t_div], t_div, g[t_div], _oparams(c))
            info["case"] = ci
            divergences.append(info)
            assert ok, info
    rates = {"cases": len(meta["cases"]), "free_running_token_exact": exact_tokens,
             "teacher_forced_max_rel_logit_err": worst, "bit_identical_logit_rows": rows_exact, "rows": rows,
             "topk30_set_agree_steps": topk_ok, "topk_steps": topk_n, "divergences": divergences}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"parity_{name}.json"), "w") as f:
        json.dump(rates, f, indent=1)
    print(name, json.dumps(rates))
    assert topk_ok == topk_n, rates
    assert exact_tokens >= MIN_EXACT[name], rates


def test_batched_rows_equal_single_rows():
    """Row i of a batch == the same utterance run alone (tokens and logits bitwise)."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    eng = _engine(cfg, sd, max_batch=4, max_text=64, max_audio=256, max_gen=200)
    rng = np.random.default_rng(3)
    utts = []
    for b in range(4):
        x = rng.integers(3, 500, size=int(rng.integers(3, 30))).tolist()
        tp = [0, 5, 11, 2][b]
        y = rng.integers(0, 64, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(10, 40))))
    p = SamplingParams(top_k=20, top_p=0.9, temperature=0.9)
    seeds = [11, 12, 13, 14]
    batch = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
    for b in range(4):
        one = eng.generate([utts[b]], p, seeds=[seeds[b]], parity=True, record_logits=True)
        assert one["gen"][0].tolist() == batch["gen"][b].tolist(), b
        for t in range(len(one["logits"])):
            assert torch.equal(one["logits"][t][0], batch["logits"][t][b]), (b, t)


def test_batch32_rows_equal_single_rows():
    """At B = 32 (C5; decode GEMMs on the tiled kernel instead of the <= 16-row GEMV) rows
    of a 32-row batch equal the same utterances run alone (tokens bitwise), on the
    on-device sampler."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    eng = _engine(cfg, sd, max_batch=32, max_text=64, max_audio=256, max_gen=200)
    rng = np.random.default_rng(4)
    utts = []
    for b in range(32):
        x = rng.integers(3, 500, size=int(rng.integers(3, 30))).tolist()
        tp = int(rng.integers(0, 12))
        y = rng.integers(0, 64, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(10, 40))))
    p = SamplingParams(top_k=20, top_p=0.9, temperature=0.9)
    seeds = list(range(100, 132))
    batch = eng.generate(utts, p, seeds=seeds)
    for b in (0, 15, 16, 31):
        one = eng.generate([utts[b]], p, seeds=[seeds[b]])
        assert one["gen"][0].tolist() == batch["gen"][b].tolist(), b


def test_out_of_range_ids_raise_before_any_launch():
    """Text ids >= the text vocabulary and prompt codes >= the audio vocabulary raise
    IndexError (the reference's nn.Embedding does) instead of reaching the embedding
    gathers; the engine keeps working afterwards."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    eng = _engine(cfg, synthetic_weights(cfg, 7), max_batch=1, max_text=64, max_audio=256, max_gen=64)
    p = SamplingParams(top_k=20, top_p=0.9)
    with pytest.raises(IndexError):
        eng.generate([Utterance(x=[5, cfg.backbone.text_vocab_size], y=[], tgt_y_len=10)], p, seeds=[1])
    with pytest.raises(IndexError):
        eng.generate([Utterance(x=[5, 6], y=[1, 65535, 2], tgt_y_len=20)], p, seeds=[1])
    out = eng.generate([Utterance(x=[5, 6], y=[1, 2], tgt_y_len=20)], p, seeds=[1])
    assert len(out["gen"][0]) > 0


def test_graph_fast_path_matches_eager_launches():
    """hipGraph replay == plain launches (production Philox noise, same seeds)."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    eng = _engine(cfg, sd, max_batch=3, max_text=64, max_audio=256, max_gen=200)
    utts = [Utterance(x=[5, 6, 7, 8, 9], y=[], tgt_y_len=30), Utterance(x=[9, 300, 2], y=[4, 5, 68], tgt_y_len=40),
            Utterance(x=list(range(3, 40)), y=[1, 1, 1, 68], tgt_y_len=20)]
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8, silence_tokens=(1,), stop_repetition=2)
    a = eng.generate(utts, p, seeds=[1, 2, 3], use_graph=True, chunk=7)
    b = eng.generate(utts, p, seeds=[1, 2, 3], use_graph=False, chunk=5)
    for i in range(3):
        assert a["gen"][i].tolist() == b["gen"][i].tolist()
        assert a["gen"][i][-1].item() == cfg.eog_inference


def test_mid_width_teacher_forced():
    """True 2b-2b widths (d 2304, 8x256 heads, FFN 9216, V 65541), 2+2 layers: GPU vs
    CPU oracle teacher-forced, batch of 2 with a voice-clone prompt."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    meta, _ = _load("golden_mid")
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = _engine(cfg, sd, max_batch=2, max_text=64, max_audio=128, max_gen=64)
    cases = meta["cases"]
    utts = [Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"]) for c in cases]
    out = eng.generate(utts, [_params(c) for c in cases], seeds=[c["seed"] for c in cases], parity=True,
                       record_logits=True)
    n_exact = 0
    for b, c in enumerate(cases):
        one = {"gen": [out["gen"][b]], "logits": [[l[b]] for l in out["logits"]]}
        w, ex = teacher_forced_check(cfg, sd, utts[b], _oparams(c), c["seed"], one, rtol=0.02)
        n_exact += int(out["gen"][b].tolist() == c["gen"])
        print(f"mid row {b}: max rel logit err {w:.3g}, bit-identical rows {ex}/{len(out['gen'][b])}")
    print(f"mid: free-running token-exact vs reference {n_exact}/{len(cases)}")


def test_mid_width_batch32_rows_equal_single_rows():
    """True 2b-2b widths (2+2 layers), where the decode step runs the register-resident-X
    GEMVs (gate/up, down, o / cross-o, the 65 541-row head) and the 17..32-row GEMM: every
    kernel choice keeps a row's sums independent of the batch, so rows of a 32-row batch
    equal the same utterances run alone and in a batch of 8 (tokens and logits bitwise)."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import SamplingParams, Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    meta, _ = _load("golden_mid")
    cfg = named_config(meta["config"], **meta["config_kw"])
    sd = synthetic_weights(cfg, meta["weight_seed"])
    eng = _engine(cfg, sd, max_batch=32, max_text=64, max_audio=128, max_gen=48)
    rng = np.random.default_rng(5)
    utts = []
    for b in range(32):
        x = rng.integers(3, 4000, size=int(rng.integers(4, 40))).tolist()   # mid: 4 096 text ids
        tp = int(rng.integers(0, 40))
        y = rng.integers(0, 65536, size=tp).tolist() + ([cfg.y_sep_token] if tp else [])
        utts.append(Utterance(x=x, y=y, tgt_y_len=len(y) + int(rng.integers(8, 24))))
    p = SamplingParams(top_k=30, top_p=0.9, temperature=0.8)
    seeds = list(range(200, 232))
    batch = eng.generate(utts, p, seeds=seeds, parity=True, record_logits=True)
    for rows in ([0], [31], list(range(8, 16))):
        part = eng.generate([utts[b] for b in rows], p, seeds=[seeds[b] for b in rows], parity=True,
                            record_logits=True)
        for i, b in enumerate(rows):
            assert part["gen"][i].tolist() == batch["gen"][b].tolist(), b
            for t in range(min(len(part["logits"]), len(part["gen"][i]))):   # the row's own steps
                assert torch.equal(part["logits"][t][i], batch["logits"][t][b]), (b, t)


def test_sampler_kernel_vs_reference_golden():
    """On-device sampler on the reference's sampler golden cases (V = 65541)."""
    _need_gpu()
    import ctypes as C
    from tests.golden.make_golden import make_sampler_logits
    from t5gemma_tts_amd import _lib
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import reference_noise
    from t5gemma_tts_amd.weights import synthetic_weights
    meta, _ = _load("golden_sampler")
    cfg = named_config("tiny")
    cfg.audio_vocab_size = 65536
    cfg.empty_token, cfg.eog, cfg.audio_pad_token, cfg.eos, cfg.y_sep_token = 65536, 65537, 65538, 65539, 65540
    sd = synthetic_weights(cfg, 3)
    eng = _engine(cfg, sd, max_batch=1, max_text=16, max_audio=256, max_gen=128)
    L = eng.L
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ok = amb = stalled = 0
    for c in meta["cases"]:
        V = c["V"]
        logits = make_sampler_logits(c["logit_seed"], V, c["scale"], c["quant"])
        # the kernel reads noise[row][cur_num_gen]: put the draw at step 100 (clear of the EOS guard)
        noise = torch.ones(1, 101, V, dtype=BF16)
        noise[0, 100] = reference_noise(c["noise_seed"], 1, V)[0]
        noise = noise.to("cuda")
        row = _lib.SamplerRow(top_k=c["top_k"], top_k_list_len=0, top_k_list_off=0, top_p=c["top_p"],
                              min_p=c["min_p"], temperature=c["temperature"], stop_repetition=0, n_silence=0,
                              silence_off=0, eos_disabled=0, seed_lo=0, seed_hi=0)
        # state far from every stop rule: the sampled token is the multinomial draw itself
        state = _lib.SamplerState(cur_num_gen=100, current_length=200, prompt_offset=1, target_total=-1,
                                  est_total=1000, prev_token=-1, consec_silence=0, first_input_len=5, done=0,
                                  ambiguous_steps=0, last_token=-1, next_pos=0.0)
        tk = (C.c_int32 * 1)()
        assert L.t5g_sampler_setup(eng.h, 1, C.byref(row), C.byref(state), tk, 0, tk, 0,
                                   C.c_void_p(noise.data_ptr()), 101, st) == 0
        lg = torch.zeros(1, V + 16, dtype=BF16, device="cuda")
        lg[0, :V] = logits.to("cuda")
        assert L.t5g_sample_only(eng.h, 1, C.c_void_p(lg.data_ptr()), V + 16, st) == 0
        out = (_lib.SamplerState * 1)()
        assert L.t5g_read_state(eng.h, out, 1, st) == 0
        flags = (C.c_int32 * 1)()
        L.t5g_read_flags(eng.h, flags, 1, st)
        tok = out[0].last_token
        amb += flags[0] & 1
        if flags[0] & 4:
            # a tie order the device does not reproduce: the row stalled for the host
            stalled += 1
            hs = _lib.SamplerState()
            ht = C.c_int32()
            lg_h = logits.contiguous()
            nz_h = noise[0, 100].cpu().contiguous()
            assert L.t5g_host_sample(C.c_void_p(lg_h.data_ptr()), V, C.byref(row), tk, tk, C.byref(state),
                                     C.c_void_p(nz_h.data_ptr()), cfg.eos, 10, 250.0, 0, 2000.0, 128, 4096,
                                     C.byref(hs), C.byref(ht)) == 0
            tok = ht.value
        if tok == c["token"]:
            ok += 1
        else:
            print("mismatch", {k: c[k] for k in ("logit_seed", "top_k", "top_p", "min_p", "temperature")},
                  tok, c["token"])
    print(f"sampler: {ok}/{len(meta['cases'])} exact, {amb} top-p cuts inside a tie group, {stalled} of them "
          "resolved on the host")
    assert ok == len(meta["cases"])


@pytest.mark.parametrize("max_audio,max_gen", [(96, 40), (40, 96)])
def test_generate_without_target_length(max_audio, max_gen):
    """tgt_y_lens=None (the reference accepts it, modeling_t5gemma_voice.py:624-660: no time
    budget, decoder progress over a 2 s lookahead) on a default-sized engine: generation
    stops at EOS or at the engine's capacity, and every step the reference sampler would
    also have taken is teacher-forced exact (this path used to raise). The second
    case makes the cache capacity (max_audio - prompt) the cap, so the forced-EOS step samples
    at cur_num_gen == budget: the parity noise buffer holds budget + 1 steps."""
    _need_gpu()
    from t5gemma_tts_amd.config import named_config
    from t5gemma_tts_amd.engine import Utterance
    from t5gemma_tts_amd.weights import synthetic_weights
    cfg = named_config("tiny")
    sd = synthetic_weights(cfg, 7)
    eng = _engine(cfg, sd, max_batch=2, max_text=32, max_audio=max_audio, max_gen=max_gen)
    cap = min(max_gen, max_audio - 3)
    c = {"top_k": 30, "top_p": 0.9, "min_p": 0.0, "temperature": 0.8, "stop_repetition": 3, "silence_tokens": []}
    u = Utterance(x=[5, 17, 301, 44, 9], y=[3, 60, cfg.y_sep_token], tgt_y_len=None)
    out = eng.generate([u], _params(c), seeds=[11], parity=True, record_logits=True)
    g = out["gen"][0].tolist()
    assert 1 <= len(g) <= cap + 1
    if g[-1] == cfg.eog_inference and len(g) >= cap:   # capacity stop: the last EOS is the engine's
        out = {"gen": [out["gen"][0][:-1]], "logits": out["logits"][:-1]}
    teacher_forced_check(cfg, sd, u, _oparams(c), 11, out, rtol=0.02)
