"""GPU parity: libt5gtts.so kernels / engine vs the CPU oracle and the reference's
golden vectors. Run on an MI355X (``pytest -m gpu``)."""
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


def _load(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    npz = os.path.join(GOLDEN, name + ".npz")
    return meta, (dict(np.load(npz)) if os.path.exists(npz) else {})


def _bf16_from_bits(a):
    return torch.from_numpy(a.astype(np.int16)).view(BF16)


# --------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K,epi,splits", [
    (1, 4096, 2304, 0, 1), (8, 4096, 2304, 0, 1), (8, 2304, 2048, 4, 4), (16, 2304, 9216, 4, 8),
    (8, 18432, 2304, 3, 1), (8, 2304, 2304, 2, 1), (8, 65541, 2304, 1, 1), (40, 4096, 2304, 0, 1),
    (200, 2304, 2048, 0, 1), (300, 18432, 2304, 3, 1), (5, 300, 128, 0, 1),
])
def test_gemm_p16_vs_fp32(M, N, K, epi, splits):
    _need_gpu()
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
                    C.c_void_p(bd.data_ptr()), C.c_void_p(Y.data_ptr()), Y.shape[-1], epi, st)
    assert rc == 0
    torch.cuda.synchronize()
    acc = X.float() @ W.float().t()
    if epi == 4:
        got = Y.sum(0).cpu()
        assert torch.allclose(got, acc, rtol=1e-5, atol=1e-3 * acc.abs().max().item())
        return
    got = Y.float().cpu()
    if epi == 0:
        ref = acc.to(BF16).float()
    elif epi == 1:
        ref = (acc + bias.float()).to(BF16).float()
    elif epi == 2:
        ref = torch.nn.functional.gelu((acc + bias.float()).to(BF16).float()).to(BF16).float()
    else:  # GeGLU over interleaved 16-row groups (gate, up, gate, up, ...)
        a3 = acc.view(M, N // 32, 2, 16)
        gate, up = a3[:, :, 0].reshape(M, -1), a3[:, :, 1].reshape(M, -1)
        act = torch.nn.functional.gelu(gate.to(BF16).float(), approximate="tanh").to(BF16).float()
        ref = (act * up.to(BF16).float()).to(BF16).float()
    # fp32 accumulation-order differences may flip a bf16 rounding: <= 1 ulp, rare
    diff = (got - ref).abs()
    ulp = ref.abs().clamp(min=1e-30) * 2 ** -7
    assert (diff <= ulp * 1.01 + 1e-6).all(), diff.max()
    assert (diff == 0).float().mean() > 0.97


# --------------------------------------------------------------------------- engine
def _engine(cfg, sd, **kw):
    from t5gemma_tts_amd.engine import T5GemmaTTSEngine
    return T5GemmaTTSEngine(cfg, sd, device="cuda:0", **kw)


def _params(c):
    from t5gemma_tts_amd.engine import SamplingParams
    return SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                          stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))


@pytest.mark.parametrize("name", ["golden_tiny", "golden_tiny_eager", "golden_tiny_window"])
def test_tiny_engine_vs_reference_golden(name):
    """Free-running parity mode vs the reference's own token ids; per-step logits vs
    the reference logits within bf16 rounding."""
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
    exact_tokens = 0
    worst = 0.0
    for ci, c in enumerate(meta["cases"]):
        out = eng.generate([Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])], _params(c),
                           seeds=[c["seed"]], parity=True, record_logits=True)
        ref = _bf16_from_bits(arrs[f"logits_{ci}"]).float()
        got = torch.stack([l[0].float().cpu() for l in out["logits"]])
        n = min(len(ref), len(got))
        d = (got[:n] - ref[:n]).abs().max().item()
        worst = max(worst, d)
        if out["gen"][0].tolist() == c["gen"]:
            exact_tokens += 1
        else:
            # a divergence must be explained by a near-tie in the logits at the first differing step
            g, r = out["gen"][0].tolist(), c["gen"]
            k = next(i for i in range(min(len(g), len(r))) if g[i] != r[i]) if any(
                a != b for a, b in zip(g, r)) else min(len(g), len(r))
            print(f"case {ci}: diverged at step {k}")
    print(f"{name}: {exact_tokens}/{len(meta['cases'])} token-exact, max |logit diff| {worst:.4g}")
    assert worst < 0.05
    assert exact_tokens >= len(meta["cases"]) - 1


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
    ok = amb = 0
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
        if flags[0] & 1:
            # tie group straddles the top-p cut: parity mode resolves it on the host
            amb += 1
            hs = _lib.SamplerState()
            ht = C.c_int32()
            lg_h = logits.contiguous()
            nz_h = noise[0, 100].cpu().contiguous()
            assert L.t5g_host_sample(C.c_void_p(lg_h.data_ptr()), V, C.byref(row), tk, tk, C.byref(state),
                                     C.c_void_p(nz_h.data_ptr()), cfg.eos, 10, 250.0, 0, 2000.0, 128,
                                     C.byref(hs), C.byref(ht)) == 0
            tok = ht.value
        if tok == c["token"]:
            ok += 1
        else:
            print("mismatch", {k: c[k] for k in ("logit_seed", "top_k", "top_p", "min_p", "temperature")},
                  tok, c["token"])
    print(f"sampler: {ok}/{len(meta['cases'])} exact, {amb} ambiguous")
    assert ok == len(meta["cases"])
