"""GPU debug probe for the exact-order kernels: saves outputs for CPU-side analysis."""
import ctypes as C, json, os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import t5gemma_tts_amd  # noqa
from t5gemma_tts_amd import _lib
BF16 = torch.bfloat16
out = {}
L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
# 1) attention (1, 903) and (60, 60)
for Tq, Tk, causal, window in [(1, 903, 1, 0), (60, 60, 0, 0)]:
    Hq, Hkv, D, cap = 8, 4, 256, max(Tk, 64)
    g = torch.Generator().manual_seed(Tq * 1000 + Tk + window)
    q = torch.randn(Tq, Hq, D, generator=g).to(BF16)
    k = torch.randn(Hkv, Tk, D, generator=g).to(BF16)
    v = torch.randn(Hkv, Tk, D, generator=g).to(BF16)
    kc = torch.zeros(1, Hkv, cap, D, dtype=BF16); vc = torch.zeros(1, Hkv, cap, D, dtype=BF16)
    kc[0, :, :Tk], vc[0, :, :Tk] = k, v
    qd, kd, vd = q.reshape(Tq, Hq * D).cuda(), kc.cuda(), vc.cuda()
    i32 = dict(dtype=torch.int32, device="cuda")
    q_row = torch.zeros(Tq, **i32); q_pos = torch.arange(Tq, **i32)
    q_len = torch.tensor([Tq], **i32); kv_len = torch.tensor([Tk], **i32)
    o = torch.zeros(Tq, Hq * D, dtype=BF16, device="cuda")
    rc = L.t5g_exact_attention(C.c_void_p(qd.data_ptr()), Tq, C.c_void_p(q_row.data_ptr()), C.c_void_p(q_pos.data_ptr()),
                               C.c_void_p(q_len.data_ptr()), C.c_void_p(kd.data_ptr()), C.c_void_p(vd.data_ptr()), cap,
                               C.c_void_p(kv_len.data_ptr()), Hq, Hkv, D, causal, window, 1.0 / 16, 8,
                               C.c_void_p(o.data_ptr()), st)
    torch.cuda.synchronize()
    np.save(os.path.join(REPO, "gpurun_out", f"dbg_attn_{Tq}_{Tk}.npy"), o.cpu().view(torch.int16).numpy())
# 2) tiny golden case 0, step-0 logits: exact, fast, host oracle with cpu_order
from t5gemma_tts_amd.config import named_config
from t5gemma_tts_amd.engine import SamplingParams, T5GemmaTTSEngine, Utterance
from t5gemma_tts_amd.weights import synthetic_weights
meta = json.load(open(os.path.join(REPO, "tests/golden/golden_tiny.json")))
Z = np.load(os.path.join(REPO, "tests/golden/golden_tiny.npz"))
cfg = named_config(meta["config"], **meta["config_kw"]); sd = synthetic_weights(cfg, meta["weight_seed"])
eng = T5GemmaTTSEngine(cfg, sd, device="cuda:0", max_batch=1, max_text=64, max_audio=256, max_gen=200)
c = meta["cases"][0]
u = Utterance(x=c["x"], y=c["y"], tgt_y_len=c["tgt"])
p = SamplingParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"], temperature=c["temperature"],
                   stop_repetition=c["stop_repetition"], silence_tokens=tuple(c["silence_tokens"]))
for mode in (True, False):
    r = eng.generate([u], p, seeds=[c["seed"]], parity=True, record_logits=True, exact=mode)
    lg = r["logits"][0][0].float().cpu()
    ref = torch.from_numpy(Z["logits_0"][0].astype(np.int16)).view(BF16).float()
    print("exact" if mode else "fast", "step0 max|diff|", float((lg - ref).abs().max()), "max|ref|", float(ref.abs().max()),
          "equal frac", float((lg == ref).float().mean()), "tokens equal", r["gen"][0].tolist() == c["gen"], flush=True)
import oracle.t5g_oracle as O
from oracle import cpu_order
cpu_order.install(O)
torch.set_num_threads(16)
sdc = {k: v.cpu() for k, v in sd.items()}
orc = O.T5GemmaTTSOracle(cfg, sdc)
ro = orc.generate(c["x"], c["y"], c["tgt"], O.SamplerParams(top_k=c["top_k"], top_p=c["top_p"], min_p=c["min_p"],
                  temperature=c["temperature"], stop_repetition=c["stop_repetition"],
                  silence_tokens=tuple(c["silence_tokens"])), seed=c["seed"], record_logits=True)
lo = ro["logits"][0].float()
print("host cpu_order oracle step0 equal frac", float((lo == ref).float().mean()), "tokens equal", ro["gen"].view(-1).tolist() == c["gen"])
