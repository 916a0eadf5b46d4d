import ctypes as C, os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["T5G_LIB"] = os.path.join(REPO, "t5gemma-tts_amd", "lib", "libt5gtts_dbg.so")
sys.path.insert(0, REPO)
import t5gemma_tts_amd  # noqa
from t5gemma_tts_amd import _lib
BF16 = torch.bfloat16
L = _lib.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
buf = torch.zeros(64 * 8 * 4 * 4096, dtype=torch.float32, device="cuda")
L.t5g_dbg_set_exact.argtypes = [C.c_void_p]
assert L.t5g_dbg_set_exact(C.c_void_p(buf.data_ptr())) == 0
Tq, Tk, causal, window = 1, 903, 1, 0
Hq, Hkv, D, cap = 8, 4, 256, 903
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
print("rc", rc)
np.save(os.path.join(REPO, "gpurun_out", "dbg_attn_buf.npy"), buf.view(64, 8, 4, 4096)[0].cpu().numpy())
