"""Diagnose the many-token GEMM against an fp64 reference (GPU only): worst element by
|error| / (bf16 spacing + fp32 accumulation floor), for the old and the new kernel."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd import _lib  # noqa: E402

BF16 = torch.bfloat16
L = _lib.lib()
dev = "cuda"
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)


def spacing(x):
    return torch.exp2(torch.floor(torch.log2(x.abs().clamp(min=2.0 ** -126))) - 7)


for (M, N, K, epi) in [(130, 2304, 2304, 0), (130, 2304, 2304, 2), (300, 2304, 9216, 0)]:
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    X = torch.randn(M, K, generator=g).to(BF16)
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16)
    bias = (torch.randn(N, generator=g) * 0.02).to(BF16)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device=dev)
    Wd = W.to(dev)
    assert L.t5g_pack_weight(C.c_void_p(Wd.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
    exact = X.double() @ W.double().t()
    S = X.double().abs() @ W.double().abs().t()
    floor = 2.0 ** -24 * K ** 0.5 * S
    for flag in (0, 0x100):
        Y = torch.zeros(M, N, dtype=BF16, device=dev)
        Xd, bd = X.to(dev), bias.to(dev)
        assert L.t5g_gemm(C.c_void_p(Xd.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, 1,
                          C.c_void_p(bd.data_ptr()), C.c_void_p(Y.data_ptr()), N, epi | flag, st) == 0
        torch.cuda.synchronize()
        y = Y.double().cpu()
        if epi == 0:
            e = (y - exact).abs() / (spacing(exact) + floor)
            i = int(e.argmax()); r, c = divmod(i, N)
            print(f"M={M} K={K} epi={epi} {'new' if flag else 'old'}: worst {e.max():.2f} at ({r},{c}) got {y[r, c]:.6g} "
                  f"exact {exact[r, c]:.8g} floor {floor[r, c]:.3g}", flush=True)
        else:
            pre = exact + bias.double()
            # invert: compare pre-activations implied by the kernel's bf16 rounding of acc+bias
            ref = torch.nn.functional.gelu(pre.float().to(BF16).float()).double()
            d = (y - ref).abs()
            i = int(d.argmax()); r, c = divmod(i, N)
            print(f"M={M} K={K} epi={epi} {'new' if flag else 'old'}: max|d| {d.max():.4g} at ({r},{c}) got {y[r, c]:.6g} "
                  f"gelu(bf16(exact pre)) {ref[r, c]:.6g} exact pre {pre[r, c]:.8g}", flush=True)
            # worst in output spacings among moderate magnitudes
            sp = spacing(ref)
            e = d / sp
            mask = ref.abs() > 0.01
            e = torch.where(mask, e, torch.zeros_like(e))
            i = int(e.argmax()); r, c = divmod(i, N)
            print(f"     worst (|out|>0.01) {e.max():.2f} spacings at ({r},{c}) got {y[r, c]:.6g} ref {ref[r, c]:.6g} "
                  f"exact pre {pre[r, c]:.8g}")
