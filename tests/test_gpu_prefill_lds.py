"""The LDS-staged many-token GEMM (csrc/gemm.hip gemm_pfl_kernel) against the register
ring (gemm_pf_kernel): bitwise on token counts whose last tile is ragged (rows >= M are
out-of-range LDS-DMA pieces that land at once), and run to run. Round 3 saw the last token
tile's sums vary inside the engine; the cause was this wave's ds_reads of stage k - 1 still
pending at the barrier after which another wave's LDS-DMA overwrites that stage
(wait_vm_barrier now waits lgkmcnt(0) as well)."""
import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu
BF16 = torch.bfloat16
PREFILL, PREFILL_REG = 0x100, 0x200


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("M,N,K,epi", [
    (12 * 152, 4096, 2304, 0), (16 * 152, 4096, 2304, 0), (12 * 152, 18432, 2304, 3), (16 * 152, 2304, 9216, 0),
    (12 * 60, 2304, 2048, 0), (16 * 152 - 5, 2304, 2304, 2), (130, 4096, 2304, 0),
])
def test_lds_prefill_equals_register_ring(M, N, K, epi):
    _need_gpu()
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(M + N + K)
    X = torch.randn(M, K, generator=g).to(BF16).cuda()
    W = (torch.randn(N, K, generator=g) * 0.02).to(BF16).cuda()
    bias = (torch.randn(N, generator=g) * 0.1).to(BF16).cuda()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    Wp = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=BF16, device="cuda")
    assert L.t5g_pack_weight(C.c_void_p(W.data_ptr()), N, K, K, C.c_void_p(Wp.data_ptr()), st) == 0
    n_out = N // 2 if epi == 3 else N

    def run(flags):
        Y = torch.full((M, n_out), 7.0, dtype=BF16, device="cuda")
        assert L.t5g_gemm(C.c_void_p(X.data_ptr()), K, M, C.c_void_p(Wp.data_ptr()), N, K, 1,
                          C.c_void_p(bias.data_ptr()), C.c_void_p(Y.data_ptr()), n_out, epi | flags, st) == 0
        return Y

    ref = run(PREFILL | PREFILL_REG)
    outs = [run(PREFILL) for _ in range(12)]
    torch.cuda.synchronize()
    for i, o in enumerate(outs):
        bad = int((o.view(torch.int16) != ref.view(torch.int16)).sum())
        assert bad == 0, f"launch {i}: {bad} outputs differ from the register ring"
