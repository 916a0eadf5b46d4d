"""Driver for the MFMA-utilisation PMC pass (tools/gpu_r2_mfma.sh): the MFMA-bound
kernels of this build at their workload shapes -- prefill / encoder GEMM (gate/up over
1216 tokens, bf16), XCodec2 decoder (B = 32 x 500 frames, f32 MFMA), XCodec2 encoder
(10 s prompt), Whisper encoder (large-v3-turbo dims, 30 s window)."""
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    from t5gemma_tts_amd import _lib
    L = _lib.lib()
    dev = torch.device("cuda:0")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    # prefill GEMMs at the C3 decoder prefill (1216 tokens = 8 x 152) and a C5 one (4864):
    # the LDS-staged kernel (gemm_pfl_kernel, the engine's) and the register ring
    # (gemm_pf_kernel, flag 0x200) on the same operands
    for M in (1216, 4864):
        for N, K, epi in ((18432, 2304, 3), (2304, 9216, 0), (4096, 2304, 0)):
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            p = torch.empty(L.t5g_packed_bytes(N, K) // 2, dtype=torch.bfloat16, device=dev)
            _lib.check(L.t5g_pack_weight(C.c_void_p(w.data_ptr()), N, K, K, C.c_void_p(p.data_ptr()), st), "pack")
            X = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
            ldy = N // 2 if epi == 3 else N
            Y = torch.empty(M, ldy, dtype=torch.bfloat16, device=dev)
            arr = (C.c_void_p * 1)(p.data_ptr())
            for flag in (0x100, 0x300):
                us = C.c_float()
                _lib.check(L.t5g_time_gemm(C.c_void_p(X.data_ptr()), K, M, arr, 1, N, K, 1, C.c_void_p(Y.data_ptr()),
                                           ldy, epi | flag, 10, st, C.byref(us)), "prefill")
                print(f"prefill M={M} N={N} K={K} {'lds' if flag == 0x100 else 'reg'} us {us.value:.1f} "
                      f"TF/s {2 * M * N * K / us.value / 1e6:.1f}", flush=True)
            del w, p
    # XCodec2 decoder, B = 32 x 500 frames
    from t5gemma_tts_amd.codec import XCodec2Decoder, codec_16k, synthetic_codec_weights
    cfg = codec_16k()
    codec = XCodec2Decoder(cfg, synthetic_codec_weights(cfg, 1), device="cuda:0", max_batch=32, max_frames=500)
    codes = torch.randint(0, 65536, (32, 500), device="cuda", dtype=torch.int32)
    for _ in range(3):
        codec.decode(codes)
    torch.cuda.synchronize()
    del codec
    # XCodec2 encoder, 10 s
    from make_golden_codec_enc import test_wave
    from t5gemma_tts_amd.codec_enc import XCodec2Encoder, encoder_16k, synthetic_encoder_weights
    ecfg = encoder_16k()
    enc = XCodec2Encoder(ecfg, synthetic_encoder_weights(ecfg, 32), device="cuda:0", max_seconds=11)
    wav = test_wave(160000, 6).cuda()
    for _ in range(3):
        enc.encode(wav)
    torch.cuda.synchronize()
    del enc
    # Whisper encoder at large-v3-turbo dims
    from t5gemma_tts_amd import whisper_asr as wa
    d = wa.dims_large_v3_turbo()
    m = wa.WhisperModel(d, wa.synthetic_weights(d, 42), device="cuda:0", max_seconds=11)
    m.log_mel(wav)
    for _ in range(3):
        m.encode(0, 1000)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
