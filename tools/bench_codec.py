"""Time the XCodec2 decoder (xc2_decode) on the GPU at C5-like shapes and report
frames/s, real-time factor and achieved fp32 MFMA TFLOP/s. GPU only."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import t5gemma_tts_amd  # noqa: E402,F401
from t5gemma_tts_amd.codec import XCodec2Decoder, codec_16k, codec_44k, synthetic_codec_weights  # noqa: E402


def flops_per_frame(cfg, T):
    h, i, q = cfg.hidden_size, cfg.intermediate_size, cfg.quantization_dim
    lin = q * len(cfg.quantization_levels) + q * h + 7 * h * h + 8 * 3 * h * h
    lin += cfg.num_hidden_layers * (4 * h * h + 2 * h * i)
    lin += (cfg.n_fft + 2) * h + cfg.n_fft * cfg.spec_ld
    attn = cfg.num_hidden_layers * 2 * h * T      # QK^T and PV per query frame
    return 2 * (lin + attn)


def main():
    which = os.environ.get("CODEC", "16k")
    cfg = codec_16k() if which == "16k" else codec_44k()
    # SHAPES="32x751,8x500": the B x T decodes to time (default the round-1 set)
    shapes = [tuple(int(v) for v in s.split("x")) for s in os.environ.get("SHAPES", "1x500,8x500,32x500").split(",")]
    out = []
    for B, T in shapes:
        codec = XCodec2Decoder(cfg, synthetic_codec_weights(cfg, 1), device="cuda:0", max_batch=B, max_frames=T)
        codes = torch.randint(0, cfg.codebook_size, (B, T), device="cuda", dtype=torch.int32)
        wav = torch.empty(B, T * cfg.hop_length, device="cuda")
        us = C.c_float()
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = codec.L.xc2_time_decode(codec.h, C.c_void_p(codes.data_ptr()), B, T, C.c_void_p(wav.data_ptr()), 5,
                                     st, C.byref(us))
        assert rc == 0, rc
        sec = us.value * 1e-6
        fl = flops_per_frame(cfg, T) * B * T
        r = {"codec": which, "B": B, "T": T, "ms": round(us.value / 1e3, 3), "frames_per_s": round(B * T / sec, 1),
             "audio_s_per_wall_s": round(B * T / 50.0 / sec, 1), "tflops": round(fl / sec / 1e12, 2),
             "frac_f32_mfma_peak": round(fl / sec / 157.3e12, 3)}
        g_us, g_fl, g_n = C.c_float(), C.c_double(), C.c_int32()
        rc = codec.L.xc2_time_gemms(codec.h, C.c_void_p(codes.data_ptr()), B, T, C.c_void_p(wav.data_ptr()), 5,
                                    st, C.byref(g_us), C.byref(g_fl), C.byref(g_n))
        assert rc == 0, rc
        r.update({"gemm_us": round(g_us.value, 1), "gemm_launches": g_n.value, "gemm_flops": g_fl.value,
                  "gemm_tflops": round(g_fl.value / (g_us.value * 1e-6) / 1e12, 2),
                  "gemm_frac_f32_mfma_peak": round(g_fl.value / (g_us.value * 1e-6) / 157.3e12, 3)})
        print(json.dumps(r), flush=True)
        out.append(r)
        codec.close()
        del codec
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
