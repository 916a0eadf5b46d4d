// Elementwise functions of the reference's CPU numerics, restated for the exact-order
// (parity) kernels. Host- and device-compilable: the CPU test suite builds this header
// with g++ and compares every bf16 input against torch's own CPU kernels
// (tests/test_exact_math_cpu.py), and the GPU tests run the same functions on device.
//
// torch 2.10 CPU (AVX2 kernels: aten registers no AVX-512 variant of these stubs):
// * gelu(approximate='tanh') ([tf] T5GemmaMLP, modeling_t5gemma.py:81-97 via ACT2FN
//   gelu_pytorch_tanh): x3 = (x*x)*x; inner = kBeta*(x + kKappa*x3);
//   out = (0.5*x) * (1 + tanh(inner)); tanh is Sleef_tanhf8_u10, which returns exactly
//   +-1 for |inner| > 8.664339742 (below that its result rounds like the exact tanh once
//   the output is cast to bf16: all 65,536 bf16 inputs agree).
// * gelu() (erf; predict_layer nn.GELU(), hf_export/modeling_t5gemma_voice.py:469-478):
//   for a contiguous bf16 tensor on an AVX-512 host this is oneDNN's eltwise_gelu_erf
//   (aten gelu_out_cpu -> ideep). After the bf16 cast its results equal
//   (x * (1 + erf(x*M_SQRT1_2))) * 0.5 with the exact erf on every bf16 input (overflow at
//   |x| >= 2^127 included), except that outputs below FLT_MIN come out as zero.
// * cos / sin of the fp32 RoPE angle: torch is built with MKL, so the reference's float
//   cos / sin are MKL VML's vmsCos / vmsSin (VML_HA, ~0.6 ulp, proprietary). After the
//   bf16 cast they equal the correctly rounded value except on ~2.5e-7 of the angles; the
//   exceptions over every angle this model's position formulas can produce are listed in
//   data/rope_trig_exc.bin (tools/cpu_order/make_rope_table.py, made on the reference
//   host) and looked up here (rope_trig).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef T5G_HD
#define T5G_HD __host__ __device__
#endif

#if defined(__clang__)
#define T5G_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define T5G_NO_CONTRACT
#endif

namespace t5g_exact {

T5G_HD inline float gelu_tanh(float x) {
    T5G_NO_CONTRACT
    const float kBeta = 0.7978845608028654f, kKappa = 0.044715f;
    const float x3 = (x * x) * x;
    const float inner = kBeta * (x + kKappa * x3);
    const float t = fabsf(inner) > 8.664339742f ? copysignf(1.0f, inner) : (float)tanh((double)inner);
    return (0.5f * x) * (1.0f + t);
}

T5G_HD inline float gelu_erf(float x) {
    T5G_NO_CONTRACT
    const float y = x * 0.70710678118654752f;
    const float r = (x * (1.0f + (float)erf((double)y))) * 0.5f;
    return fabsf(r) < 1.17549435e-38f ? 0.0f * r : r;
}

T5G_HD inline float rope_cos(float ang) { return (float)cos((double)ang); }
T5G_HD inline float rope_sin(float ang) { return (float)sin((double)ang); }

// bf16-rounded cos (which = 0) / sin (1) of a RoPE angle as the reference host rounds it:
// the correctly rounded value unless the angle is in the exception table exc (n sorted
// (angle bits, cos_bf16 | sin_bf16 << 16) pairs; null: none). Returned as the bf16 value
// in a float.
T5G_HD inline float rope_trig(float ang, int which, const uint32_t* exc, int n) {
    const float cr = which ? rope_sin(ang) : rope_cos(ang);
    uint32_t key;
    memcpy(&key, &ang, 4);
    int lo = 0, hi = exc ? n : 0;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (exc[2 * mid] < key) lo = mid + 1;
        else hi = mid;
    }
    uint32_t bits;
    if (exc && lo < n && exc[2 * lo] == key) {
        bits = (which ? exc[2 * lo + 1] >> 16 : exc[2 * lo + 1] & 0xFFFFu) << 16;
    } else {   // round to nearest even bf16
        uint32_t u;
        memcpy(&u, &cr, 4);
        bits = ((u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u);
    }
    float r;
    memcpy(&r, &bits, 4);
    return r;
}

}  // namespace t5g_exact
