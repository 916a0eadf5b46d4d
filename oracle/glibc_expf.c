/* expf of the reference host's C library -- TEST INFRASTRUCTURE ONLY (the checker of the
 * GPU kernels' sdpa_expf, csrc/common.h; loaded by oracle/sdpa_emu.py through ctypes).
 *
 * aten's CPU flash attention (the reference's F.scaled_dot_product_attention on bf16 CPU
 * tensors) calls std::exp on floats in two places: the running-max rescale
 * exp_tmp = exp(max_old - max_new) and the p of each kv block's tail past its 16-multiple
 * prefix. Both resolve to glibc's expf. The reference host (and this image) runs glibc 2.35
 * (Ubuntu 2.35-0ubuntu3), whose expf is the IFUNC-selected FMA variant of
 * sysdeps/ieee754/flt-32/e_expf.c: exp(x) = 2^(k/32) * 2^(r/32) with a 32-entry table
 * and a cubic in r evaluated in double with fused multiply-adds. It is not correctly rounded:
 * on (-87, 0] it differs from the correctly rounded expf on 96 956 inputs -- the round-4
 * restatement used the correctly rounded value, which broke parity at one element of a
 * 4 101-token prefill. The constants below were read out of the host's
 * libm.so.6 (.rodata of the FMA variant), and this function equals that expf on all 2^32
 * float inputs (tools/cpu_order/check_glibc_expf.c).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static const uint64_t EXPF_T[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

float oracle_glibc_expf(float x) {
    uint32_t bits;
    memcpy(&bits, &x, 4);
    const uint32_t abstop = (bits >> 20) & 0x7ff;
    const double xd = (double)x;
    if (abstop > 0x42a) {   /* |x| >= 88 */
        if (bits == 0xff800000u) return 0.0f;
        if (abstop > 0x7f7) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;
        if (x < -0x1.9fe368p6f) return 0.0f;
        if (x < -0x1.9d1d9ep6f) return 0x1p-149f;   /* __math_may_uflowf: 0x1.4p-75f squared */
    }
    const double InvLn2N = 0x1.71547652b82fep+5, SHIFT = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-20, C1 = 0x1.ebfce50fac4f3p-13, C2 = 0x1.62e42ff0c52d6p-6;
    const double z = fma(InvLn2N, xd, SHIFT);
    uint64_t ki;
    memcpy(&ki, &z, 8);
    const double kd = z - SHIFT;
    const double r = fma(InvLn2N, xd, -kd);
    const uint64_t t = EXPF_T[ki & 31] + (ki << 47);
    double s;
    memcpy(&s, &t, 8);
    const double p = fma(r, C0, C1);
    const double r2 = r * r;
    double y = fma(r, C2, 1.0);
    y = fma(p, r2, y);
    return (float)(y * s);
}

void oracle_glibc_expf_v(const float* x, float* y, long n) {
    for (long i = 0; i < n; ++i) y[i] = oracle_glibc_expf(x[i]);
}
