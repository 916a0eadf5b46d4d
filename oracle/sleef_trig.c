/* TEST INFRASTRUCTURE -- restatement of the cos / sin the reference host evaluates for
 * RoPE (torch 2.10 CPU: Tensor.cos / .sin on float32 -> Vectorized<float>::cos / sin ->
 * SLEEF Sleef_cosf16_u10 / Sleef_sinf16_u10, i.e. SLEEF's xcosf_u1 / xsinf_u1 built with
 * FMA). The reference calls them in [tf] T5GemmaRotaryEmbedding.forward
 * (hf_export/modeling_t5gemma_voice.py:516-531 builds the float PM positions, the rotary
 * embedding takes emb.cos() / emb.sin()). SLEEF is a third-party library absent from
 * /root/reference (torch links it statically); its published algorithm is restated here:
 *   |d| < 125: Cody-Waite reduction by pi (sin) / around odd multiples of pi/2 (cos) with
 *              the three-float split of pi, in float-float (double-float) arithmetic;
 *   |d| >= 125: SLEEF's Payne-Hanek rempif; here the same reduction mod pi/2 computed
 *              exactly in double (three-double split of pi/2), then SLEEF's own quadrant
 *              fix-up in float-float;
 *   then the shared odd polynomial in float-float and the sign from the quadrant.
 * Pinned against torch.sin / torch.cos of this host (tests/test_sleef_trig_cpu.py). The
 * device copy is csrc/exact_math.h (t5g_exact::rope_cos / rope_sin). */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float x, y; } df;

static inline df df_add_f_f(float x, float y) { float s = x + y; df r = {s, x - s + y}; return r; }
static inline df df_add2_f_f(float x, float y) {
    float s = x + y, v = s - x;
    df r = {s, (x - (s - v)) + (y - v)};
    return r;
}
static inline df df_add_df_f(df x, float y) { float s = x.x + y; df r = {s, x.x - s + y + x.y}; return r; }
static inline df df_add2_df_f(df x, float y) {
    float s = x.x + y, v = s - x.x;
    float t = (x.x - (s - v)) + (y - v);
    df r = {s, t + x.y};
    return r;
}
static inline df df_add_f_df(float x, df y) { float s = x + y.x; df r = {s, x - s + y.x + y.y}; return r; }
static inline df df_add2_df_df(df x, df y) {
    float s = x.x + y.x, v = s - x.x;
    float t = (x.x - (s - v)) + (y.x - v);
    df r = {s, t + (x.y + y.y)};
    return r;
}
static inline df df_mul_df_df(df x, df y) {
    float s = x.x * y.x;
    df r = {s, fmaf(x.x, y.y, fmaf(x.y, y.x, fmaf(x.x, y.x, -s)))};
    return r;
}
static inline float df_mul_f_df_df(df x, df y) { return fmaf(x.x, y.x, fmaf(x.y, y.x, x.x * y.y)); }
static inline df df_squ(df x) {
    float s = x.x * x.x;
    df r = {s, fmaf(x.x + x.x, x.y, fmaf(x.x, x.x, -s))};
    return r;
}
static inline df df_normalize(df x) { float s = x.x + x.y; df r = {s, x.x - s + x.y}; return r; }

static inline float mulsignf(float x, float y) {
    uint32_t a, b;
    memcpy(&a, &x, 4);
    memcpy(&b, &y, 4);
    a ^= b & 0x80000000u;
    memcpy(&x, &a, 4);
    return x;
}

#define PI_A2f 3.1414794921875f
#define PI_B2f 0.00011315941810607910156f
#define PI_C2f 1.9841872589410058936e-09f
#define TRIGRANGEMAX2f 125.0f

/* d = i * pi/2 + r, |r| <= pi/4, r as a normalized float-float (exact reduction in double) */
static inline void reduce_half_pi(float d, int* i, df* r) {
    const double P1 = 1.5707963267341256;       /* pi/2 split: 33 + 33 + 53 bits */
    const double P2 = 6.077100506303966e-11;
    const double P3 = 2.0222662487959506e-21;
    const double q = rint((double)d * 0.6366197723675814);
    const double t = (((double)d - q * P1) - q * P2) - q * P3;
    const float hi = (float)t;
    const float lo = (float)(t - (double)hi);
    *i = (int)q;
    r->x = hi;
    r->y = lo;
}

static inline float poly_tail(df s, df t) {
    df s2 = df_squ(s);
    float u = 2.6083159809786593541503e-06f;
    u = fmaf(u, s2.x, -0.0001981069071916863322258f);
    u = fmaf(u, s2.x, 0.00833307858556509017944336f);
    df x = df_add_f_df(1.0f, df_mul_df_df(df_add_f_f(-0.166666597127914428710938f, u * s2.x), s2));
    return df_mul_f_df_df(t, x);
}

float sleef_sinf_u1(float d) {
    int q;
    df s;
    if (fabsf(d) < TRIGRANGEMAX2f) {
        const float u = rintf(d * (float)M_1_PI);
        q = (int)u;
        const float v = fmaf(u, -PI_A2f, d);
        s = df_add2_f_f(v, u * -PI_B2f);
        s = df_add_df_f(s, u * -PI_C2f);
    } else {
        int i;
        df x;
        reduce_half_pi(d, &i, &x);
        q = ((i & 3) * 2 + (x.x > 0 ? 2 : 1)) >> 2;
        if ((i & 1) == 1) {
            df h = {mulsignf(3.1415927410125732422f * -0.5f, x.x), mulsignf(-8.7422776573475857731e-08f * -0.5f, x.x)};
            x = df_add2_df_df(x, h);
        }
        s = df_normalize(x);
    }
    float u = poly_tail(s, s);
    if (q & 1) u = -u;
    if (d == 0.0f && signbit(d)) u = d;
    return u;
}

float sleef_cosf_u1(float d) {
    int q;
    df s;
    if (fabsf(d) < TRIGRANGEMAX2f) {
        const float dq = fmaf(rintf(fmaf(d, (float)M_1_PI, -0.5f)), 2.0f, 1.0f);
        q = (int)dq;
        s = df_add2_f_f(d, dq * (-PI_A2f * 0.5f));
        s = df_add2_df_f(s, dq * (-PI_B2f * 0.5f));
        s = df_add2_df_f(s, dq * (-PI_C2f * 0.5f));
    } else {
        int i;
        df x;
        reduce_half_pi(d, &i, &x);
        q = ((i & 3) * 2 + (x.x > 0 ? 8 : 7)) >> 1;
        if ((i & 1) == 0) {
            const float y = x.x > 0 ? 0.0f : -1.0f;
            df h = {mulsignf(3.1415927410125732422f * -0.5f, y), mulsignf(-8.7422776573475857731e-08f * -0.5f, y)};
            x = df_add2_df_df(x, h);
        }
        s = df_normalize(x);
    }
    float u = poly_tail(s, s);
    if ((q & 2) == 0) u = -u;
    return u;
}

/* batch entry points for the tests */
void sleef_sinf_n(const float* x, float* y, long n) { for (long i = 0; i < n; ++i) y[i] = sleef_sinf_u1(x[i]); }
void sleef_cosf_n(const float* x, float* y, long n) { for (long i = 0; i < n; ++i) y[i] = sleef_cosf_u1(x[i]); }
