/* Exhaustive check (run in the build container = the reference host): oracle/glibc_expf.c
 * == this host's libm expf on all 2^32 float inputs, and how often that expf differs from
 * the correctly rounded value on (-87, 0] (the softmax's x - max range).
 *   gcc -O2 -mfma tools/cpu_order/check_glibc_expf.c oracle/glibc_expf.c -lm -o /tmp/chk && /tmp/chk */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
float oracle_glibc_expf(float x);
int main(void) {
    uint64_t bad = 0, cr_diff = 0;
    for (uint64_t u = 0; u < 0x100000000ull; ++u) {
        const uint32_t b = (uint32_t)u;
        float x;
        memcpy(&x, &b, 4);
        const float a = expf(x), m = oracle_glibc_expf(x);
        if (memcmp(&a, &m, 4) != 0 && !(isnan(a) && isnan(m))) {
            if (bad < 10) printf("x=%a libm=%a restated=%a\n", x, a, m);
            ++bad;
        }
        if (x <= 0.f && x > -87.f && (float)exp((double)x) != a) ++cr_diff;
    }
    printf("all 2^32 inputs: %llu mismatches; libm expf != correctly rounded on (-87, 0]: %llu inputs\n",
           (unsigned long long)bad, (unsigned long long)cr_diff);
    return bad != 0;
}
