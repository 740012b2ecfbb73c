/* rand_fract_check.c -- compiled and run by tests/test_rand_fract_cpu.py against the CPU oracle
 * (TEST INFRASTRUCTURE).  The kernel's rand() takes fract with v_fract_f32, which equals
 * x - floor(x) except where that difference rounds to 1.0 (a negative x within 2^-25 of zero).
 * x = sin(y) * 43758.5453 with the contract's software sin (the oracle's and the
 * kernel's are the same bits): every float argument y the RNG can form lies in [1, 2^25]
 * (seed in [0, 1) plus an index that stops growing at 2^24, plus at most 3 x 64 + 3 in the
 * cooperative unit-sphere rounds).  This checks every one of them. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
float rvcp_oracle_sinf(float x);
int main(void) {
    uint64_t n = 0, hits = 0; uint32_t lo = 0x3f800000u, hi = 0x4c000000u;
    float minpos = 1.0f;
    for (uint32_t b = lo; b <= hi; b++) {
        float y; memcpy(&y, &b, 4);
        float x = rvcp_oracle_sinf(y) * 43758.5453f;
        float f = x - floorf(x);
        n++;
        if (f == 1.0f) { hits++; if (hits < 10) printf("hit y=%a x=%a\n", y, x); }
        if (x < 0 && -x < minpos) minpos = -x;
    }
    printf("checked %llu rand arguments in [1, 2^25]: fract == 1.0 in %llu; smallest |x| of negative x: %a\n",
           (unsigned long long)n, (unsigned long long)hits, minpos);
    return hits != 0;
}
