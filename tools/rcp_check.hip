// rcp_check.hip -- exhaustive check that a fast reciprocal equals IEEE 1/x (round to nearest)
// on gfx950.  Candidate: r = v_rcp_f32(d); e = fma(-d, r, 1); r' = fma(e, r, r).
// Every mantissa of every exponent in [lo, hi] and both signs.  Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o rcp_check rcp_check.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void check(int exp_lo, int exp_hi, unsigned long long *bad, unsigned *first)
{
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;       // 23-bit mantissa
    if (m >= (1u << 23)) return;
    for (int e = exp_lo; e <= exp_hi; ++e) {
        for (uint32_t s = 0; s < 2; ++s) {
            const uint32_t bits = (s << 31) | ((uint32_t)(e + 127) << 23) | m;
            const float d = __uint_as_float(bits);
            const float exact = 1.0f / d;                           // IEEE (div_scale/fmas/fixup)
            const float r = __builtin_amdgcn_rcpf(d);
            const float err = __builtin_fmaf(-d, r, 1.0f);
            const float fast = __builtin_fmaf(err, r, r);
            if (__float_as_uint(fast) != __float_as_uint(exact)) {
                const unsigned long long n = atomicAdd(bad, 1ull);
                if (n < 8) first[n] = bits;
            }
        }
    }
}

int main()
{
    unsigned long long *bad;
    unsigned *first;
    hipMalloc(&bad, sizeof(unsigned long long));
    hipMalloc(&first, 8 * sizeof(unsigned));
    // every normal exponent the guarded fast path admits (|x| in [2^-126, 2^126)), then the
    // excluded top binade for contrast
    const int ranges[][2] = {{-126, -64}, {-63, 0}, {1, 63}, {64, 125}, {126, 126}};
    for (auto &rg : ranges) {
        hipMemset(bad, 0, sizeof(unsigned long long));
        hipLaunchKernelGGL(check, dim3((1u << 23) / 256), dim3(256), 0, 0, rg[0], rg[1], bad, first);
        unsigned long long h = 0;
        unsigned f[8] = {0};
        hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
        printf("exponents [%d, %d]: %llu mismatches", rg[0], rg[1], h);
        for (int i = 0; i < 8 && i < (int)h; i++) printf(" %08x", f[i]);
        printf("\n");
    }
    return 0;
}
