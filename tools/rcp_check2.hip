// rcp_check2.hip -- exhaustive check of the class-guarded fast reciprocal over ALL 2^32 float
// bit patterns on gfx950: r = v_rcp_f32(d); f = fma(fma(-d, r, 1), r, r); the fast value is
// used iff f is a normal number (v_cmp_class: not zero / subnormal / inf / NaN), and then it
// must equal the IEEE quotient 1.0f / d bit for bit.  Build:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o rcp_check2 rcp_check2.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void check(uint32_t hi, unsigned long long *bad, unsigned long long *used,
                      unsigned *first)
{
    const uint32_t bits = (hi << 24) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float d = __uint_as_float(bits);
    const float r = __builtin_amdgcn_rcpf(d);
    const float f = __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
    // class mask: bit 8 = +normal, bit 3 = -normal (v_cmp_class_f32 encoding)
    const bool normal = __builtin_amdgcn_classf(f, (1 << 8) | (1 << 3));
    if (!normal) return;
    atomicAdd(used, 1ull);
    const float exact = 1.0f / d;
    if (__float_as_uint(f) != __float_as_uint(exact)) {
        const unsigned long long n = atomicAdd(bad, 1ull);
        if (n < 8) first[n] = bits;
    }
}

int main()
{
    unsigned long long *bad, *used;
    unsigned *first;
    hipMalloc(&bad, 8);
    hipMalloc(&used, 8);
    hipMalloc(&first, 32);
    hipMemset(bad, 0, 8);
    hipMemset(used, 0, 8);
    for (uint32_t hi = 0; hi < 256; hi++)
        hipLaunchKernelGGL(check, dim3((1u << 24) / 256), dim3(256), 0, 0, hi, bad, used, first);
    unsigned long long b = 0, u = 0;
    unsigned f[8] = {0};
    hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&u, used, 8, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("all 2^32 inputs: fast path taken for %llu, mismatches %llu", u, b);
    for (int i = 0; i < 8 && i < (int)b; i++) printf(" %08x", f[i]);
    printf("\n");
    return b == 0 ? 0 : 1;
}
