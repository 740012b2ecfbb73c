// rvcp_sqrt.h -- the square root of the numeric contract (IEEE, correctly rounded; DESIGN.md
// §3.9) in 5 VALU instructions instead of the ~15 of the compiler's correctly-rounded sequence.
//
// Markstein's step from the hardware reciprocal square root: y = v_rsq_f32(x), g = RN(x y),
// h = RN(y / 2), r = fma(-g, g, x), s = fma(r, h, g).  tools/sqrt_check.hip runs all 2^32
// inputs on gfx950: on every x the guard below admits (positive normal numbers in
// [2^-100, 2^100]) s equals the IEEE square root bit for bit; every other input (zero, negative,
// subnormal, tiny or huge, inf, NaN) takes the IEEE sequence.
#pragma once

namespace rvcp {

__device__ __forceinline__ bool sqrt_fast_ok(float x) {
    return (x >= 0x1p-100f) & (x <= 0x1p100f);
}

__device__ __forceinline__ float sqrt_fast_core(float x) {
    const float y = __builtin_amdgcn_rsqf(x);
    const float g = x * y;
    const float h = 0.5f * y;
    const float r = __builtin_fmaf(-g, g, x);
    return __builtin_fmaf(r, h, g);
}

// The IEEE square root: the fast core where the guard admits x, else the compiler's sequence.
__device__ __forceinline__ float sqrt_ieee(float x) {
    float s = sqrt_fast_core(x);
    if (__builtin_expect(!sqrt_fast_ok(x), 0)) s = __builtin_sqrtf(x);
    return s;
}

}  // namespace rvcp
