// rvcp_mandelbrot.hip -- the reference's second compute operator,
// assets/shaders/mandelbrot.comp:1-33 (push constant {vec2 position; float scale}, one
// invocation per pixel, escape "time" i in steps of 0.005 written as grey UNORM8).
// Numeric contract: f32, IEEE division / sqrt, and the iteration contracted
// the way the reference's compiled shader evaluates it -- z.x' = fma(z.x, z.x, -(z.y*z.y)) + c.x,
// z.y' = fma(z.x + z.x, z.y, c.y) -- which, with the driver's UNORM8 conversion (the unorm_t
// table), reproduces the reference's own render (Notes/README/fractal.png) on every pixel;
// bit-identical to oracle/rvcp_oracle.c.
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace {

constexpr int kTileX = 16, kTileY = 16;

__global__ __launch_bounds__(kTileX * kTileY) void mandelbrot_kernel(
    float pos_x, float pos_y, float scale, uint32_t width, uint32_t height,
    const float *__restrict__ unorm_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_value)
{
    const uint32_t x = blockIdx.x * kTileX + threadIdx.x;
    const uint32_t y = blockIdx.y * kTileY + threadIdx.y;
    if (x >= width || y >= height) return;
    // :14-18
    const float nx = ((float)x + 0.5f) / (float)width;
    const float ny = ((float)y + 0.5f) / (float)height;
    float cx = (nx - 0.5f) * 2.0f;
    float cy = (ny - 0.5f) * 2.0f;
    cx = cx / scale + pos_x;
    cy = cy / scale + pos_y;
    cx = cx - 1.0f;
    cy = cy - 0.0f;
    // :20-31
    float zx = 0.0f, zy = 0.0f, i;
    for (i = 0.0f; i < 1.0f; i += 0.005f) {
        // :22-25; zy*zx + zx*zy == 2*(zx*zy) exactly, so the fma of (zx + zx) is the
        // contracted form of the shader's expression, not a different one
        const float nzx = __builtin_fmaf(zx, zx, -(zy * zy)) + cx;
        const float nzy = __builtin_fmaf(zx + zx, zy, cy);
        zx = nzx;
        zy = nzy;
        if (__builtin_sqrtf(__builtin_fmaf(zy, zy, zx * zx)) > 4.0f) break;   // length: §3.1 dot
    }
    // :32-33, vec4(vec3(i), 1.0) stored as UNORM8: u8 = #{k : clamp(i) >= U[k]}
    const float c = (i > 0.0f) ? ((i < 1.0f) ? i : 1.0f) : 0.0f;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 128; step >= 1; step >>= 1)
        if (c >= unorm_t[lo + step]) lo += step;
    const size_t p = (size_t)y * width + x;
    out_rgba[p] = lo | (lo << 8) | (lo << 16) | 0xFF000000u;
    if (out_value) out_value[p] = i;
}

}  // namespace

extern "C" int rvcp_launch_mandelbrot(float pos_x, float pos_y, float scale, uint32_t width,
                                      uint32_t height, const float *unorm_t, uint32_t *out_rgba,
                                      float *out_value, void *stream)
{
    const dim3 grid((width + kTileX - 1) / kTileX, (height + kTileY - 1) / kTileY);
    hipLaunchKernelGGL(mandelbrot_kernel, grid, dim3(kTileX, kTileY), 0, (hipStream_t)stream,
                       pos_x, pos_y, scale, width, height, unorm_t, out_rgba, out_value);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
