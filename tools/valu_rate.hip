// valu_rate.hip -- issue rate of v_fma_f32 vs v_pk_fma_f32 (and v_pk_add/mul_f32) on gfx950,
// all SIMDs busy, 8 waves per SIMD, 8 independent chains per lane.  Prints the wall time,
// wave-instructions per SIMD per clock AT AN ASSUMED 2.4 GHz and the lane-FLOP rate.  The
// clock-independent figure comes from running it under rocprofv3 --pmc SQ_INSTS_VALU
// GRBM_GUI_ACTIVE (tools/pmc_valu.py): wave-instructions / (GRBM cycles per XCD x 1024 SIMDs).
// Each launch runs `iters` x 8 instructions per lane (default 65536: ~5 ms, long enough for
// the GRBM clock quotient, MI355X_MICROARCH.md "DVFS give-back").
//   make -C tools build/valu_rate && tools/build/valu_rate [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>


#define FMA8(op)                                                                          \
    asm volatile(op " %0, %0, %8, %9\n\t" op " %1, %1, %8, %9\n\t" op " %2, %2, %8, %9\n\t"  \
                 op " %3, %3, %8, %9\n\t" op " %4, %4, %8, %9\n\t" op " %5, %5, %8, %9\n\t"   \
                 op " %6, %6, %8, %9\n\t" op " %7, %7, %8, %9"                                \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),    \
                   "+v"(a7)                                                                   \
                 : "v"(m), "v"(c))

__global__ void k_fma(float *out, float seed, int kIters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 0.999f, c = 1e-3f;
    for (int i = 0; i < kIters; i++) { FMA8("v_fma_f32"); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// The same v_fma_f32 streams with inline-constant operands (one VGPR read per instruction)
// and with 16 independent chains: whether operand reads, not the issue slot, set the rate.
#define FMA8IC                                                                              \
    asm volatile("v_fma_f32 %0, %0, 0.5, 1.0\n\tv_fma_f32 %1, %1, 0.5, 1.0\n\t"           \
                 "v_fma_f32 %2, %2, 0.5, 1.0\n\tv_fma_f32 %3, %3, 0.5, 1.0\n\t"           \
                 "v_fma_f32 %4, %4, 0.5, 1.0\n\tv_fma_f32 %5, %5, 0.5, 1.0\n\t"           \
                 "v_fma_f32 %6, %6, 0.5, 1.0\n\tv_fma_f32 %7, %7, 0.5, 1.0"                 \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),    \
                   "+v"(a7))

__global__ void k_fma_ic(float *out, float seed, int kIters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < kIters; i++) { FMA8IC; }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void k_fma16(float *out, float seed, int kIters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b0 = a0 + 8, b1 = a0 + 9, b2 = a0 + 10, b3 = a0 + 11, b4 = a0 + 12, b5 = a0 + 13,
          b6 = a0 + 14, b7 = a0 + 15;
    const float m = 0.999f, c = 1e-3f;
    for (int i = 0; i < kIters / 2; i++) {
        FMA8("v_fma_f32");
        asm volatile("v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\t"
                     "v_fma_f32 %2, %2, %8, %9\n\tv_fma_f32 %3, %3, %8, %9\n\t"
                     "v_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\t"
                     "v_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9"
                     : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
                     : "v"(m), "v"(c));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] =
        a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
}

// v_mov_b32 (no arithmetic): the bare issue rate of a one-operand VALU instruction
__global__ void k_mov(float *out, float seed, int kIters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 1.0f;
    for (int i = 0; i < kIters; i++) {
        asm volatile("v_mov_b32 %0, %8\n\tv_mov_b32 %1, %8\n\tv_mov_b32 %2, %8\n\t"
                     "v_mov_b32 %3, %8\n\tv_mov_b32 %4, %8\n\tv_mov_b32 %5, %8\n\t"
                     "v_mov_b32 %6, %8\n\tv_mov_b32 %7, %8"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                     : "v"(m));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// In-kernel clock (MI355X_MICROARCH.md "DVFS give-back" item 6): the same streams with one
// s_memtime / s_memrealtime stamp pair around the loop per wave; shader clock = d(memtime) /
// d(memrealtime) x 100 MHz.  Run after the other kernels (>= 2 s of back-to-back launches).
__global__ void k_fma_clk(float *out, float seed, int kIters, unsigned long long *st) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 0.999f, c = 1e-3f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) { FMA8("v_fma_f32"); }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
        st[2 * w] = t1 - t0;
        st[2 * w + 1] = r1 - r0;
    }
}

__global__ void k_fma_ic_clk(float *out, float seed, int kIters, unsigned long long *st) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < kIters; i++) { FMA8IC; }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
        st[2 * w] = t1 - t0;
        st[2 * w + 1] = r1 - r0;
    }
}

typedef float v2f __attribute__((ext_vector_type(2)));

__global__ void k_pkfma(float *out, float seed, int kIters) {
    v2f a0 = {seed + threadIdx.x, seed}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const v2f m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    for (int i = 0; i < kIters; i++) { FMA8("v_pk_fma_f32"); }
    const v2f s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

#define ADD8(op)                                                                          \
    asm volatile(op " %0, %0, %8\n\t" op " %1, %1, %8\n\t" op " %2, %2, %8\n\t"              \
                 op " %3, %3, %8\n\t" op " %4, %4, %8\n\t" op " %5, %5, %8\n\t"               \
                 op " %6, %6, %8\n\t" op " %7, %7, %8"                                        \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),    \
                   "+v"(a7)                                                                   \
                 : "v"(m))

__global__ void k_add(float *out, float seed, int kIters) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
          a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 1e-3f;
    for (int i = 0; i < kIters; i++) { ADD8("v_add_f32"); }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void k_pkadd(float *out, float seed, int kIters) {
    v2f a0 = {seed + threadIdx.x, seed}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const v2f m = {1e-3f, 2e-3f};
    for (int i = 0; i < kIters; i++) { ADD8("v_pk_add_f32"); }
    const v2f s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

__global__ void k_pkmul(float *out, float seed, int kIters) {
    v2f a0 = {seed + threadIdx.x, seed}, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const v2f m = {0.999f, 0.998f};
    for (int i = 0; i < kIters; i++) { ADD8("v_pk_mul_f32"); }
    const v2f s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

template <typename K>
static void run(const char *name, K kern, int lanes_per_instr, int flops_per_lane, float *out,
                int blocks, int threads, int kIters) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0f, kIters);   // warm
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0f, kIters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double s = ms * 1e-3 / 5;
    const double waves = (double)blocks * threads / 64;
    const double winstr = waves * kIters * 8;
    const double simds = 256.0 * 4;
    const double clk = 2.4e9;
    std::printf("%-14s %8.3f ms  wave-instr/SIMD/clk(@2.4GHz) %.3f  cycles/instr %.2f  "
                "TFLOP/s %.1f\n",
                name, s * 1e3, winstr / simds / (s * clk), simds * s * clk / winstr,
                winstr * 64 * lanes_per_instr * flops_per_lane / s * 1e-12);
}

template <typename K>
static void run_clk(const char *name, K kern, float *out, int blocks, int threads, int kIters) {
    const size_t waves = (size_t)blocks * threads / 64;
    unsigned long long *st = nullptr;
    if (hipMalloc(&st, waves * 16) != hipSuccess) return;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int r = 0; r < 20; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0f, kIters, st);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, 1.0f, kIters, st);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long *h = (unsigned long long *)std::malloc(waves * 16);
    (void)hipMemcpy(h, st, waves * 16, hipMemcpyDeviceToHost);
    double *ghz = (double *)std::malloc(waves * sizeof(double));
    double cyc_sum = 0;
    for (size_t w = 0; w < waves; w++) {
        ghz[w] = h[2 * w + 1] ? (double)h[2 * w] / (double)h[2 * w + 1] * 0.1 : 0.0;
        cyc_sum += (double)h[2 * w];
    }
    std::qsort(ghz, waves, sizeof(double), [](const void *x, const void *y) {
        const double d = *(const double *)x - *(const double *)y;
        return d < 0 ? -1 : d > 0 ? 1 : 0;
    });
    const double clk = ghz[waves / 2] * 1e9;
    const double s = ms * 1e-3;
    const double winstr = (double)waves * kIters * 8;
    const double simds = 256.0 * 4;
    // per SIMD: the instructions issued / the shader cycles of the kernel at the in-kernel clock
    std::printf("%-14s %8.3f ms  in-kernel clock %.3f GHz (p10 %.3f, p90 %.3f)  "
                "wave-instr/SIMD/shader-clk %.3f  cycles/instr %.2f\n",
                name, s * 1e3, clk * 1e-9, ghz[waves / 10], ghz[waves * 9 / 10],
                winstr / simds / (s * clk), simds * s * clk / winstr);
    std::free(h);
    std::free(ghz);
    (void)hipFree(st);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 65536;
    const int threads = 256, blocks = 256 * 8;   // 8 waves per SIMD
    float *out = nullptr;
    if (hipMalloc(&out, sizeof(float) * threads * blocks) != hipSuccess) return 2;
    run("v_fma_f32", k_fma, 1, 2, out, blocks, threads, iters);
    run("v_pk_fma_f32", k_pkfma, 2, 2, out, blocks, threads, iters);
    run("v_add_f32", k_add, 1, 1, out, blocks, threads, iters);
    run("v_pk_add_f32", k_pkadd, 2, 1, out, blocks, threads, iters);
    run("v_pk_mul_f32", k_pkmul, 2, 1, out, blocks, threads, iters);
    run("v_fma_f32 ic", k_fma_ic, 1, 2, out, blocks, threads, iters);
    run("v_fma_f32 x16", k_fma16, 1, 2, out, blocks, threads, iters);
    run("v_mov_b32", k_mov, 1, 0, out, blocks, threads, iters);
    run_clk("v_fma_f32 clk", k_fma_clk, out, blocks, threads, iters);
    run_clk("v_fma_f32 ic clk", k_fma_ic_clk, out, blocks, threads, iters);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
