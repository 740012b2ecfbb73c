// traffic_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against
// known byte counts, for the access widths the path kernels use:
//   read16   coalesced 16 B per lane (float4)                  -- wide streaming read
//   read4    coalesced 4 B per lane                            -- narrow streaming read
//   rec48    one 48-B record per lane (3 x float4), records contiguous across lanes
//            (the SurfRecord list of the path kernel)
//   write16  coalesced 16 B per lane
//   write4   coalesced 4 B per lane
//   scat4    4 B per lane to scattered pixels (a fixed odd-stride permutation: every line
//            is eventually fully written, but by lanes of different waves) -- the frame stores
// Every buffer is 1 GiB, four times the 256 MiB Infinity Cache, and each kernel runs 3 times.
// Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`;
// tools/traffic_calib.py divides the counters by the byte counts printed here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr size_t kBytes = size_t(1) << 30;
constexpr int kBlock = 256;

__global__ void read16(const float4 *__restrict__ in, size_t n, float *__restrict__ sink)
{
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const float4 v = in[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1.2345f) sink[0] = acc;     // never true for the zero-filled input; keeps the loads
}

__global__ void read4(const float *__restrict__ in, size_t n, float *__restrict__ sink)
{
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        acc += in[i];
    if (acc == 1.2345f) sink[0] = acc;
}

struct Rec48 { float4 a, b, c; };

__global__ void rec48(const Rec48 *__restrict__ in, size_t n, float *__restrict__ sink)
{
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const Rec48 r = in[i];
        acc += r.a.x + r.b.y + r.c.z + r.c.w;
    }
    if (acc == 1.2345f) sink[0] = acc;
}

__global__ void write16(float4 *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        out[i] = make_float4((float)i, 1.0f, 2.0f, 3.0f);
}

__global__ void write4(float *__restrict__ out, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        out[i] = (float)i;
}

__global__ void scat4(unsigned *__restrict__ out, size_t n)
{
    // i -> (i * 40503) mod n, n a power of two and the multiplier odd: a permutation
    for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        out[(i * 40503u) & (n - 1)] = (unsigned)i;
}

int main()
{
    void *buf = nullptr;
    float *sink = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc((void **)&sink, sizeof(float)));
    CHECK(hipMemset(buf, 0, kBytes));
    CHECK(hipDeviceSynchronize());
    const int grid = 8192;                            // 32 blocks of 4 waves per CU
    const size_t n16 = kBytes / 16, n4 = kBytes / 4, n48 = kBytes / 48;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(read16, dim3(grid), dim3(kBlock), 0, 0, (const float4 *)buf, n16, sink);
        hipLaunchKernelGGL(read4, dim3(grid), dim3(kBlock), 0, 0, (const float *)buf, n4, sink);
        hipLaunchKernelGGL(rec48, dim3(grid), dim3(kBlock), 0, 0, (const Rec48 *)buf, n48, sink);
        hipLaunchKernelGGL(write16, dim3(grid), dim3(kBlock), 0, 0, (float4 *)buf, n16);
        hipLaunchKernelGGL(write4, dim3(grid), dim3(kBlock), 0, 0, (float *)buf, n4);
        hipLaunchKernelGGL(scat4, dim3(grid), dim3(kBlock), 0, 0, (unsigned *)buf, n4);
        CHECK(hipDeviceSynchronize());
        // the write kernels leave non-zero data; restore the zero input for the next reads
        CHECK(hipMemset(buf, 0, kBytes));
        CHECK(hipDeviceSynchronize());
    }
    std::printf("bytes read16 %zu read4 %zu rec48 %zu write16 %zu write4 %zu scat4 %zu\n",
                kBytes, kBytes, n48 * 48, kBytes, kBytes, kBytes);
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
