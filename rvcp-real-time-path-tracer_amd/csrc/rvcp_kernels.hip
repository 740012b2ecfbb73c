// rvcp_kernels.hip -- gfx950 (CDNA4) path-tracing kernel for the hot path of
// YXHXianYu/RVCP-Real-Time-Path-Tracer: assets/shaders/ray_tracer_games101_branch.comp,
// dispatched from src/ray_tracer/vulkan.rs:446.
//
// Design:
//  * Persistent wave64 "ray machine".  Every lane owns one pixel at a time and advances it
//    through an explicit state machine; each loop iteration the whole wave traces exactly one
//    ray per lane (a primary, path or shadow ray) through the brute-force triangle scan, then
//    every lane runs the small shading step that produces its next ray.  A lane whose pixel
//    finishes takes the next pixel from a per-wave chunk of the frame queue (one atomic per
//    64 pixels), so lanes never idle while the frame has work.  This replaces the
//    reference's lockstep SPP x bounce loops (:494, :413), which leave ~70 % of an 8x8 wave
//    idle waiting for the longest path.
//  * The scan reads the triangles with wave-uniform addresses, so they arrive as scalar
//    loads into SGPRs (s_load_dwordx*), broadcast to all 64 lanes; the scan is VALU-bound.
//  * The primary ray does not depend on the RNG (:491 is outside the SPP loop), so its hit
//    record is computed once per pixel and reused by every sample.
//  * The hit record (interpolated normal, material) is resolved once per traversal for the
//    nearest face only, instead of once per accepted face.
//
// Numerics: float32, no contraction (-ffp-contract=off), IEEE correctly
// rounded division and sqrt, the software sin shared with the CPU oracle by contract, so
// every pixel is bit-identical to oracle/rvcp_oracle.c.
#include <hip/hip_runtime.h>

#include "rvcp_internal.h"
#include "../../include/rvcp.h"

namespace rvcp {
namespace {

// ------------------------------------------------------------------------------------
// vec3 algebra with GLSL evaluation order
// ------------------------------------------------------------------------------------
struct f3 { float x, y, z; };
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float len(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return muls(a, 1.0f / __builtin_sqrtf(dot(a, a))); }
__device__ __forceinline__ float fractf(float x) { return x - __builtin_floorf(x); }
__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

constexpr float kPi = 3.1415926f;       // ray_tracer_games101_branch.comp:6
constexpr uint32_t kLight = 3u;         // MATERIAL_LIGHT :25

// Software sin: the DESIGN.md §3.2 contract (same algorithm as the oracle).
__device__ __forceinline__ float pt_sinf(float x) {
    if (!(__builtin_fabsf(x) < 1.0e30f)) return x - x;
    const float q = __builtin_rintf(x * 0.636619772367581343f);
    float r = __builtin_fmaf(q, -1.57079637050628662109375f, x);
    r = __builtin_fmaf(q, 4.37113900018624283e-8f, r);
    const float z = r * r;
    const float ps = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z,
                                    -1.6666654611e-1f);
    const float s = __builtin_fmaf(ps, z * r, r);
    const float pc = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f),
                                    z, 4.166664568298827e-2f);
    const float c = __builtin_fmaf(pc, z * z, __builtin_fmaf(-0.5f, z, 1.0f));
    const float qm = q - 4.0f * __builtin_floorf(q * 0.25f);
    const int j = (int)qm;
    const float v = (j & 1) ? c : s;
    return (j & 2) ? -v : v;
}

// rand(), :159-162: index += 1; fract(sin(seed + index) * 43758.5453)
__device__ __forceinline__ float rnd(float seed, float &idx) {
    idx = idx + 1.0f;
    return fractf(pt_sinf(seed + idx) * 43758.5453f);
}

// Tone map + UNORM8 (:498-500) by the threshold table of DESIGN.md §3.3.
__device__ __forceinline__ uint32_t gamma_u8(float c, const float *__restrict__ T) {
    const float x = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = 128; step >= 1; step >>= 1)
        if (x >= T[lo + step]) lo += step;
    return lo;
}

// Lane actions of the ray machine.
enum : int { A_TRACE = 0, A_RR = 1, A_END = 2, A_SURF = 3, A_NEED = 4, A_DONE = 5 };
// Kinds of the ray a lane is tracing.
enum : int { K_PRIMARY = 0, K_PATH = 1, K_SHADOW = 2 };

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t rank_in(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace

// ------------------------------------------------------------------------------------
// The persistent path-tracing kernel
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void games101_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters)
{
    const uint32_t lane = lane_id();
    const uint32_t wave_global =
        __builtin_amdgcn_readfirstlane((blockIdx.x * kBlock + threadIdx.x) / kWave);

    // wave-uniform queue state: [chunk_next, chunk_end) of pixels owned by this wave
    uint32_t chunk_next = wave_global * kChunk;
    uint32_t chunk_end = chunk_next + kChunk;
    if (chunk_next > A.n_pixels) chunk_next = A.n_pixels;
    if (chunk_end > A.n_pixels) chunk_end = A.n_pixels;
    bool exhausted = false;

    const float sppf = (float)A.spp;
    const float Wf = (float)A.width, Hf = (float)A.height;

    // ---- lane state ----
    int action = A_NEED, kind = K_PRIMARY;
    uint32_t pix = 0, k = 0, depth = 0, trav = 0, waves_iter = 0;
    float seed = 0.0f, ridx = 0.0f;
    f3 acc = mk(0, 0, 0), att = mk(1, 1, 1), col = mk(0, 0, 0);
    f3 P_pos = mk(0, 0, 0), P_nrm = mk(0, 0, 0);   // cached primary hit (surface)
    uint32_t P_mat = 0;
    f3 S_pos = mk(0, 0, 0), S_nrm = mk(0, 0, 0);   // current shading point
    uint32_t S_mat = 0;
    f3 nee_C = mk(0, 0, 0);
    float nee_dist = 0.0f;
    f3 ro = mk(0, 0, 0), rd = mk(0, 0, 1);
    float rtmin = 0.0f, rtmax = 0.0f;

    for (;;) {
        // ============ settle: advance every lane until it has a ray or is done ============
        for (;;) {
            // --- Russian roulette + BRDF sample (:461-478) ---
            if (action == A_RR) {
                if (rnd(seed, ridx) > A.rr) {
                    action = A_END;
                } else {
                    f3 p;
                    do {                                              // :195-201
                        const float rx = rnd(seed, ridx);
                        const float ry = rnd(seed, ridx);
                        const float rz = rnd(seed, ridx);
                        p = mk(2.0f * rx - 1.0f, 2.0f * ry - 1.0f, 2.0f * rz - 1.0f);
                    } while (dot(p, p) >= 1.0f);
                    const f3 h = dot(p, S_nrm) > 0.0f ? p : neg(p);   // :207-210
                    const f3 wi = normalize(h);                       // :212-214
                    const float cosw = dot(S_nrm, wi);
                    const MatRecord m = mats[S_mat];
                    const f3 f = cosw > 0.0f ? divs(ld3(m.albedo), kPi) : mk(0, 0, 0);
                    const float pdf = dot(wi, S_nrm) > 0.0f ? 0.5f / kPi : 0.0f;
                    const float denom = __builtin_fmaxf(0.1f, pdf) * A.rr;
                    att = mulv(att, divs(muls(f, cosw), denom));       // :465-471
                    depth += 1;
                    ro = add(S_pos, muls(wi, A.eps));                  // :473-478
                    rd = wi;
                    rtmin = A.t_min;
                    rtmax = A.t_max;
                    kind = K_PATH;
                    const bool stop = att.x < A.att_stop && att.y < A.att_stop &&
                                      att.z < A.att_stop;             // :415-419
                    action = (depth >= A.max_bounces || stop) ? A_END : A_TRACE;
                }
            }
            // --- end of one sample: color += L / SPP (:495) ---
            if (action == A_END) {
                acc = add(acc, divs(col, sppf));
                k += 1;
                if (k >= A.spp) {
                    const uint32_t rgba = gamma_u8(acc.x, gamma_t) | (gamma_u8(acc.y, gamma_t) << 8) |
                                          (gamma_u8(acc.z, gamma_t) << 16) | 0xFF000000u;
                    out_rgba[pix] = rgba;
                    if (A.want_linear) {
                        out_lin[3 * (size_t)pix + 0] = acc.x;
                        out_lin[3 * (size_t)pix + 1] = acc.y;
                        out_lin[3 * (size_t)pix + 2] = acc.z;
                    }
                    action = A_NEED;
                } else {
                    depth = 0;
                    att = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    S_pos = P_pos;
                    S_nrm = P_nrm;
                    S_mat = P_mat;
                    action = A_SURF;
                }
            }
            // --- surface event: light sample (:384-404) and the shadow ray (:434-447) ---
            if (action == A_SURF) {
                const float pl = rnd(seed, ridx) * A.light_total;
                uint32_t li = A.n_lights;
                for (uint32_t i = 0; i < A.n_lights; ++i) {
                    if (pl <= lights[i].cum) { li = i; break; }
                }
                if (li >= A.n_lights) {
                    action = A_RR;      // no luminous face: no NEE term
                } else {
                    const LightRecord &L = lights[li];
                    const float x = __builtin_sqrtf(rnd(seed, ridx));
                    const float y = rnd(seed, ridx);
                    const f3 Xp = add(add(muls(ld3(L.v0), 1.0f - x), muls(ld3(L.v1), x * (1.0f - y))),
                                      muls(ld3(L.v2), x * y));                     // :324
                    const f3 dv = sub(Xp, S_pos);
                    const float dist = len(dv);                                    // :438
                    const f3 ws = divs(dv, dist);                                  // :439
                    const float cosp = dot(S_nrm, ws);
                    const MatRecord m = mats[S_mat];
                    const f3 f = cosp > 0.0f ? divs(ld3(m.albedo), kPi) : mk(0, 0, 0);
                    f3 C = mulv(mulv(att, ld3(L.le)), f);                          // :450-458
                    C = muls(C, cosp);
                    C = muls(C, dot(ld3(L.n), neg(ws)));
                    C = divs(C, dist * dist * A.light_pdf);
                    nee_C = C;
                    nee_dist = dist;
                    ro = add(S_pos, muls(ws, A.eps));                              // :441-446
                    rd = ws;
                    rtmin = A.t_min;
                    rtmax = A.t_max;
                    kind = K_SHADOW;
                    action = A_TRACE;
                }
            }
            // --- take new pixels from the frame queue (wave-uniform control flow) ---
            uint64_t need = __ballot(action == A_NEED);
            while (need != 0ull) {
                if (chunk_next >= chunk_end) {
                    if (exhausted) break;
                    uint32_t base = 0;
                    if (lane == (uint32_t)__builtin_ctzll(need))
                        base = atomicAdd((unsigned int *)&counters[1], kChunk);
                    base = __builtin_amdgcn_readfirstlane(
                               __shfl(base, (int)__builtin_ctzll(need))) + A.static_chunks;
                    if (base >= A.n_pixels) { exhausted = true; break; }
                    chunk_next = base;
                    chunk_end = base + kChunk < A.n_pixels ? base + kChunk : A.n_pixels;
                }
                const uint32_t avail = chunk_end - chunk_next;
                const uint32_t r = rank_in(need);
                const bool mine = ((need >> lane) & 1ull) && r < avail;
                const uint64_t got = __ballot(mine);
                if (mine) {
                    // ---- start a pixel: main(), :486-491 ----
                    pix = chunk_next + r;
                    const uint32_t lr = pix / A.width;
                    const uint32_t x = pix - lr * A.width;
                    const uint32_t gy = ((lr >> 3) * A.shard_count + A.shard_index) * 8u + (lr & 7u);
                    const float u_ = ((float)x + 0.5f) / Wf;
                    const float v_ = ((float)gy + 0.5f) / Hf;
                    // srand, :153-155
                    const float sa = fractf(pt_sinf(A.time) * 43758.5453f);
                    const float sb = fractf(pt_sinf(u_) * 22578.5453f);
                    const float sc = fractf(pt_sinf(v_) * 114514.1919f);
                    seed = fractf(sa + sb + sc);
                    ridx = 0.0f;
                    // sample_ray, :217-235
                    const f3 uv_pos = add(add(ld3(A.pos), muls(ld3(A.u), u_ - 0.5f)),
                                          muls(ld3(A.v), v_ - 0.5f));
                    const f3 dv = sub(uv_pos, ld3(A.cam_pos));
                    const float t_coef = len(dv) / A.base_len;
                    ro = ld3(A.cam_pos);
                    rd = normalize(dv);
                    rtmin = A.t_near * t_coef;
                    rtmax = A.t_far * t_coef;
                    kind = K_PRIMARY;
                    k = 0;
                    acc = mk(0, 0, 0);
                    action = A_TRACE;
                }
                chunk_next += __builtin_popcountll(got);
                need &= ~got;
            }
            if (exhausted && action == A_NEED) action = A_DONE;
            if (!__any(action == A_RR || action == A_END || action == A_SURF)) break;
        }
        if (!__any(action == A_TRACE)) break;
        waves_iter += 1;

        // ============ trace: brute-force nearest hit (:283-298, :238-260) ============
        int best = -1;
        float bt = rtmax;
        if (action == A_TRACE) {
            trav += 1;
            for (uint32_t i = 0; i < A.n_faces; ++i) {
                const TriRecord T = tri[i];
                const f3 s = mk(ro.x - T.v0[0], ro.y - T.v0[1], ro.z - T.v0[2]);
                const f3 e1 = ld3(T.e1), e2 = ld3(T.e2);
                const f3 s1 = cross(rd, e2);
                const f3 s2 = cross(s, e1);
                const float f = 1.0f / dot(s1, e1);
                const float t = f * dot(s2, e2);
                const float b1 = f * dot(s1, s);
                const float b2 = f * dot(s2, rd);
                // == !(b1<0 || 1<b1 || b2<0 || 1<b2 || 1<b1+b2 || t<t_min || t_max<t)
                //    && t <= t_max  (DESIGN.md §3.5 proves the equivalence, NaN included)
                const bool ok = (b1 >= 0.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f) &
                                (t >= rtmin) & (t <= bt);
                if (ok) { bt = t; best = (int)i; }
            }
        }

        // ============ post-trace shading ============
        if (action == A_TRACE) {
            if (kind == K_SHADOW) {
                // :447-459 -- visibility of the light sample
                const f3 hp = best >= 0 ? add(ro, muls(rd, bt))
                                        : mk(__builtin_inff(), __builtin_inff(), __builtin_inff());
                const float dist_blocked = len(sub(hp, S_pos));
                if (__builtin_fabsf(nee_dist - dist_blocked) < A.eps) col = add(col, nee_C);
                action = A_RR;
            } else {
                // resolve the nearest hit's record (:262-278) for face `best`
                f3 hpos = mk(0, 0, 0), hn = mk(0, 0, 0);
                uint32_t hmat = 0;
                if (best >= 0) {
                    const rvcp_face_t F = faces[best];
                    const TriRecord T = tri[best];
                    const f3 s = mk(ro.x - T.v0[0], ro.y - T.v0[1], ro.z - T.v0[2]);
                    const f3 e1 = ld3(T.e1), e2 = ld3(T.e2);
                    const f3 s1 = cross(rd, e2);
                    const f3 s2 = cross(s, e1);
                    const float f = 1.0f / dot(s1, e1);
                    const float b1 = f * dot(s1, s);
                    const float b2 = f * dot(s2, rd);
                    const f3 n0 = ld3(verts[F.vertices[0]].normal);
                    const f3 n1 = ld3(verts[F.vertices[1]].normal);
                    const f3 n2 = ld3(verts[F.vertices[2]].normal);
                    f3 n = normalize(add(add(muls(n0, 1.0f - b1 - b2), muls(n1, b1)), muls(n2, b2)));
                    if (dot(n, rd) > 0.0f) n = neg(n);
                    hn = n;
                    hpos = add(ro, muls(rd, bt));
                    hmat = F.material_id;
                }
                const bool miss = best < 0;
                const bool is_light = !miss && mats[hmat].ty == kLight;
                if (kind == K_PRIMARY) {
                    if (miss || is_light) {
                        // every sample of this pixel returns the same L without using the RNG:
                        // miss -> 0.1 (:424), light at depth 0 -> Le (:425-427)
                        const f3 L = miss ? mk(0.1f, 0.1f, 0.1f) : ld3(mats[hmat].albedo);
                        const f3 Ls = divs(L, sppf);
                        for (uint32_t i = 0; i < A.spp; ++i) acc = add(acc, Ls);
                        const uint32_t rgba = gamma_u8(acc.x, gamma_t) | (gamma_u8(acc.y, gamma_t) << 8) |
                                              (gamma_u8(acc.z, gamma_t) << 16) | 0xFF000000u;
                        out_rgba[pix] = rgba;
                        if (A.want_linear) {
                            out_lin[3 * (size_t)pix + 0] = acc.x;
                            out_lin[3 * (size_t)pix + 1] = acc.y;
                            out_lin[3 * (size_t)pix + 2] = acc.z;
                        }
                        action = A_NEED;
                    } else {
                        P_pos = hpos; P_nrm = hn; P_mat = hmat;
                        S_pos = hpos; S_nrm = hn; S_mat = hmat;
                        depth = 0;
                        att = mk(1, 1, 1);
                        col = mk(0, 0, 0);
                        action = A_SURF;
                    }
                } else {  // K_PATH
                    if (miss) {
                        col = add(col, mk(0.1f, 0.1f, 0.1f));
                        action = A_END;
                    } else if (is_light) {
                        action = A_END;        // depth >= 1: no emission term (:426)
                    } else {
                        S_pos = hpos; S_nrm = hn; S_mat = hmat;
                        action = A_SURF;
                    }
                }
            }
        }
    }

    // executed traversals: one atomic per wave
    unsigned long long t64 = trav;
    for (int off = 32; off >= 1; off >>= 1) t64 += __shfl_xor(t64, off);
    if (lane == 0) {
        atomicAdd(&counters[0], t64);
        atomicAdd(&counters[2], (unsigned long long)waves_iter);
    }
}

// Frame assembly after the RCCL gather: slot k holds shard k's stripes packed.
__global__ void assemble_kernel(const uint32_t *__restrict__ gathered, uint32_t slot_rows,
                                uint32_t width, uint32_t height, uint32_t shard_count,
                                uint32_t *__restrict__ frame)
{
    const uint32_t y = blockIdx.y;
    const uint32_t stripe = y >> 3;
    const uint32_t shard = stripe % shard_count;
    const uint32_t lrow = (stripe / shard_count) * 8u + (y & 7u);
    const uint32_t *src = gathered + ((size_t)shard * slot_rows + lrow) * width;
    uint32_t *dst = frame + (size_t)y * width;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < width; x += gridDim.x * blockDim.x)
        dst[x] = src[x];
}

__global__ void fill_kernel(uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
                            uint32_t n, uint32_t rgba)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        out_rgba[i] = rgba;
        if (out_lin) { out_lin[3 * i] = 0.0f; out_lin[3 * i + 1] = 0.0f; out_lin[3 * i + 2] = 0.0f; }
    }
}

}  // namespace rvcp

extern "C" int rvcp_launch_games101(const rvcp::FrameArgs *args, const rvcp::TriRecord *tri,
                                    const void *faces, const void *verts,
                                    const rvcp::MatRecord *mats, const rvcp::LightRecord *lights,
                                    const float *gamma_t, uint32_t *out_rgba, float *out_lin,
                                    unsigned long long *counters, uint32_t grid_blocks,
                                    void *stream)
{
    hipLaunchKernelGGL(rvcp::games101_kernel, dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                       (hipStream_t)stream, *args, tri, (const rvcp_face_t *)faces,
                       (const rvcp_vertex_t *)verts, mats, lights, gamma_t, out_rgba, out_lin,
                       counters);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_launch_assemble(const uint32_t *gathered, uint32_t slot_rows, uint32_t width,
                                    uint32_t height, uint32_t shard_count, uint32_t *frame,
                                    void *stream)
{
    const uint32_t bx = (width + 255) / 256;
    hipLaunchKernelGGL(rvcp::assemble_kernel, dim3(bx, height), dim3(256), 0, (hipStream_t)stream,
                       gathered, slot_rows, width, height, shard_count, frame);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_launch_fill(uint32_t *out_rgba, float *out_lin, uint32_t n, uint32_t rgba,
                                void *stream)
{
    const uint32_t blocks = n ? (n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096 : 1;
    hipLaunchKernelGGL(rvcp::fill_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       out_rgba, out_lin, n, rgba);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_games101_occupancy(int *blocks_per_cu)
{
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_kernel, rvcp::kBlock, 0) !=
        hipSuccess)
        return -2;
    *blocks_per_cu = b;
    return 0;
}
