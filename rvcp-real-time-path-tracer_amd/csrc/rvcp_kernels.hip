// rvcp_kernels.hip -- gfx950 (CDNA4) path-tracing kernels for the hot path of
// YXHXianYu/RVCP-Real-Time-Path-Tracer: assets/shaders/ray_tracer_games101_branch.comp,
// dispatched from src/ray_tracer/vulkan.rs:446.
//
// Design:
//  * Persistent wave64 "ray machines".  Every lane owns one pixel at a time and advances it
//    through an explicit state machine that keeps the shader's RNG order, accumulation order
//    and termination rules; each loop iteration the wave traces rays through the brute-force
//    triangle scan, then every lane runs the shading step that produces its next ray(s).  A
//    lane whose pixel finishes takes the next pixel from a per-wave chunk of the frame queue
//    (one atomic per 64 pixels), so lanes never idle while the frame has work.  This replaces
//    the reference's lockstep SPP x bounce loops (:494, :413).
//      variant 1: one ray per lane per iteration (primary, path or shadow);
//      variant 2: a surface event emits its shadow ray AND its continuation ray (the RNG
//                 stream does not depend on the visibility result), both traced in one scan.
//  * The scan reads the triangles with wave-uniform addresses, so they arrive as scalar loads
//    into SGPRs (s_load_dwordx*), broadcast to all 64 lanes; the scan is VALU-bound.
//  * The primary ray does not depend on the RNG (:491 is outside the SPP loop): its hit record
//    is computed once per pixel and reused by every sample.
//  * The hit record (interpolated normal, material) is resolved once per traversal, for the
//    nearest face only.
//
// Numerics: float32, no implicit contraction (-ffp-contract=off; the
// builtins dot/cross are explicit fma chains), IEEE correctly rounded division and sqrt,
// the software sin of the contract, so every pixel is
// bit-identical to oracle/rvcp_oracle.c whichever variant runs.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

#include "rvcp_internal.h"
#include "../../include/rvcp.h"
#include "rvcp_sqrt.h"

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
// The GLSL builtins dot and cross as fused chains: dot = fma(z, z',
// fma(y, y', x*x')), cross_i = fma(a_j, b_k, -(a_k*b_j)).  Arithmetic written out in the
// shader source stays unfused.
__device__ __forceinline__ float dot(f3 a, f3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
              __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
// The IEEE square root: rvcp_sqrt.h's 5-instruction form where its guard admits x (equal to the
// correctly rounded root on every such input, tools/sqrt_check.hip), else the compiler's
// correctly-rounded sequence
__device__ __forceinline__ float sqrt_c(float x) { return sqrt_ieee(x); }
__device__ __forceinline__ float len(f3 a) { return sqrt_c(dot(a, a)); }
// 1 / sqrt by rcp_ieee below (the IEEE quotient, fast path verified over all inputs)
__device__ __forceinline__ float rcp_ieee(float den);
// normalize(v) = v * RN(1 / RN(sqrt(dot(v, v)))).  Where sqrt_fast_ok admits x = dot(v, v) the
// root s lies in [2^-50, 2^50] and its reciprocal is normal -- and wherever v_rcp + one Newton
// step gives a normal result it equals the IEEE quotient (all 2^32 inputs, tools/rcp_check2.hip)
// -- so the root's guard covers the reciprocal too: one guard and one rare branch instead of
// two.  Any other x takes the IEEE root and rcp_ieee.
__device__ __forceinline__ f3 normalize(f3 a) {
    const float x = dot(a, a);
    const float s = sqrt_fast_core(x);
    const float y = __builtin_amdgcn_rcpf(s);
    float r = __builtin_fmaf(__builtin_fmaf(-s, y, 1.0f), y, y);
    if (__builtin_expect(!sqrt_fast_ok(x), 0)) r = rcp_ieee(__builtin_sqrtf(x));
    return muls(a, r);
}
__device__ __forceinline__ float fractf(float x) { return x - __builtin_floorf(x); }
__device__ __forceinline__ f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

constexpr uint32_t kLight = 3u;         // MATERIAL_LIGHT, ray_tracer_games101_branch.comp:25

// Software sin: the DESIGN.md §3.2 contract (same algorithm as the oracle): reduction by pi
// (q = rint(x / pi), two-constant Cody-Waite with fma), one odd minimax polynomial on
// [-pi/2, pi/2], sign flipped for odd q.
constexpr float kInvPi = 0x1.45f306p-2f;          // float(1 / pi)
constexpr float kPiHi = 0x1.921fb6p+1f;           // float(pi)
constexpr float kPiLo = 0x1.777a5cp-24f;          // float(float(pi) - pi)
__device__ __forceinline__ float sin_poly(float r) {
    const float z = r * r;
    const float p = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(0x1.5dbdfep-19f, z, -0x1.9f7p-13f),
                                                  z, 0x1.110ed4p-7f), z, -0x1.55554cp-3f);
    return __builtin_fmaf(p, z * r, r);
}
__device__ __forceinline__ float pt_sinf(float x) {
    if (!(__builtin_fabsf(x) < 1.0e30f)) return x - x;
    const float q = __builtin_rintf(x * kInvPi);
    float r = __builtin_fmaf(q, -kPiHi, x);
    r = __builtin_fmaf(q, kPiLo, r);
    const float s = sin_poly(r);
    const float odd = q - 2.0f * __builtin_floorf(q * 0.5f);      // q mod 2, exact
    return odd != 0.0f ? -s : s;
}

// pt_sinf for rand()'s arguments only: seed + index with seed in [0, 1] (a fract) and index a
// float counter that stops growing at 2^24, so x lies in [1, 2^24 + 4]: finite and positive,
// q = rint(x / pi) < 2^23 is an exact integer, and its parity is the low bit of (int)q, moved
// into the sign bit.  The same arithmetic as pt_sinf without its range guard.  (The flip is an
// add: q << 31 is 0 or 2^31, and adding 2^31 mod 2^32 flips bit 31 alone -- one v_lshl_add_u32
// instead of a shift and an xor.)
__device__ __forceinline__ float pt_sinf_rand(float x) {
    const float q = __builtin_rintf(x * kInvPi);
    float r = __builtin_fmaf(q, -kPiHi, x);
    r = __builtin_fmaf(q, kPiLo, r);
    const float s = sin_poly(r);
    return __uint_as_float(__float_as_uint(s) + ((uint32_t)(int)q << 31));
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t rank_in(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// _rand's fract (:156-158) with one instruction: v_fract_f32 is x - floor(x) except where that
// rounds to 1.0 (it returns 1 - 2^-24 there), i.e. for a negative x within 2^-25 of zero.  For
// x = sin(y) * 43758.5453 no float rand() argument y in [1, 2^25] (seed + an index that stops
// growing at 2^24, plus at most 195 in coop_unit_sphere) gives such an x (the closest negative x
// is -2^-11.6): checked over all of them with the oracle's sin on the CPU
// (tests/test_rand_fract_cpu.py) and with this kernel's sin and v_fract_f32 on the GPU
// (tools/sqrt_check.hip).  DESIGN.md §3.10.
__device__ __forceinline__ float rand_of(float y) {
    return __builtin_amdgcn_fractf(pt_sinf_rand(y) * 43758.5453f);
}
// rand3's unit-cube coordinate 2 r - 1 (:197): 2 r is exact, so the fused form rounds the same
// value once, as the written two-step form does
__device__ __forceinline__ float cube_coord(float r) { return __builtin_fmaf(2.0f, r, -1.0f); }

// rand(), :159-162: index += 1; fract(sin(seed + index) * 43758.5453)
__device__ __forceinline__ float rnd(float seed, float &idx) {
    idx = idx + 1.0f;
    return rand_of(seed + idx);
}

// 1 / den, IEEE round-to-nearest (the shader's `1.0 / dot(s1, e1)`, :254).
// Fast path: v_rcp_f32 plus one FMA Newton step, kept whenever the result is a normal number
// (one v_cmp_class); otherwise -- zero, subnormal, inf or NaN result, i.e. a degenerate,
// grazing or astronomically large triangle -- the lane takes the full IEEE division.
// tools/rcp_check2.hip runs all 2^32 inputs on gfx950: the fast path is taken for
// 4,227,858,434 of them and equals the IEEE quotient bit for bit on every one.
__device__ __forceinline__ float rcp_ieee(float den) {
    const float r = __builtin_amdgcn_rcpf(den);
    float f = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    if (__builtin_expect(!__builtin_amdgcn_classf(f, (1 << 8) | (1 << 3)), 0)) f = 1.0f / den;
    return f;
}

// v / s for the three components of v, bit-identical to the IEEE quotients, for the shader's
// vector-by-scalar divisions.  y = RN(1/s) (rcp_ieee) is shared; each quotient
// is q = RN(v y) refined by Markstein's step q' = RN(q + r y) with r = v - s q exact by fma,
// which is the correctly rounded v / s whenever y = RN(1/s) and no quantity leaves the normal
// range -- guaranteed when s and every nonzero |v_i| lie in [2^-50, 2^50].  The step is
// written -RN(-(r y) - q) so that a -0 numerator keeps its -0 quotient (RN(q + r y) would give
// +0).  A lane outside that box (zero, tiny, huge, inf or NaN operands) takes the IEEE
// divisions.  tests/test_markstein_cpu.py checks the same arithmetic against IEEE division.
__device__ __forceinline__ float quot_refine(float v, float s, float y) {
    const float q = v * y;
    const float r = __builtin_fmaf(-s, q, v);
    return -__builtin_fmaf(-r, y, -q);
}
__device__ __forceinline__ bool quot_box(f3 v) {
    // |v_i| as bits << 1 (sign dropped); zero maps to 0xFFFFFFFF under the -1 of the lower test
    const uint32_t bx = __float_as_uint(v.x) << 1, by = __float_as_uint(v.y) << 1,
                   bz = __float_as_uint(v.z) << 1;
    const uint32_t hi = max(max(bx, by), bz);
    const uint32_t lo = min(min(bx - 1u, by - 1u), bz - 1u);
    return (hi <= (0x58800000u << 1)) & (lo >= (0x26800000u << 1) - 1u);   // 2^50, 2^-50
}
__device__ __forceinline__ f3 divs_y(f3 v, float s, float y) {
    f3 o = mk(quot_refine(v.x, s, y), quot_refine(v.y, s, y), quot_refine(v.z, s, y));
    const bool ok = (s >= 0x1p-50f) & (s <= 0x1p50f) & quot_box(v);
    if (__builtin_expect(!ok, 0)) o = divs(v, s);
    return o;
}
// v / s with y = RN(1/s) from v_rcp + one Newton step without rcp_ieee's class check: divs_y's
// guard admits only s in [2^-50, 2^50], where that step is the IEEE reciprocal (§3.11), and
// every other lane takes the IEEE divisions -- one guard and one rare branch instead of two.
__device__ __forceinline__ f3 divs_pos(f3 v, float s) {
    const float r = __builtin_amdgcn_rcpf(s);
    return divs_y(v, s, __builtin_fmaf(__builtin_fmaf(-s, r, 1.0f), r, r));
}

// The scan's 1 / den: rcp_ieee, except that a zero or NaN denominator keeps the fast result
// (NaN) instead of taking the IEEE division (+-inf / NaN).  Exact for the scan's decision: with
// den = +-0 the shader's t = f * dot(s2, e2) is +-inf or NaN and fails t >= t_min & t <= t_max
// (t_max < 2^24), as NaN does.  Such denominators are common -- rand() returns exactly 0.5 one
// time in a few hundred (fract of a float near 2^15 has 8 fraction bits), which gives ray
// directions with an exact zero component, parallel to the axis-aligned Cornell walls --
// and each took the whole wave through the division.
// (The denominator's class is tested inside the rare branch, so the fast path costs what
// rcp_ieee's does; a class test outside it measured 2 % slower.)
__device__ __forceinline__ float rcp_scan(float den) {
    const float r = __builtin_amdgcn_rcpf(den);
    float f = __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
    if (__builtin_expect(!__builtin_amdgcn_classf(f, (1 << 8) | (1 << 3)), 0)) {
        if (__builtin_amdgcn_classf(den, 0x39c))                     // +-normal/subnormal/inf
            f = 1.0f / den;
    }
    return f;
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

__device__ __forceinline__ uint32_t pack_rgba(f3 c, const float *__restrict__ T) {
    return gamma_u8(c.x, T) | (gamma_u8(c.y, T) << 8) | (gamma_u8(c.z, T) << 16) | 0xFF000000u;
}

__device__ __forceinline__ void store_pixel(uint32_t pix, f3 acc, const FrameArgs &A,
                                            const float *__restrict__ gamma_t,
                                            uint32_t *__restrict__ out_rgba,
                                            float *__restrict__ out_lin) {
    out_rgba[pix] = pack_rgba(acc, gamma_t);
    if (A.want_linear) {
        out_lin[3 * (size_t)pix + 0] = acc.x;
        out_lin[3 * (size_t)pix + 1] = acc.y;
        out_lin[3 * (size_t)pix + 2] = acc.z;
    }
}

// The pre-pass and the path kernels (variants 3-6, 10, BVH) leave each finished pixel's linear
// colour in `lin` (the caller's linear output, or a scratch buffer of the context) and
// tonemap_kernel converts the frame afterwards, one pixel per lane: the eight dependent table
// probes per channel of gamma_u8 otherwise ran once per finished pixel inside the path kernel,
// nearly always for a single lane of its wave.
__device__ __forceinline__ void store_acc(uint32_t pix, f3 acc, float *__restrict__ lin) {
    lin[3 * (size_t)pix + 0] = acc.x;
    lin[3 * (size_t)pix + 1] = acc.y;
    lin[3 * (size_t)pix + 2] = acc.z;
}

// One exact ray-triangle test (is_intersect_with_face, :238-260) with the nearest-hit rule
// of get_intersection_with_scene (:291), in two stages.  Stage 1: the products that do not
// need 1/den -- s = o - v0, s1 = d x e2, s2 = s x e1, den = s1.e1, n1 = s1.s, n2 = s2.d.
struct TriPart {
    f3 s2;
    float den, n1, n2;
};
__device__ __forceinline__ TriPart tri_stage1(const TriRecord &T, f3 o, f3 d) {
    const f3 s = mk(o.x - T.v0[0], o.y - T.v0[1], o.z - T.v0[2]);
    const f3 e1 = ld3(T.e1);
    const f3 s1 = cross(d, ld3(T.e2));
    TriPart P;
    P.s2 = cross(s, e1);
    P.den = dot(s1, e1);
    P.n1 = dot(s1, s);
    P.n2 = dot(P.s2, d);
    return P;
}
// Stage 2: f = 1/den, t = f (s2.e2), b1 = f n1, b2 = f n2 (:254-257); accept iff the shader
// would replace the current nearest hit whose time is `bt`.  5-compare form, DESIGN.md §3.5.
// FAST: 1/den without the class check (rcp_scan_fast) -- the scene passed scan_rcp_fast_scene
// and the ray dir_fast_ok (FrameArgs::rcp_fast).
__device__ __forceinline__ float rcp_scan_fast(float den);
template <bool FAST = false>
__device__ __forceinline__ bool tri_stage2(const TriRecord &T, const TriPart &P, float tmin,
                                           float bt, float &t_out) {
    const float f = FAST ? rcp_scan_fast(P.den) : rcp_scan(P.den);
    const float t = f * dot(P.s2, ld3(T.e2));
    const float b1 = f * P.n1;
    const float b2 = f * P.n2;
    t_out = t;
    return (b1 >= 0.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f) & (t >= tmin) & (t <= bt);
}
template <bool FAST = false>
__device__ __forceinline__ bool tri_accept(const TriRecord &T, f3 o, f3 d, float tmin, float bt,
                                           float &t_out) {
    return tri_stage2<FAST>(T, tri_stage1(T, o, d), tmin, bt, t_out);
}
// v_rcp + one Newton step, no class check: equals the IEEE quotient wherever its result is
// normal (all 2^32 inputs, tools/rcp_check2.hip), i.e. for |den| in [2^-126, 2^126]; a zero
// denominator gives NaN (rcp 0 = inf, fma(-0, inf, 1) = NaN), which rejects, as rcp_scan's kept
// fast result does.  Used where the denominator is proved +-0 or within that range for every
// ray the wave admits: the specialised scan's RVCP_SPEC_RCP_FAST (rvcp_jit.cpp `grain`) and the
// generic scan of a scene that passed scan_rcp_fast_scene (FrameArgs::rcp_fast).
__device__ __forceinline__ float rcp_scan_fast(float den) {
    const float r = __builtin_amdgcn_rcpf(den);
    return __builtin_fmaf(__builtin_fmaf(-den, r, 1.0f), r, r);
}
// dir_fast_ok: every direction component is +-0 or at least 2^-40 in magnitude (dir_grain_ok)
// and |d|_1 <= 16 -- the ray side of both proofs (rvcp_jit.cpp `kDirGrain`, `kDirMag`).
// (bits << 1) - 1 maps +-0 to 0xFFFFFFFF and orders the other magnitudes.
__device__ __forceinline__ bool dir_grain_ok(f3 d) {
    const uint32_t x = (__float_as_uint(d.x) << 1) - 1u, y = (__float_as_uint(d.y) << 1) - 1u,
                   z = (__float_as_uint(d.z) << 1) - 1u;
    return min(min(x, y), z) >= (0x2B800000u << 1) - 1u;                     // 2^-40
}
__device__ __forceinline__ bool dir_fast_ok(f3 d) {
    return (((__builtin_fabsf(d.x) + __builtin_fabsf(d.y)) + __builtin_fabsf(d.z)) <= 16.0f) &
           dir_grain_ok(d);
}
#ifdef RVCP_SPEC_SCAN        // the scene-specialised scan generated by rvcp_jit.cpp (§4.7)
#define RVCP_F32(bits) __uint_as_float(bits)
// a test's (t, index) is committed before the next test starts: without this the compiler
// interleaves all unrolled tests and spills hundreds of registers
#define RVCP_SPEC_COMMIT(t, i) do { asm volatile("" : "+v"(t), "+v"(i)); \
                                    __builtin_amdgcn_sched_barrier(0); } while (0)
// the dual scan's shadow ray: its t only (spec_scan2 keeps no face index for slot A)
#define RVCP_SPEC_COMMIT1(t) do { asm volatile("" : "+v"(t)); \
                                  __builtin_amdgcn_sched_barrier(0); } while (0)
// RVCP_SPEC_ANY(mask): does any lane of the wave pass a shadow-slot run's range mask (the
// generator's skippable blocks, rvcp_jit.cpp emit_scan)?  RVCP_SPEC_NO_SKIP (A/B only) runs
// every block.
#ifdef RVCP_SPEC_NO_SKIP
#define RVCP_SPEC_ANY(q) ((void)(q), true)
#elif defined(RVCP_SPEC_ISA_SKIP_ALL)      // tools/spec_isa.py only: the code a wave runs when
#define RVCP_SPEC_ANY(q) ((void)(q), false) // every block is skipped (never a product build)
#else
#define RVCP_SPEC_ANY(q) (__builtin_amdgcn_ballot_w64(q) != 0ull)
#endif
// The reciprocal of the specialised tests: rcp_scan, with its rare IEEE branch inline.  (A
// branch-free variant that only flags non-normal reciprocals and re-runs the wave's scan with
// the generic loop when a live ray was flagged is bit-exact too but measured 1.9x slower --
// DESIGN.md §4.7.)
#define RVCP_SPEC_RCP(den) rcp_scan(den)
// rcp_scan without the class check and its branch, where the generator has proved (rvcp_jit.cpp
// `grain`) that the denominator is +-0 or in [2^-126, 2^126] in magnitude for every ray the
// wave admits (ray_in_range with dir_grain_ok)
#define RVCP_SPEC_RCP_FAST(den) rcp_scan_fast(den)
#include RVCP_SPEC_SCAN
// The specialised scan drops products with exact-zero triangle components.  That is exact
// when no intermediate of the generic test overflows (inf * 0 = NaN rejects there, while the
// dropped term leaves a finite value): the host specialises a scene only when every |v0| <=
// 2^40 and |e1|, |e2| <= 2^41 (jit_scene_in_range), and a wave uses the unrolled scan only when
// every ray has |o|_1 <= 2^41 and |d|_1 <= 16.  Then |s| < 2^42, |s1| <= 2^46, |s2| <= 2^84,
// |den|, |n1| < 2^90, |n2| < 2^91 and |s2.e2| < 2^127: all finite.  A NaN or infinite component
// fails the compares, so non-finite rays take the generic loop too.  
// (dir_grain_ok: the premise of the generator's RVCP_SPEC_RCP_FAST reciprocals)
__device__ __forceinline__ bool ray_in_range(f3 o, f3 d) {
    return (((__builtin_fabsf(o.x) + __builtin_fabsf(o.y)) + __builtin_fabsf(o.z)) <= 0x1p41f) &
           (((__builtin_fabsf(d.x) + __builtin_fabsf(d.y)) + __builtin_fabsf(d.z)) <= 16.0f) &
           dir_grain_ok(d);
}
#endif
// A necessary condition for tri_stage2 to accept, from stage 1 alone: |n1| and |n2| at most
// RN(|den| (1 + 2^-20)) (proof: DESIGN.md §4.2).  A wave skips stage 2 of a triangle when no
// lane passes it; no result changes.
// The pretest in two halves (LDS-tiled scans): stage 1a computes s, s1 = d x e2, den and
// n1 = s1.s; only if some lane has |n1| <= m does the wave compute s2 = s x e1 and n2 (stage
// 1b) and test |n2| <= m.  The same operations on the same values as tri_stage1, so exact;
// for a mesh of small triangles most (ray, triangle) pairs of a wave already fail the first
// half, saving the 9 instructions of s2 and n2.
struct TriPartA {
    f3 s, s1;
    float den, n1, m;
};
__device__ __forceinline__ TriPartA tri_stage1a(const TriRecord &T, f3 o, f3 d) {
    TriPartA P;
    P.s = mk(o.x - T.v0[0], o.y - T.v0[1], o.z - T.v0[2]);
    P.s1 = cross(d, ld3(T.e2));
    P.den = dot(P.s1, ld3(T.e1));
    P.n1 = dot(P.s1, P.s);
    P.m = __builtin_fabsf(P.den) * 1.00000095367431640625f;      // 1 + 2^-20
    return P;
}
__device__ __forceinline__ bool tri_maybe_a(const TriPartA &P) { return __builtin_fabsf(P.n1) <= P.m; }
__device__ __forceinline__ TriPart tri_stage1b(const TriRecord &T, const TriPartA &Pa, f3 d) {
    TriPart P;
    P.s2 = cross(Pa.s, ld3(T.e1));
    P.den = Pa.den;
    P.n1 = Pa.n1;
    P.n2 = dot(P.s2, d);
    return P;
}
__device__ __forceinline__ bool tri_maybe(const TriPart &P) {
    const float m = __builtin_fabsf(P.den) * 1.00000095367431640625f;     // 1 + 2^-20
    return (__builtin_fabsf(P.n1) <= m) & (__builtin_fabsf(P.n2) <= m);
}

// Opt-in BVH (RVCP_ACCEL_BVH): nearest hit of ray (o, d) over the tree, with the scan's exact
// triangle test and its order rule -- the brute-force scan keeps the smallest t and, among
// equal t, the later face (:288-295), so candidates met in any order are kept iff
// t < bt or (t == bt and face > best).  Boxes were enlarged at build (rvcp_bvh.cpp), so the
// slab test may use a fast reciprocal.  Per-lane traversal with a private stack.
__device__ __forceinline__ bool slab(const float *b, f3 o, f3 inv, float tmin, float bt,
                                     float &tnear) {
    const float x0 = (b[0] - o.x) * inv.x, x1 = (b[3] - o.x) * inv.x;
    const float y0 = (b[1] - o.y) * inv.y, y1 = (b[4] - o.y) * inv.y;
    const float z0 = (b[2] - o.z) * inv.z, z1 = (b[5] - o.z) * inv.z;
    const float tn = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)),
                                     __builtin_fmaxf(__builtin_fminf(z0, z1), tmin));
    const float tf = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)),
                                     __builtin_fminf(__builtin_fmaxf(z0, z1), bt));
    tnear = tn;
    return tn <= tf;
}

// One leaf: its (at most kBvhLeafMax) triangles are loaded before any is tested, so the
// leaf costs one memory round trip instead of one per triangle.  The leaf-ordered triangles
// are packed as 10 floats per slot (v0, e1, e2, face id bits; leaves start at even slots, so
// 16-B aligned, rvcp_host.cpp): ceil(2.5 cnt) 16-B loads.
constexpr uint32_t kBvhLeafChunk = 4;   // triangles loaded together (one round trip; 2: 2 % slower)
template <uint32_t kCh = kBvhLeafChunk>
__device__ __forceinline__ void bvh_leaf(const TriRecord *__restrict__ btri, int32_t ref, f3 o, f3 d,
                                         float tmin, float &bt, int &best, uint32_t slots = 0) {
    const uint32_t code = ~(uint32_t)ref;
    const uint32_t first = code >> 5, cnt = (code & 31u) + 1u;
    for (uint32_t c0 = 0; c0 < cnt; c0 += kCh) {
        const float4 *base = reinterpret_cast<const float4 *>(
            reinterpret_cast<const float *>(btri + slots) + 10u * (first + c0));
        const uint32_t nc = cnt - c0 < kCh ? cnt - c0 : kCh;
        const uint32_t nld = (10u * nc + 3u) >> 2;
        float4 W[(10 * kCh + 3) / 4];
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)((10 * kCh + 3) / 4); ++k)
            if (k < nld) W[k] = base[k];
        const float *F = reinterpret_cast<const float *>(W);
#pragma unroll
        for (uint32_t k = 0; k < kCh; ++k) {
            if (k < nc) {
                TriRecord T;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    T.v0[c] = F[10 * k + c];
                    T.e1[c] = F[10 * k + 3 + c];
                    T.e2[c] = F[10 * k + 6 + c];
                }
                float t;
                const int id = __float_as_int(F[10 * k + 9]);
                if (tri_accept(T, o, d, tmin, bt, t) && (t < bt || id > best)) {
                    bt = t;
                    best = id;
                }
            }
        }
    }
}

__device__ __forceinline__ f3 slab_inv(f3 d) {
    return mk(__builtin_amdgcn_rcpf(d.x != 0.0f ? d.x : 1e-30f),
              __builtin_amdgcn_rcpf(d.y != 0.0f ? d.y : 1e-30f),
              __builtin_amdgcn_rcpf(d.z != 0.0f ? d.z : 1e-30f));
}

typedef __attribute__((address_space(3))) int32_t lds_i32;
#ifndef RVCP_BVH_NEAREST_BREAK_REL
#define RVCP_BVH_NEAREST_BREAK_REL 40
#endif

// 4-wide traversal (rvcp_bvh.cpp), over the byte-quantised nodes (Bvh4QNode, 64 B: four 16-B
// loads in flight together per step).  A step tests the node's four boxes, sorts the children
// by entry distance (5-comparator network, misses keyed +inf), pushes the hit ones but the
// nearest -- farthest first -- and continues with the nearest.  Leaves are tested by bvh_leaf.
// The slab test may cull only boxes entered beyond the current nearest hit (tn > bt): the hit
// rule keeps a later face at equal t, so a box entered exactly at bt must still be visited.
// Each child bound is decoded straight into slab time, t = q * (scale * inv) + (origin - o) *
// inv, with the near and far bytes chosen by the sign of the ray's inverse direction (the
// ordered slab test: an inverted unused child is never entered); the roundings of that form
// are relative errors of a few ulp of t, far below the build's box enlargement, and a NaN from
// it only widens a slab, so nothing a float box keeps is culled.  (The 128-B float nodes the
// quantised ones come from measured 180 vs 151 ms per C5 frame)
// LDS = true: the stack is the caller's LDS column (stk[i * kBlock]; the lanes of a wave hit
// distinct banks whatever their depths); LDS = false: a private array (the pre-pass kernel,
// whose 1024-thread blocks would need 128 KiB of LDS).
__device__ __forceinline__ void bvh4_cas(float &ka, int32_t &ca, float &kb, int32_t &cb) {
    const bool sw = kb < ka;
    const float k = sw ? kb : ka;
    const int32_t c = sw ? cb : ca;
    kb = sw ? ka : kb;
    cb = sw ? ca : cb;
    ka = k;
    ca = c;
}

__device__ __forceinline__ float ubyte_f(uint32_t w, int c) { return (float)((w >> (8 * c)) & 0xFFu); }

template <bool LDS>
__device__ __noinline__ void bvh_nearest(const Bvh4Node *__restrict__ nodes,
                                         const TriRecord *__restrict__ btri, int32_t root,
                                         lds_i32 *stk, f3 o, f3 d, float tmin, float &bt,
                                         int &best, uint32_t n4 = 0, uint32_t slots = 0) {
    const f3 inv = slab_inv(d);
    int32_t priv[LDS ? 1 : kBvhStack];
    int sp = 0;
    int32_t ref = root;
    const Bvh4QNode *__restrict__ qn = reinterpret_cast<const Bvh4QNode *>(nodes + n4);
    const bool px = inv.x >= 0.0f, py = inv.y >= 0.0f, pz = inv.z >= 0.0f;
    // Speculative while-while: a lane that reaches a leaf parks it and keeps stepping through
    // nodes until every lane holds a parked leaf (or cannot step), then the wave tests the
    // parked leaves together -- node steps and leaf tests each run with most lanes active
    // instead of the wave paying for both whenever its lanes are mixed.  Culling uses the bt
    // of the tests done so far, which is never below the final one, so nothing is lost; the
    // order rule makes the nearest hit independent of the order leaves are tested in.
    bool alive = true, parked = false;
    int32_t lref = 0;
    for (;;) {
        for (;;) {
            if (alive && ref < 0 && !parked) {
                parked = true;
                lref = ref;
                if (sp == 0) alive = false;
                else { sp -= 1; ref = LDS ? stk[sp * kBlock] : priv[sp]; }
            }
            const bool step = alive && ref >= 0;
            if (!__any(step) || __all(parked || !alive)) break;
#if RVCP_BVH_NEAREST_BREAK_REL > 0
            // as bvh_pool's node phase (RVCP_BVH_NODE_BREAK_REL)
            if (__popcll(__ballot(step)) * 64u <= (unsigned)RVCP_BVH_NEAREST_BREAK_REL * (unsigned)__popcll(__ballot(alive)) &&
                __any(parked)) break;
#endif
            if (step) {
                const float4 *q = reinterpret_cast<const float4 *>(qn + ref);
                const float4 w0 = q[0], w1 = q[1], w2 = q[2];
                const int4 r = reinterpret_cast<const int4 *>(qn + ref)[3];
                const float ax = w0.w * inv.x, ay = w1.x * inv.y, az = w1.y * inv.z;
                const float bx = (w0.x - o.x) * inv.x, by = (w0.y - o.y) * inv.y, bz = (w0.z - o.z) * inv.z;
                const uint32_t lx = __float_as_uint(w1.z), ly = __float_as_uint(w1.w), lz = __float_as_uint(w2.x);
                const uint32_t hx = __float_as_uint(w2.y), hy = __float_as_uint(w2.z), hz = __float_as_uint(w2.w);
                const uint32_t nx = px ? lx : hx, fx = px ? hx : lx;
                const uint32_t ny = py ? ly : hy, fy = py ? hy : ly;
                const uint32_t nz = pz ? lz : hz, fz = pz ? hz : lz;
                float kk[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float tn = __builtin_fmaxf(
                        __builtin_fmaxf(__builtin_fmaf(ubyte_f(nx, c), ax, bx), __builtin_fmaf(ubyte_f(ny, c), ay, by)),
                        __builtin_fmaxf(__builtin_fmaf(ubyte_f(nz, c), az, bz), tmin));
                    const float tf = __builtin_fminf(
                        __builtin_fminf(__builtin_fmaf(ubyte_f(fx, c), ax, bx), __builtin_fmaf(ubyte_f(fy, c), ay, by)),
                        __builtin_fminf(__builtin_fmaf(ubyte_f(fz, c), az, bz), bt));
                    kk[c] = tn <= tf ? tn : __builtin_inff();
                }
                float k0 = kk[0], k1 = kk[1], k2 = kk[2], k3 = kk[3];
                int32_t c0 = r.x, c1 = r.y, c2 = r.z, c3 = r.w;
                bvh4_cas(k0, c0, k1, c1);
                bvh4_cas(k2, c2, k3, c3);
                bvh4_cas(k0, c0, k2, c2);
                bvh4_cas(k1, c1, k3, c3);
                bvh4_cas(k1, c1, k2, c2);
                const float inf = __builtin_inff();
                if (k3 < inf) { if (LDS) stk[sp * kBlock] = c3; else priv[sp] = c3; sp += 1; }
                if (k2 < inf) { if (LDS) stk[sp * kBlock] = c2; else priv[sp] = c2; sp += 1; }
                if (k1 < inf) { if (LDS) stk[sp * kBlock] = c1; else priv[sp] = c1; sp += 1; }
                if (k0 < inf) ref = c0;
                else if (sp == 0) alive = false;
                else { sp -= 1; ref = LDS ? stk[sp * kBlock] : priv[sp]; }
            }
        }
        if (parked) {
            bvh_leaf(btri, lref, o, d, tmin, bt, best, slots);
            parked = false;
        }
        if (!__any(alive)) break;
    }
}

// One 4-wide node step of a lane (the body of bvh_nearest's node branch): pushes the hit
// children but the nearest, continues with the nearest or pops; `alive` drops when the stack
// is empty.
__device__ __forceinline__ void bvh4_step(const Bvh4QNode *__restrict__ qn, lds_i32 *stk, f3 o,
                                          f3 inv, bool px, bool py, bool pz, float tmin, float bt,
                                          int32_t &ref, int &sp, bool &alive) {
    const float4 *q = reinterpret_cast<const float4 *>(qn + ref);
    const float4 w0 = q[0], w1 = q[1], w2 = q[2];
    const int4 r = reinterpret_cast<const int4 *>(qn + ref)[3];
    const float ax = w0.w * inv.x, ay = w1.x * inv.y, az = w1.y * inv.z;
    const float bx = (w0.x - o.x) * inv.x, by = (w0.y - o.y) * inv.y, bz = (w0.z - o.z) * inv.z;
    const uint32_t lx = __float_as_uint(w1.z), ly = __float_as_uint(w1.w), lz = __float_as_uint(w2.x);
    const uint32_t hx = __float_as_uint(w2.y), hy = __float_as_uint(w2.z), hz = __float_as_uint(w2.w);
    const uint32_t nx = px ? lx : hx, fx = px ? hx : lx;
    const uint32_t ny = py ? ly : hy, fy = py ? hy : ly;
    const uint32_t nz = pz ? lz : hz, fz = pz ? hz : lz;
    float kk[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float tn = __builtin_fmaxf(
            __builtin_fmaxf(__builtin_fmaf(ubyte_f(nx, c), ax, bx), __builtin_fmaf(ubyte_f(ny, c), ay, by)),
            __builtin_fmaxf(__builtin_fmaf(ubyte_f(nz, c), az, bz), tmin));
        const float tf = __builtin_fminf(
            __builtin_fminf(__builtin_fmaf(ubyte_f(fx, c), ax, bx), __builtin_fmaf(ubyte_f(fy, c), ay, by)),
            __builtin_fminf(__builtin_fmaf(ubyte_f(fz, c), az, bz), bt));
        kk[c] = tn <= tf ? tn : __builtin_inff();
    }
    float k0 = kk[0], k1 = kk[1], k2 = kk[2], k3 = kk[3];
    int32_t c0 = r.x, c1 = r.y, c2 = r.z, c3 = r.w;
    bvh4_cas(k0, c0, k1, c1);
    bvh4_cas(k2, c2, k3, c3);
    bvh4_cas(k0, c0, k2, c2);
    bvh4_cas(k1, c1, k3, c3);
    bvh4_cas(k1, c1, k2, c2);
    const float inf = __builtin_inff();
    if (k3 < inf) { stk[sp * kBlock] = c3; sp += 1; }
    if (k2 < inf) { stk[sp * kBlock] = c2; sp += 1; }
    if (k1 < inf) { stk[sp * kBlock] = c1; sp += 1; }
    if (k0 < inf) ref = c0;
    else if (sp == 0) alive = false;
    else { sp -= 1; ref = stk[sp * kBlock]; }
}

// Wave-pooled traversal (bvh_pool): the wave's new shadow rays (lanes nA, in lane order) and
// path rays (nB) form one list of up to 128 rays; every lane takes the next untaken ray as soon
// as its current one is finished, with the speculative while-while steps of bvh_nearest, so a
// wave's 64 lanes share its rays instead of each waiting for its own longest traversal.  A
// ray's (o, d) is read from its owner lane's registers (ds_bpermute via the wave's LDS table of
// owners, tab[128]), its (t, face) is left in res[2 owner + (path ray)] and read back by the
// owner.  Same traversal per ray, so the same nearest hits.
// (inlined into the path kernel with two-triangle leaf loads: 112 VGPRs without spills, C5
// BVH 138 -> 97.5 ms per frame, profiles/history/r03zj_bvh_pool_ab.log, r03zk_bvh_pool_ab.log)
//
// Carried traversals: once every new ray is taken and at most kBvhCarryMax lanes still hold an
// unfinished one, the pool may stop and let the wave go on with its next iteration; those lanes
// keep their traversal (BvhCarry, its stack stays in the lane's LDS column) and resume it first
// in the next call.  A wave's iteration otherwise lasts as long as its longest traversal, with
// most lanes idle at the end (lane utilisation 0.30 in C5).  The owner of an unfinished ray is
// `frozen`: it neither resolves nor emits rays until all its submitted rays have results (a
// result slot holds the face -2 until written).  Carrying is allowed only while the frame
// queue still has pixels and the call took at least kBvhCarryMinRays new rays, so each call
// makes progress and the last iterations drain everything.
constexpr uint32_t kBvhPoolChunk = 2;      // leaf triangles loaded together in bvh_pool
// The node phase of the speculative while-while loop also ends once at most
// RVCP_BVH_NODE_BREAK_REL / 64 of the lanes holding a ray can still step and some lane holds a
// parked leaf: the parked lanes test their leaves instead of idling behind the few still
// descending.  C5 with the BVH 69.16 -> 52.06 ms per frame at 40 / 64 with 4-triangle leaves
// (32: 53.02, 48: 52.42; the absolute form, at most N stepping lanes: 54.6 ms at N = 36-40,
// 103 ms at 64 = if-if; profiles/history/r05u_ab_bvhnb.log, r05v_ab_bvhnb2.log, r05w_ab_bvhnb3.log);
// with 2-triangle leaves 48 / 64 is best (46.75 ms; 40: 47.03, 52: 47.36, 56: 49.38,
// profiles/history/r05zf_ab_bvhtune2.log, r05zg_ab_bvhtune3.log).  Leaf order does not change a nearest hit (the
// order rule), so neither does the schedule.
#ifndef RVCP_BVH_NODE_BREAK_REL
#define RVCP_BVH_NODE_BREAK_REL 48
#endif
#ifndef RVCP_BVH_CARRY_MAX
#define RVCP_BVH_CARRY_MAX 48
#endif
#ifndef RVCP_BVH_CARRY_MIN_RAYS
#define RVCP_BVH_CARRY_MIN_RAYS 32
#endif
constexpr uint32_t kBvhCarryMax = RVCP_BVH_CARRY_MAX;
constexpr uint32_t kBvhCarryMinRays = RVCP_BVH_CARRY_MIN_RAYS;
struct BvhCarry {
    bool has = false;       // holds an unfinished traversal
    uint32_t key = 0;       // its result slot: owner lane * 2 + (path ray ? 1 : 0)
    int32_t ref = 0;        // next node (>= 0) or leaf (< 0)
    int sp = 0;             // stack depth (the stack is the lane's LDS column)
    float bt = 0.0f;
    int best = -1;
    float stop = 0.0f;      // a shadow ray ends once bt <= stop (shadow_stop); -inf: never
};

// The shadow ray's early end (bvh_pool).  Resolve A (:447-449) only asks whether
// |dist - |hp - p|| < eps, hp = a_o + a_d t at the nearest hit t.  With a_o = p + ws eps (rounded)
// and a_d = ws, the computed |hp - p| is at most (eps + t)(1 + 8u) + 10 u M for any t in
// [0, dist] (u = 2^-24, M = max |p_k| + eps + dist: the rounding of a_o, of a_d t, of the sum, of
// hp - p, of the dot product and of the root), so every hit with t <= stop below -- the one
// found and the nearest, which is no farther -- gives |hp - p| <= dist - eps: the light sample
// is blocked either way, and the traversal may end at the first such hit.  The margin is
// 2^-18 (M + dist + eps), four times what that bound needs, so the float evaluation of stop
// (a few ulps of dist) stays inside it.  t_min < 0 (hits behind the origin) or a non-finite
// dist: never (-inf / NaN compare false).
__device__ __forceinline__ float shadow_stop(float eps, float t_min, f3 p, float dist) {
    const float M = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(p.x), __builtin_fabsf(p.y)),
                                    __builtin_fabsf(p.z)) + eps + dist;
    const float stop = dist - 2.0f * eps - 0x1p-18f * (M + dist + eps);
    return t_min >= 0.0f ? stop : -__builtin_inff();
}
__device__ __forceinline__ void bvh_pool(const Bvh4Node *__restrict__ nodes,
                                      const TriRecord *__restrict__ btri, int32_t root,
                                      lds_i32 *stk, uint8_t *tab, float2 *res, uint32_t lane,
                                      bool nA_, bool nB_, f3 a_o, f3 a_d, f3 b_o, f3 b_d,
                                      float tmin, float tmax, bool may_carry, BvhCarry &c,
                                      bool &subA, bool &subB, bool &frozen, float &btA, int &bestA,
                                      float &btB, int &bestB, uint32_t n4, uint32_t slots,
                                      float ibtA, int ibestA, float ibtB, int ibestB,
                                      float istopA) {
    const uint64_t mA = __ballot(nA_), mB = __ballot(nB_);
    const uint32_t nA = (uint32_t)__builtin_popcountll(mA);
    const uint32_t nr = nA + (uint32_t)__builtin_popcountll(mB);
    const float2 pending = make_float2(tmax, __int_as_float(-2));
    if (nA_) { tab[rank_in(mA)] = (uint8_t)lane; res[2 * lane] = pending; subA = true; }
    if (nB_) { tab[nA + rank_in(mB)] = (uint8_t)lane; res[2 * lane + 1] = pending; subB = true; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool carry_ok = may_carry && nr >= kBvhCarryMinRays;      // wave-uniform
    const Bvh4QNode *__restrict__ qn = reinterpret_cast<const Bvh4QNode *>(nodes + n4);
    uint32_t next = 0;                  // the list's next untaken ray (wave-uniform)
    bool alive = c.has, parked = false;
    f3 o = mk(0, 0, 0), inv = mk(1, 1, 1), d = mk(0, 0, 1);
    bool px = true, py = true, pz = true;
    int32_t lref = 0;
    if (__any(c.has)) {                 // resume the carried traversals: their rays' (o, d)
        const int src = c.has ? (int)(c.key >> 1) : (int)lane;
        const f3 oa = mk(__shfl(a_o.x, src), __shfl(a_o.y, src), __shfl(a_o.z, src));
        const f3 da = mk(__shfl(a_d.x, src), __shfl(a_d.y, src), __shfl(a_d.z, src));
        const f3 ob = mk(__shfl(b_o.x, src), __shfl(b_o.y, src), __shfl(b_o.z, src));
        const f3 db = mk(__shfl(b_d.x, src), __shfl(b_d.y, src), __shfl(b_d.z, src));
        if (c.has) {
            const bool isA = (c.key & 1u) == 0u;
            o = isA ? oa : ob;
            d = isA ? da : db;
            inv = slab_inv(d);
            px = inv.x >= 0.0f; py = inv.y >= 0.0f; pz = inv.z >= 0.0f;
        }
    }
    for (;;) {
        const uint64_t M = __ballot(!c.has);
        if (M && next < nr) {
            const uint32_t k = rank_in(M);
            const bool take = !c.has && next + k < nr;
            const uint32_t rr = next + k;
            const int src = take ? (int)tab[rr] : (int)lane;
            const f3 oa = mk(__shfl(a_o.x, src), __shfl(a_o.y, src), __shfl(a_o.z, src));
            const f3 da = mk(__shfl(a_d.x, src), __shfl(a_d.y, src), __shfl(a_d.z, src));
            const f3 ob = mk(__shfl(b_o.x, src), __shfl(b_o.y, src), __shfl(b_o.z, src));
            const f3 db = mk(__shfl(b_d.x, src), __shfl(b_d.y, src), __shfl(b_d.z, src));
            // the ray's starting bound and candidate: t_max / none, or the hybrid prefix's hit
            const float i_tA = __shfl(ibtA, src), i_tB = __shfl(ibtB, src);
            const int i_bA = __shfl(ibestA, src), i_bB = __shfl(ibestB, src);
            const float i_sA = __shfl(istopA, src);
            if (take) {
                const bool isA = rr < nA;
                c.key = 2u * (uint32_t)src + (isA ? 0u : 1u);
                o = isA ? oa : ob;
                d = isA ? da : db;
                inv = slab_inv(d);
                px = inv.x >= 0.0f; py = inv.y >= 0.0f; pz = inv.z >= 0.0f;
                c.ref = root;
                c.sp = 0;
                c.bt = isA ? i_tA : i_tB;
                c.best = isA ? i_bA : i_bB;
                c.stop = isA ? i_sA : -__builtin_inff();
                c.has = true;
                // (a shadow ray the hybrid prefix already blocked needs no traversal)
                alive = !(c.bt <= c.stop);
                parked = false;
            }
            const uint32_t pm = (uint32_t)__builtin_popcountll(M);
            next += pm < nr - next ? pm : nr - next;
        }
        if (!__any(c.has)) break;
        // node phase: step until every lane with a ray holds a parked leaf or is finished
        for (;;) {
            if (c.has && alive && c.ref < 0 && !parked) {
                parked = true;
                lref = c.ref;
                if (c.sp == 0) alive = false;
                else { c.sp -= 1; c.ref = stk[c.sp * kBlock]; }
            }
            const bool step = c.has && alive && c.ref >= 0;
            if (!__any(step) || __all(!c.has || parked || !alive)) break;
#if RVCP_BVH_NODE_BREAK_REL > 0
            // few lanes still stepping while the parked ones wait: test the parked leaves now
            if (__popcll(__ballot(step)) * 64u <= (unsigned)RVCP_BVH_NODE_BREAK_REL * (unsigned)__popcll(__ballot(c.has)) &&
                __any(parked)) break;
#endif
            if (step) bvh4_step(qn, stk, o, inv, px, py, pz, tmin, c.bt, c.ref, c.sp, alive);
        }
        if (parked) {
            bvh_leaf<kBvhPoolChunk>(btri, lref, o, d, tmin, c.bt, c.best, slots);
            parked = false;
            if (c.bt <= c.stop) alive = false;      // a shadow ray already blocked (shadow_stop)
        }
        if (c.has && !alive) {          // this ray is done: leave its result for the owner
            res[c.key] = make_float2(c.bt, __int_as_float(c.best));
            c.has = false;
        }
        if (carry_ok && next >= nr &&
            (uint32_t)__builtin_popcountll(__ballot(c.has)) <= kBvhCarryMax)
            break;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float2 va = res[2 * lane], vb = res[2 * lane + 1];
    const bool readyA = !subA || __float_as_int(va.y) != -2;
    const bool readyB = !subB || __float_as_int(vb.y) != -2;
    frozen = !(readyA && readyB);
    if (!frozen) {
        if (subA) { btA = va.x; bestA = __float_as_int(va.y); }
        if (subB) { btB = vb.x; bestB = __float_as_int(vb.y); }
        subA = false;
        subB = false;
    }
}

// Hit record of face `best` for ray (o, d) hit at time t (:262-278).
__device__ __forceinline__ void hit_record(const TriRecord *__restrict__ tri,
                                           const rvcp_face_t *__restrict__ faces,
                                           const rvcp_vertex_t *__restrict__ verts, int best,
                                           f3 o, f3 d, float t, f3 &pos, f3 &n, uint32_t &mat) {
    const rvcp_face_t F = faces[best];
    const TriRecord T = tri[best];
    const f3 s = mk(o.x - T.v0[0], o.y - T.v0[1], o.z - T.v0[2]);
    const f3 e1 = ld3(T.e1), e2 = ld3(T.e2);
    const f3 s1 = cross(d, e2);
    const f3 s2 = cross(s, e1);
    const float f = rcp_ieee(dot(s1, e1));
    const float b1 = f * dot(s1, s);
    const float b2 = f * dot(s2, d);
    const f3 n0 = ld3(verts[F.vertices[0]].normal);
    const f3 n1 = ld3(verts[F.vertices[1]].normal);
    const f3 n2 = ld3(verts[F.vertices[2]].normal);
    n = normalize(add(add(muls(n0, 1.0f - b1 - b2), muls(n1, b1)), muls(n2, b2)));
    if (dot(n, d) > 0.0f) n = neg(n);
    pos = add(o, muls(d, t));
    mat = F.material_id;
}

// uv of shard-local pixel `pix` (main :487-488); stripes of 8 rows are dealt round-robin.
__device__ __forceinline__ void pixel_uv(const FrameArgs &A, uint32_t pix, float &u_, float &v_) {
    const uint32_t lr = pix / A.width;
    const uint32_t x = pix - lr * A.width;
    const uint32_t gy = ((lr >> 3) * A.shard_count + A.shard_index) * 8u + (lr & 7u);
    u_ = ((float)x + 0.5f) / (float)A.width;
    v_ = ((float)gy + 0.5f) / (float)A.height;
}

// A frame's camera constants and time seed: FrameArgs' own, or a batch frame's FrameCam
// (FrameArgs::batch_cams, integrator mode 2 batches)
struct Cam {
    f3 cam_pos, u, v, pos;
    float base_len, t_near, t_far, time;
};
__device__ __forceinline__ Cam cam_of(const FrameArgs &A) {
    return Cam{ld3(A.cam_pos), ld3(A.u), ld3(A.v), ld3(A.pos), A.base_len, A.t_near, A.t_far, A.time};
}
__device__ __forceinline__ Cam cam_load(const float *__restrict__ c) {
    return Cam{ld3(c), ld3(c + 3), ld3(c + 6), ld3(c + 9), c[12], c[13], c[14], c[15]};
}

// srand, :153-155
__device__ __forceinline__ float pixel_seed(const Cam &C, float u_, float v_) {
    const float sa = fractf(pt_sinf(C.time) * 43758.5453f);
    const float sb = fractf(pt_sinf(u_) * 22578.5453f);
    const float sc = fractf(pt_sinf(v_) * 114514.1919f);
    return fractf(sa + sb + sc);
}
__device__ __forceinline__ float pixel_seed(const FrameArgs &A, float u_, float v_) {
    return pixel_seed(cam_of(A), u_, v_);
}

// sample_ray, :217-235 (frame constants from the host)
__device__ __forceinline__ void primary_ray(const Cam &C, float u_, float v_, f3 &o, f3 &d,
                                            float &tmin, float &tmax) {
    const f3 uv_pos = add(add(C.pos, muls(C.u, u_ - 0.5f)), muls(C.v, v_ - 0.5f));
    const f3 dv = sub(uv_pos, C.cam_pos);
    const float t_coef = len(dv) / C.base_len;
    o = C.cam_pos;
    d = normalize(dv);
    tmin = C.t_near * t_coef;
    tmax = C.t_far * t_coef;
}
__device__ __forceinline__ void primary_ray(const FrameArgs &A, float u_, float v_, f3 &o, f3 &d,
                                            float &tmin, float &tmax) {
    primary_ray(cam_of(A), u_, v_, o, d, tmin, tmax);
}

// Hit record of face `best` from its FaceShade record (same arithmetic as hit_record).
__device__ __forceinline__ void hit_shade(const TriRecord *__restrict__ tri,
                                          const FaceShade *__restrict__ shade, int best, f3 o,
                                          f3 d, float t, f3 &pos, f3 &n, FaceShade &fs) {
    const TriRecord T = tri[best];
    fs = shade[best];
    const f3 s = mk(o.x - T.v0[0], o.y - T.v0[1], o.z - T.v0[2]);
    const f3 e1 = ld3(T.e1), e2 = ld3(T.e2);
    const f3 s1 = cross(d, e2);
    const f3 s2 = cross(s, e1);
    const float f = rcp_ieee(dot(s1, e1));
    const float b1 = f * dot(s1, s);
    const float b2 = f * dot(s2, d);
    n = normalize(add(add(muls(ld3(fs.n0), 1.0f - b1 - b2), muls(ld3(fs.n1), b1)),
                      muls(ld3(fs.n2), b2)));
    if (dot(n, d) > 0.0f) n = neg(n);
    pos = add(o, muls(d, t));
}

// Primary ray of pixel `pix` (main :486-491): srand + sample_ray.
__device__ __forceinline__ void start_pixel(const FrameArgs &A, uint32_t pix, float &seed,
                                            float &ridx, f3 &o, f3 &d, float &tmin, float &tmax) {
    float u_, v_;
    pixel_uv(A, pix, u_, v_);
    seed = pixel_seed(A, u_, v_);
    ridx = 0.0f;
    primary_ray(A, u_, v_, o, d, tmin, tmax);
}
// The same for queue pixel `pix` of a mode-2 batch (FrameArgs::batch_cams): pixel
// pix % frame_pixels of frame pix / frame_pixels, with that frame's camera and time.
__device__ __forceinline__ void start_batch_pixel(const FrameArgs &A, uint32_t pix, float &seed,
                                                  float &ridx, f3 &o, f3 &d, float &tmin,
                                                  float &tmax) {
    const uint32_t f = pix / A.frame_pixels;
    const Cam C = cam_load(A.batch_cams + 16u * f);
    float u_, v_;
    pixel_uv(A, pix - f * A.frame_pixels, u_, v_);
    seed = pixel_seed(C, u_, v_);
    ridx = 0.0f;
    primary_ray(C, u_, v_, o, d, tmin, tmax);
}
__device__ __forceinline__ void start_any(const FrameArgs &A, uint32_t pix, float &seed,
                                          float &ridx, f3 &o, f3 &d, float &tmin, float &tmax) {
    if (A.batch_cams) start_batch_pixel(A, pix, seed, ridx, o, d, tmin, tmax);
    else start_pixel(A, pix, seed, ridx, o, d, tmin, tmax);
}
// Output index of queue pixel `pix` (frame f's outputs start f * frame_stride pixels in).
__device__ __forceinline__ uint32_t batch_out(const FrameArgs &A, uint32_t pix) {
    if (!A.batch_cams) return pix;
    const uint32_t f = pix / A.frame_pixels;
    return pix + f * (A.frame_stride - A.frame_pixels);
}

// NEE half of a surface event (:431-440 + sample_light_games101 :384-404): the light sample,
// the contribution C the shadow ray will add if it sees the sample (:450-458), and the
// shadow ray direction.  Returns false when there is no luminous face.
__device__ __forceinline__ bool nee_sample(const FrameArgs &A, const LightRecord *__restrict__ lights,
                                           f3 alb_pi, f3 S_pos, f3 S_nrm, f3 att,
                                           float seed, float &ridx, f3 &C, float &dist, f3 &ws) {
    const float pl = rnd(seed, ridx) * A.light_total;
    f3 Lv0, Lv1, Lv2, Ln, Lle;
    if (A.lights_same) {
        // every record samples the same face, and pl <= the last cum always holds (pl =
        // rand * total <= total, the same sum), so the pick is record 0: wave-uniform reads
        const LightRecord &L = lights[0];
        Lv0 = ld3(L.v0); Lv1 = ld3(L.v1); Lv2 = ld3(L.v2); Ln = ld3(L.n); Lle = ld3(L.le);
    } else {
        uint32_t li = A.n_lights;
        for (uint32_t i = 0; i < A.n_lights; ++i) {
            if (pl <= lights[i].cum) { li = i; break; }
        }
        if (li >= A.n_lights) return false;
        const LightRecord &L = lights[li];
        Lv0 = ld3(L.v0); Lv1 = ld3(L.v1); Lv2 = ld3(L.v2); Ln = ld3(L.n); Lle = ld3(L.le);
    }
    const float x = sqrt_c(rnd(seed, ridx));                                       // :319
    const float y = rnd(seed, ridx);                                               // :320
    const f3 Xp = add(add(muls(Lv0, 1.0f - x), muls(Lv1, x * (1.0f - y))),
                      muls(Lv2, x * y));                                           // :324
    const f3 dv = sub(Xp, S_pos);
    {   // dist = length(dv) (:438), ws = dv / dist (:439): as normalize, the root's guard makes
        // the fast reciprocal of dist exact and puts dist in quot_box's range, so one guard
        // (with the components' box) covers the root, the reciprocal and the quotients
        const float x2 = dot(dv, dv);
        dist = sqrt_fast_core(x2);
        const float y0 = __builtin_amdgcn_rcpf(dist);
        const float y = __builtin_fmaf(__builtin_fmaf(-dist, y0, 1.0f), y0, y0);
        ws = mk(quot_refine(dv.x, dist, y), quot_refine(dv.y, dist, y), quot_refine(dv.z, dist, y));
        if (__builtin_expect(!(sqrt_fast_ok(x2) & quot_box(dv)), 0)) {
            dist = len(dv);
            ws = divs_pos(dv, dist);
        }
    }
    const float cosp = dot(S_nrm, ws);
    const f3 f = cosp > 0.0f ? alb_pi : mk(0, 0, 0);                               // :344-349
    C = mulv(mulv(att, Lle), f);                                                   // :450-458
    C = muls(C, cosp);
    C = muls(C, dot(Ln, neg(ws)));
    C = divs_pos(C, dist * dist * A.light_pdf);
    return true;
}

// Continuation half of a surface event (:461-471): Russian roulette, the uniform hemisphere
// direction and the attenuation update.  Returns false when the path ends at RR.
__device__ __forceinline__ bool brdf_continue(const FrameArgs &A, const MatRecord &m, f3 S_nrm,
                                              float seed, float &ridx, f3 &att, f3 &wi) {
    if (rnd(seed, ridx) > A.rr) return false;                                      // :462
    f3 p;
    do {                                                                           // :195-201
        const float rx = rnd(seed, ridx);
        const float ry = rnd(seed, ridx);
        const float rz = rnd(seed, ridx);
        p = mk(cube_coord(rx), cube_coord(ry), cube_coord(rz));
    } while (dot(p, p) >= 1.0f);
    const f3 h = dot(p, S_nrm) > 0.0f ? p : neg(p);                                // :207-210
    wi = normalize(h);                                                             // :212-214
    const float cosw = dot(S_nrm, wi);
    const f3 f = cosw > 0.0f ? ld3(m.alb_pi) : mk(0, 0, 0);
    const float pdf = dot(wi, S_nrm) > 0.0f ? 0.5f / 3.1415926f : 0.0f;            // :358-365
    const float denom = __builtin_fmaxf(0.1f, pdf) * A.rr;
    att = mulv(att, divs_pos(muls(f, cosw), denom));                                   // :465-471
    return true;
}

// Continuation, after the direction: the attenuation update of :465-471 for direction wi
// (wi = normalize(h), h the hemisphere-flipped unit-ball sample, :207-214).
// dot(wi, S_nrm) is dot(S_nrm, wi) bit for bit (each product commutes), so the pdf test is the
// cosine test and the divisor is one of two frame constants (FrameArgs::brdf_den, whose IEEE
// reciprocals the host computed: divs_y with them is divs_pos).
__device__ __forceinline__ void brdf_finish(const FrameArgs &A, f3 alb_pi, f3 S_nrm, f3 p,
                                            f3 &att, f3 &wi) {
    const f3 h = dot(p, S_nrm) > 0.0f ? p : neg(p);
    wi = normalize(h);
    const float cosw = dot(S_nrm, wi);
    const bool pos = cosw > 0.0f;
    const f3 f = pos ? alb_pi : mk(0, 0, 0);
    att = mulv(att, divs_y(muls(f, cosw), pos ? A.brdf_den[1] : A.brdf_den[0],
                           pos ? A.brdf_rcp[1] : A.brdf_rcp[0]));
}

// random_in_unit_sphere (:195-201) for every lane with `need`, cooperatively: each round the
// n lanes still rejecting get K = 2^floor(log2(64/n)) lanes, which evaluate K consecutive
// candidates of the OWNER's rand() stream (candidate c uses indices ridx+3c+1..ridx+3c+3, the
// exact integers the sequential loop would reach by +1.0f steps).  The owner keeps the first
// accepted candidate in stream order and advances ridx just past it, so the result and the
// rand() index are bit-identical to the do-while; a wave needs ~3 rounds instead of the ~7
// its unluckiest lane needs sequentially.  Wave-uniform control flow; `tab` is this wave's
// 64-byte LDS scratch.
__device__ __forceinline__ void coop_unit_sphere(bool need, float seed, float &ridx, f3 &p_out,
                                                 uint32_t lane, uint8_t *tab) {
    for (;;) {
        const uint64_t M = __ballot(need);
        if (M == 0ull) break;
        const uint32_t n = (uint32_t)__builtin_popcountll(M);
        if (n > kWave / 2) {
            // K = 1: every lane still rejecting tests its own next candidate -- the same
            // candidate the compacted form below would hand it, without the LDS round trips
            const float rx = rand_of(seed + (ridx + 1.0f));
            const float ry = rand_of(seed + (ridx + 2.0f));
            const float rz = rand_of(seed + (ridx + 3.0f));
            const f3 p = mk(cube_coord(rx), cube_coord(ry), cube_coord(rz));
            if (need) {
                ridx = ridx + 3.0f;
                if (!(dot(p, p) >= 1.0f)) {
                    p_out = p;
                    need = false;
                }
            }
            continue;
        }
        // floor(log2(64 / n)) = 6 - ceil(log2 n) (64 / n >= 2^k <=> n <= 2^(6-k)), from the
        // wave-uniform n without an integer division; at most 32 candidates per lane (n = 1
        // leaves half the wave idle, a 0.476^32 chance of another round), so that every owner's
        // segment of the acceptance ballot lies in one 32-bit half
        const uint32_t lgK0 = 6u - (n > 1u ? 32u - (uint32_t)__builtin_clz(n - 1u) : 0u);
        const uint32_t lgK = lgK0 < 5u ? lgK0 : 5u;
        const uint32_t K = 1u << lgK;
        const uint32_t r = rank_in(M);
        if (need) tab[r] = (uint8_t)lane;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t j = lane >> lgK, c = lane & (K - 1u);
        const bool worker = j < n;
        const int owner = worker ? (int)tab[j] : (int)lane;
        const float s_seed = __shfl(seed, owner);
        const float base = __shfl(ridx, owner) + (float)(3u * c);
        const float rx = rand_of(s_seed + (base + 1.0f));
        const float ry = rand_of(s_seed + (base + 2.0f));
        const float rz = rand_of(s_seed + (base + 3.0f));
        const f3 p = mk(cube_coord(rx), cube_coord(ry), cube_coord(rz));
        // (the acceptance and the worker masks ANDed in scalar registers: a ballot of the
        // combined predicate materialised it in a VGPR and compared it again)
        const uint64_t AM = __builtin_amdgcn_ballot_w64(!(dot(p, p) >= 1.0f)) &
                            __builtin_amdgcn_ballot_w64(worker);
        // this owner's K acceptance bits (workers r K .. r K + K - 1, K <= 32)
        const uint32_t off = r << lgK;
        const uint32_t segmask = K >= 32u ? ~0u : ((1u << K) - 1u);
        const uint32_t seg = (uint32_t)(AM >> off) & segmask;
        const bool got = need && seg != 0u;
        const uint32_t cstar = (uint32_t)__builtin_ctz(seg | 0x80000000u);   // seg != 0: its lowest bit
        const int src = got ? (int)(off + cstar) : (int)lane;
        const f3 pp = mk(__shfl(p.x, src), __shfl(p.y, src), __shfl(p.z, src));
        if (got) {
            p_out = pp;
            ridx = ridx + (float)(3u * (cstar + 1u));
            need = false;
        } else if (need) {
            ridx = ridx + (float)(3u * K);
        }
    }
}

__device__ __forceinline__ bool att_stop(const FrameArgs &A, f3 att) {          // :415-419
    return att.x < A.att_stop && att.y < A.att_stop && att.z < A.att_stop;
}


// Static chunks: full 64-pixel waves (fewest wave-instructions for the work) unless that
// leaves fewer than two waves per SIMD, in which case the pixels are spread over up to two
// waves per SIMD, at least kMinStatic each (latency hiding matters more for tiny frames).  Returns the waves that get a static chunk and its size.
__host__ __device__ inline void static_split(uint32_t n, uint32_t grid_waves, uint32_t n_simds,
                                             uint32_t &waves, uint32_t &chunk) {
    uint32_t w = (n + kChunk - 1) / kChunk;
    const uint32_t spread = (n + kMinStatic - 1) / kMinStatic;
    const uint32_t floor_w = spread < 2u * n_simds ? spread : 2u * n_simds;
    if (w < floor_w) w = floor_w;
    if (w > grid_waves) w = grid_waves;
    if (w < 1u) w = 1u;
    uint32_t c = (n + w - 1) / w;
    chunk = c < 1u ? 1u : (c > kChunk ? kChunk : c);
    waves = w;
}

// Wave-uniform frame-queue state: [next, end) pixels owned by this wave; the pixels it has
// handed to its lanes since t0 (s_memrealtime ticks) set the size of its next grab.
struct Queue {
    uint32_t next, end;
    uint32_t taken;
    uint64_t t0;
    bool exhausted;
};

__device__ __forceinline__ Queue queue_init(const FrameArgs &A) {
    const uint32_t wave_global =
        __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) / kWave);
    Queue q;
    q.next = wave_global * A.static_chunk;
    q.end = q.next + A.static_chunk;
    if (q.next > A.n_pixels) q.next = A.n_pixels;
    if (q.end > A.n_pixels) q.end = A.n_pixels;
    q.taken = 0;
    q.t0 = __builtin_amdgcn_s_memrealtime();
    q.exhausted = false;
    return q;
}

// Hand pixels to the lanes in `need` (must be called in wave-uniform control flow).  Lanes
// that receive one get got=true and their pixel index.
//
// Grab size: pixels a wave grabs but has not yet handed out wait for ITS lanes to free up
// (a pixel is a serial chain of SPP samples), so when the queue runs dry a large grab strands
// up to a grab's worth of work behind busy lanes while other waves idle.  Each wave therefore
// grabs what it consumes in a short window: chunk = clamp(rate x chunk_window, chunk_min,
// dyn_chunk), rate = pixels it handed out / time since its start.  Expensive pixels (C3: ~4)
// keep the stranded tail short; cheap ones (mode 2: 64) keep the head atomic uncontended.
__device__ __forceinline__ void queue_take(Queue &q, uint64_t need, uint32_t lane,
                                           const FrameArgs &A,
                                           unsigned long long *__restrict__ counters,
                                           bool &got, uint32_t &pix) {
    got = false;
    while (need != 0ull) {
        if (q.next >= q.end) {
            if (q.exhausted) break;
            const int leader = (int)__builtin_ctzll(need);
            const uint64_t dt = __builtin_amdgcn_s_memrealtime() - q.t0 + 1ull;
            const uint64_t want = (uint64_t)q.taken * A.chunk_window / dt;
            uint32_t c = want > A.dyn_chunk ? A.dyn_chunk : (uint32_t)want;
            c = __builtin_amdgcn_readfirstlane(c < A.chunk_min ? A.chunk_min : c);
            uint32_t base = 0;
            if (lane == (uint32_t)leader) base = atomicAdd((unsigned int *)&counters[1], c);
            base = __builtin_amdgcn_readfirstlane(__shfl(base, leader)) + A.static_chunks;
            if (base >= A.n_pixels) { q.exhausted = true; break; }
            q.next = base;
            q.end = base + c < A.n_pixels ? base + c : A.n_pixels;
        }
        const uint32_t avail = q.end - q.next;
        const uint32_t r = rank_in(need);
        const bool mine = ((need >> lane) & 1ull) && r < avail;
        const uint64_t given = __ballot(mine);
        if (mine) { pix = q.next + r; got = true; }
        q.next += __builtin_popcountll(given);
        q.taken += __builtin_popcountll(given);
        need &= ~given;
    }
}

// Mode 2's pixel starts (srand's three sines, sample_ray's root and divisions: ~150 VALU per
// pixel, main :486-491), computed for a whole grab at once, one pixel per lane, into this wave's
// 64 LDS slots, instead of per pixel when a lane takes it -- in the persistent kernel a few lanes
// take a pixel in most iterations, so the start ran at a few lanes per instruction.  A slot holds
// (d, seed) and (o, t_min) + t_max; a lane taking pixel p reads slot p - base.  Each pixel's
// start is the same arithmetic as before, so the frames are unchanged.
#ifndef RVCP_LEGACY_PREFILL
#define RVCP_LEGACY_PREFILL 1
#endif
struct StartSlot {
    float4 ds;      // d.xyz, seed
    float4 ot;      // o.xyz, t_min
    float tmax;
};
__device__ __forceinline__ void start_any(const FrameArgs &A, uint32_t pix, float &seed,
                                          float &ridx, f3 &o, f3 &d, float &tmin, float &tmax);
__device__ __forceinline__ void prefill_starts(const FrameArgs &A, uint32_t base, uint32_t n,
                                               uint32_t lane, StartSlot *slots) {
    if (lane < n) {
        float seed, ridx, tmin, tmax;
        f3 o, d;
        start_any(A, base + lane, seed, ridx, o, d, tmin, tmax);
        slots[lane].ds = make_float4(d.x, d.y, d.z, seed);
        slots[lane].ot = make_float4(o.x, o.y, o.z, tmin);
        slots[lane].tmax = tmax;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// queue_take for mode 2 with prefilled starts: a lane that gets pixel `pix` also gets its start
// (read from its slot before the next grab refills the slots).
__device__ __forceinline__ void queue_take_started(Queue &q, uint64_t need, uint32_t lane,
                                                   const FrameArgs &A,
                                                   unsigned long long *__restrict__ counters,
                                                   StartSlot *slots, uint32_t &base, bool &got,
                                                   uint32_t &pix, float &seed, float &ridx, f3 &o,
                                                   f3 &d, float &tmin, float &tmax) {
    got = false;
    while (need != 0ull) {
        if (q.next >= q.end) {
            if (q.exhausted) break;
            const int leader = (int)__builtin_ctzll(need);
            const uint64_t dt = __builtin_amdgcn_s_memrealtime() - q.t0 + 1ull;
            const uint64_t want = (uint64_t)q.taken * A.chunk_window / dt;
            uint32_t c = want > A.dyn_chunk ? A.dyn_chunk : (uint32_t)want;
            c = __builtin_amdgcn_readfirstlane(c < A.chunk_min ? A.chunk_min : c);
            uint32_t b = 0;
            if (lane == (uint32_t)leader) b = atomicAdd((unsigned int *)&counters[1], c);
            b = __builtin_amdgcn_readfirstlane(__shfl(b, leader)) + A.static_chunks;
            if (b >= A.n_pixels) { q.exhausted = true; break; }
            q.next = b;
            q.end = b + c < A.n_pixels ? b + c : A.n_pixels;
            base = b;
            prefill_starts(A, base, q.end - base, lane, slots);
        }
        const uint32_t avail = q.end - q.next;
        const uint32_t r = rank_in(need);
        const bool mine = ((need >> lane) & 1ull) && r < avail;
        const uint64_t given = __ballot(mine);
        if (mine) {
            pix = q.next + r;
            got = true;
            const StartSlot &S = slots[pix - base];
            const float4 ds = S.ds, ot = S.ot;
            d = mk(ds.x, ds.y, ds.z);
            seed = ds.w;
            o = mk(ot.x, ot.y, ot.z);
            tmin = ot.w;
            tmax = S.tmax;
            ridx = 0.0f;
        }
        // the slots a later grab overwrites have been read (wave-ordered LDS accesses)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        q.next += __builtin_popcountll(given);
        q.taken += __builtin_popcountll(given);
        need &= ~given;
    }
}

// Wave-level counters already summed over the lanes (kept in SGPRs by the caller).
__device__ __forceinline__ void flush_wave_counters(unsigned long long *__restrict__ counters,
                                                    uint32_t lane, uint32_t trav_wave,
                                                    uint32_t iters) {
    if (lane == 0) {
        atomicAdd(&counters[0], (unsigned long long)trav_wave);
        atomicAdd(&counters[2], (unsigned long long)iters);
    }
}
// The shader clock the kernel ran at, measured in the product kernel itself (bench.py's
// roofline.shader_clock_ghz): the first wave of every workgroup of a path kernel stamps
// s_memtime (shader-clock ticks) and s_memrealtime (100 MHz) when it starts and when it ends,
// and lane 0 accumulates (sum of the end stamps - sum of the start stamps) in
// counters[kClockWord] / [kClockWord + 1] with vector atomics (unsigned wrap-around makes the
// two halves of the difference separable, so no stamp is held across the kernel: no register
// cost; a cache line of their own, away from the queue head's atomics).  The host reports their
// quotient x 0.1 GHz (rvcp_stats_t::shader_clock_ghz), the wave-time-weighted mean clock.
__device__ __forceinline__ void clock_stamp(unsigned long long *__restrict__ counters,
                                            uint32_t lane, bool first_wave, bool end) {
#ifdef RVCP_NO_CLOCK_STAMP
    return;         // A/B only (tools/ab_cases/stamp.txt)
#endif
    if (!first_wave) return;
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
        atomicAdd(&counters[kClockWord], end ? c : 0ull - c);
        atomicAdd(&counters[kClockWord + 1], end ? r : 0ull - r);
    }
}
__device__ __forceinline__ void flush_counters(unsigned long long *__restrict__ counters,
                                               uint32_t lane, uint32_t trav, uint32_t iters) {
    unsigned long long t64 = trav;
    for (int off = 32; off >= 1; off >>= 1) t64 += __shfl_xor(t64, off);
    if (lane == 0) {
        atomicAdd(&counters[0], t64);
        atomicAdd(&counters[2], (unsigned long long)iters);
    }
}

// Lane actions of the single-ray machine.
enum : int { A_TRACE = 0, A_RR = 1, A_END = 2, A_SURF = 3, A_NEED = 4, A_DONE = 5 };
// Kinds of a traced ray.
enum : int { K_NONE = -1, K_PRIMARY = 0, K_PATH = 1, K_SHADOW = 2 };

}  // namespace

#ifndef RVCP_JIT   // the scene-specialised module (rvcp_jit.cpp) holds only the path kernels
// ======================================================================================
// Variant 1: one ray per lane per iteration
// ======================================================================================
__global__ __launch_bounds__(kBlock) void games101_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters)
{
    const uint32_t lane = lane_id();
    Queue q = queue_init(A);
    const float sppf = (float)A.spp;
    const float inv_spp = rcp_ieee(sppf);     // divs_y's shared reciprocal

    int action = A_NEED, kind = K_PRIMARY;
    uint32_t pix = 0, k = 0, depth = 0, trav = 0, iters = 0;
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
            if (action == A_RR) {                                   // :461-478
                f3 wi;
                if (!brdf_continue(A, mats[S_mat], S_nrm, seed, ridx, att, wi)) {
                    action = A_END;
                } else {
                    depth += 1;
                    ro = add(S_pos, muls(wi, A.eps));
                    rd = wi;
                    rtmin = A.t_min;
                    rtmax = A.t_max;
                    kind = K_PATH;
                    action = (depth >= A.max_bounces || att_stop(A, att)) ? A_END : A_TRACE;
                }
            }
            if (action == A_END) {                                  // color += L / SPP (:495)
                acc = add(acc, divs_y(col, sppf, inv_spp));
                k += 1;
                if (k >= A.spp) {
                    store_pixel(pix, acc, A, gamma_t, out_rgba, out_lin);
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
            if (action == A_SURF) {                                 // :431-447
                f3 ws;
                if (!nee_sample(A, lights, ld3(mats[S_mat].alb_pi), S_pos, S_nrm, att, seed, ridx,
                                nee_C, nee_dist, ws)) {
                    action = A_RR;
                } else {
                    ro = add(S_pos, muls(ws, A.eps));
                    rd = ws;
                    rtmin = A.t_min;
                    rtmax = A.t_max;
                    kind = K_SHADOW;
                    action = A_TRACE;
                }
            }
            {   // take new pixels from the frame queue (wave-uniform control flow)
                bool got;
                uint32_t np = pix;
                queue_take(q, __ballot(action == A_NEED), lane, A, counters, got, np);
                if (got) {
                    pix = np;
                    start_pixel(A, pix, seed, ridx, ro, rd, rtmin, rtmax);
                    kind = K_PRIMARY;
                    k = 0;
                    acc = mk(0, 0, 0);
                    action = A_TRACE;
                }
            }
            if (q.exhausted && action == A_NEED) action = A_DONE;
            if (!__any(action == A_RR || action == A_END || action == A_SURF)) break;
        }
        if (!__any(action == A_TRACE)) break;
        iters += 1;

        // ============ trace: brute-force nearest hit (:283-298) ============
        int best = -1;
        float bt = rtmax;
        if (action == A_TRACE) {
            trav += 1;
            for (uint32_t i = 0; i < A.n_faces; ++i) {
                float t;
                if (tri_accept(tri[i], ro, rd, rtmin, bt, t)) { bt = t; best = (int)i; }
            }
        }

        // ============ post-trace shading ============
        if (action == A_TRACE) {
            if (kind == K_SHADOW) {                                 // :447-459
                const f3 hp = best >= 0 ? add(ro, muls(rd, bt))
                                        : mk(__builtin_inff(), __builtin_inff(), __builtin_inff());
                const float dist_blocked = len(sub(hp, S_pos));
                if (__builtin_fabsf(nee_dist - dist_blocked) < A.eps) col = add(col, nee_C);
                action = A_RR;
            } else {
                f3 hpos = mk(0, 0, 0), hn = mk(0, 0, 0);
                uint32_t hmat = 0;
                if (best >= 0) hit_record(tri, faces, verts, best, ro, rd, bt, hpos, hn, hmat);
                const bool miss = best < 0;
                const bool is_light = !miss && mats[hmat].ty == kLight;
                if (kind == K_PRIMARY) {
                    if (miss || is_light) {
                        // every sample returns the same L without touching the RNG:
                        // miss -> 0.1 (:424), light at depth 0 -> Le (:425-427)
                        const f3 L = miss ? mk(0.1f, 0.1f, 0.1f) : ld3(mats[hmat].albedo);
                        const f3 Ls = divs(L, sppf);
                        for (uint32_t i = 0; i < A.spp; ++i) acc = add(acc, Ls);
                        store_pixel(pix, acc, A, gamma_t, out_rgba, out_lin);
                        action = A_NEED;
                    } else {
                        P_pos = hpos; P_nrm = hn; P_mat = hmat;
                        S_pos = hpos; S_nrm = hn; S_mat = hmat;
                        depth = 0;
                        att = mk(1, 1, 1);
                        col = mk(0, 0, 0);
                        action = A_SURF;
                    }
                } else {                                            // K_PATH
                    if (miss) {
                        col = add(col, mk(0.1f, 0.1f, 0.1f));
                        action = A_END;
                    } else if (is_light) {
                        action = A_END;     // depth >= 1: no emission term (:426)
                    } else {
                        S_pos = hpos; S_nrm = hn; S_mat = hmat;
                        action = A_SURF;
                    }
                }
            }
        }
    }
    flush_counters(counters, lane, trav, iters);
}

// ======================================================================================
// Variant 2: a surface event emits its shadow ray (A) and its continuation ray (B); both are
// traced by one scan.  The RNG stream of a path does not depend on the shadow result, so
// sampling the continuation before the shadow ray is resolved keeps every rand() in order;
// the NEE term of bounce d is added before the miss/emission term of bounce d+1, as in the
// shader.
// ======================================================================================
__global__ __launch_bounds__(kBlock) void games101_dual_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters)
{
    const uint32_t lane = lane_id();
    Queue q = queue_init(A);
    const float sppf = (float)A.spp;
    const float inv_spp = rcp_ieee(sppf);     // divs_y's shared reciprocal

    bool need_pixel = true, done = false;
    uint32_t pix = 0, k = 0, depth = 0, trav = 0, iters = 0;
    float seed = 0.0f, ridx = 0.0f;
    f3 acc = mk(0, 0, 0), att = mk(1, 1, 1), col = mk(0, 0, 0);
    f3 P_pos = mk(0, 0, 0), P_nrm = mk(0, 0, 0);
    uint32_t P_mat = 0;
    // ray A: pending shadow ray of the last surface event
    bool hasA = false;
    f3 a_o = mk(0, 0, 0), a_d = mk(0, 0, 1), a_p = mk(0, 0, 0), nee_C = mk(0, 0, 0);
    float nee_dist = 0.0f;
    // ray B: primary or continuation ray
    int kindB = K_NONE;
    f3 b_o = mk(0, 0, 0), b_d = mk(0, 0, 1);
    float b_tmin = 0.0f, b_tmax = 0.0f;

    for (;;) {
        // ---- new pixels (wave-uniform) ----
        {
            bool got;
            uint32_t np = pix;
            queue_take(q, __ballot(need_pixel && !done), lane, A, counters, got, np);
            if (got) {
                pix = np;
                start_pixel(A, pix, seed, ridx, b_o, b_d, b_tmin, b_tmax);
                kindB = K_PRIMARY;
                hasA = false;
                k = 0;
                acc = mk(0, 0, 0);
                need_pixel = false;
            } else if (need_pixel && q.exhausted) {
                done = true;
            }
        }
        if (!__any(hasA || kindB != K_NONE)) break;
        iters += 1;

        // ---- scan: both rays against every triangle ----
        int bestA = -1, bestB = -1;
        float btA = A.t_max, btB = b_tmax;
        trav += (hasA ? 1u : 0u) + (kindB != K_NONE ? 1u : 0u);
#pragma unroll 2
        for (uint32_t i = 0; i < A.n_faces; ++i) {
            const TriRecord T = tri[i];
            float tA, tB;
            if (tri_accept(T, a_o, a_d, A.t_min, btA, tA)) { btA = tA; bestA = (int)i; }
            if (tri_accept(T, b_o, b_d, b_tmin, btB, tB)) { btB = tB; bestB = (int)i; }
        }

        // ---- resolve A: visibility of the light sample (:447-459) ----
        if (hasA) {
            const f3 hp = bestA >= 0 ? add(a_o, muls(a_d, btA))
                                     : mk(__builtin_inff(), __builtin_inff(), __builtin_inff());
            const float dist_blocked = len(sub(hp, a_p));
            if (__builtin_fabsf(nee_dist - dist_blocked) < A.eps) col = add(col, nee_C);
        }

        // ---- resolve B ----
        bool surf = false, ended = false;
        f3 S_pos = P_pos, S_nrm = P_nrm;
        uint32_t S_mat = P_mat;
        if (kindB != K_NONE) {
            f3 hpos = mk(0, 0, 0), hn = mk(0, 0, 0);
            uint32_t hmat = 0;
            if (bestB >= 0) hit_record(tri, faces, verts, bestB, b_o, b_d, btB, hpos, hn, hmat);
            const bool miss = bestB < 0;
            const bool is_light = !miss && mats[hmat].ty == kLight;
            if (kindB == K_PRIMARY) {
                if (miss || is_light) {
                    const f3 L = miss ? mk(0.1f, 0.1f, 0.1f) : ld3(mats[hmat].albedo);
                    const f3 Ls = divs(L, sppf);
                    for (uint32_t i = 0; i < A.spp; ++i) acc = add(acc, Ls);
                    store_pixel(pix, acc, A, gamma_t, out_rgba, out_lin);
                    need_pixel = true;
                } else {
                    P_pos = hpos; P_nrm = hn; P_mat = hmat;
                    S_pos = hpos; S_nrm = hn; S_mat = hmat;
                    depth = 0;
                    att = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    surf = true;
                }
            } else {                                                    // K_PATH
                if (miss) {
                    col = add(col, mk(0.1f, 0.1f, 0.1f));
                    ended = true;
                } else if (is_light) {
                    ended = true;
                } else {
                    S_pos = hpos; S_nrm = hn; S_mat = hmat;
                    surf = true;
                }
            }
        } else if (hasA) {
            ended = true;       // the path ended at its last surface event (RR / depth / att)
        }
        hasA = false;
        kindB = K_NONE;

        // ---- end samples and emit the next surface event (loops only without lights) ----
        for (;;) {
            if (ended) {
                ended = false;
                acc = add(acc, divs_y(col, sppf, inv_spp));
                k += 1;
                if (k >= A.spp) {
                    store_pixel(pix, acc, A, gamma_t, out_rgba, out_lin);
                    need_pixel = true;
                } else {
                    depth = 0;
                    att = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    S_pos = P_pos; S_nrm = P_nrm; S_mat = P_mat;
                    surf = true;
                }
            }
            if (surf) {
                surf = false;
                const MatRecord m = mats[S_mat];
                f3 ws;
                if (nee_sample(A, lights, ld3(m.alb_pi), S_pos, S_nrm, att, seed, ridx, nee_C,
                               nee_dist, ws)) {
                    a_o = add(S_pos, muls(ws, A.eps));
                    a_d = ws;
                    a_p = S_pos;
                    hasA = true;
                }
                f3 wi;
                if (brdf_continue(A, m, S_nrm, seed, ridx, att, wi)) {
                    depth += 1;
                    if (!(depth >= A.max_bounces || att_stop(A, att))) {
                        b_o = add(S_pos, muls(wi, A.eps));
                        b_d = wi;
                        b_tmin = A.t_min;
                        b_tmax = A.t_max;
                        kindB = K_PATH;
                    }
                }
                if (!hasA && kindB == K_NONE) ended = true;
            }
            if (!__any(ended)) break;
        }
    }
    flush_counters(counters, lane, trav, iters);
}

#endif  // RVCP_JIT
// ======================================================================================
// Variant 3, kernel 1: primary pre-pass, one pixel per lane.  Traces every primary ray once
// (all lanes busy, no divergence), finishes miss / light pixels in closed form (their samples
// never touch the RNG, :424-428), and appends every other pixel with its primary hit record to
// a compact list for the path kernel (one atomic per wave).
// ======================================================================================
constexpr uint32_t kPrimaryBlock = 256;   // one list append (global atomic) per block

template <bool BVH, bool SPEC>
__device__ __forceinline__ void primary_body(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const float *__restrict__ gamma_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters,
    SurfRecord *__restrict__ surf, const FaceShade *__restrict__ shade,
    const Bvh4Node *__restrict__ bvh_nodes, const TriRecord *__restrict__ bvh_tris,
    const float *__restrict__ cams, uint32_t frame_stride)
{
    __shared__ uint32_t block_count, block_base;
    const uint32_t lane = lane_id();
    const uint32_t pix = blockIdx.x * kPrimaryBlock + threadIdx.x;
    // a batch's frames in one launch (cams != nullptr): frame blockIdx.y, its camera and time
    // from the call's 16-float records, its outputs frame_stride pixels after the previous one's
    const Cam C = cams ? cam_load(cams + 16u * blockIdx.y) : cam_of(A);
    const uint32_t pix_base = A.pix_base + blockIdx.y * frame_stride;
    const bool live = pix < A.n_pixels;
    if (threadIdx.x == 0) block_count = 0;
    __syncthreads();
    bool is_surf = false;
    f3 hpos = mk(0, 0, 0), hn = mk(0, 0, 0), halb = mk(0, 0, 0);
    uint32_t hmat = 0;
    float u_ = 0.0f, v_ = 0.0f;
    if (live) {
        float tmin, tmax;
        f3 o, d;
        pixel_uv(A, pix, u_, v_);
        primary_ray(C, u_, v_, o, d, tmin, tmax);
        int best = -1;
        float bt = tmax;
        if (BVH) {
            // the hybrid's prefix faces first (FrameArgs::bvh_prefix), then the BVH over the rest
            if (A.bvh_prefix) {
#ifdef RVCP_SPEC_SCAN
                if (SPEC && !__any(!(ray_in_range(o, d) && tmin > 0.0f))) {
                    spec_scan1(o, d, tmin, bt, best);
                } else
#endif
                for (uint32_t i = 0; i < A.bvh_prefix; ++i) {
                    float t;
                    if (tri_accept(tri[i], o, d, tmin, bt, t)) { bt = t; best = (int)i; }
                }
            }
            bvh_nearest<false>(bvh_nodes, bvh_tris, A.bvh_root, nullptr, o, d, tmin, bt, best, A.bvh_n4, A.bvh_slots);
        }
#ifdef RVCP_SPEC_SCAN
        // the scene-specialised scan (§4.7) where every primary ray of the wave is in its range
        // (ray_in_range, t_min > 0), as the path kernels' scans
        else if (SPEC && !__any(!(ray_in_range(o, d) && tmin > 0.0f))) {
            spec_scan1(o, d, tmin, bt, best);
        }
#endif
        else {
#pragma unroll 2
            for (uint32_t i = 0; i < A.n_faces; ++i) {
                float t;
                if (tri_accept(tri[i], o, d, tmin, bt, t)) { bt = t; best = (int)i; }
            }
        }
        FaceShade fs;
        fs.ty = 0;
        if (best >= 0) {
            hit_shade(tri, shade, best, o, d, bt, hpos, hn, fs);
            hmat = fs.mat;
            halb = ld3(fs.alb_pi);
        }
        const bool miss = best < 0;
        const bool is_light = !miss && fs.ty == kLight;
        if (miss || is_light) {
            const f3 L = miss ? mk(0.1f, 0.1f, 0.1f) : ld3(mats[hmat].albedo);
            const f3 Ls = divs(L, (float)A.spp);
            f3 acc = mk(0, 0, 0);
            for (uint32_t i = 0; i < A.spp; ++i) acc = add(acc, Ls);
            store_acc(pix_base + pix, acc, out_lin);
        } else {
            is_surf = true;
        }
    }
    // append the block's surface pixels to the list: LDS aggregation, one global atomic
    const uint64_t m = __ballot(is_surf);
    uint32_t wave_off = 0;
    if (lane == 0 && m) wave_off = atomicAdd(&block_count, (uint32_t)__builtin_popcountll(m));
    wave_off = __shfl(wave_off, 0);
    __syncthreads();
    if (threadIdx.x == 0) {
        block_base = block_count ? atomicAdd((unsigned int *)&counters[3], block_count) : 0u;
        const uint32_t lim = A.n_pixels - blockIdx.x * kPrimaryBlock;
        atomicAdd(&counters[0], (unsigned long long)(lim < kPrimaryBlock ? lim : kPrimaryBlock));
    }
    __syncthreads();
    if (is_surf) {
        SurfRecord r;
        r.pos[0] = hpos.x; r.pos[1] = hpos.y; r.pos[2] = hpos.z; r.pix = pix_base + pix;
        r.nrm[0] = hn.x; r.nrm[1] = hn.y; r.nrm[2] = hn.z; r.seed = pixel_seed(C, u_, v_);
        r.alb_pi[0] = halb.x; r.alb_pi[1] = halb.y; r.alb_pi[2] = halb.z; r.mat = hmat;
        surf[block_base + wave_off + rank_in(m)] = r;
    }
}

#ifndef RVCP_JIT
template <bool BVH>
__global__ __launch_bounds__(kPrimaryBlock) void games101_primary_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const float *__restrict__ gamma_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters,
    SurfRecord *__restrict__ surf, const FaceShade *__restrict__ shade,
    const Bvh4Node *__restrict__ bvh_nodes, const TriRecord *__restrict__ bvh_tris,
    const float *__restrict__ cams, uint32_t frame_stride)
{
    primary_body<BVH, false>(A, tri, faces, verts, mats, gamma_t, out_rgba, out_lin, counters,
                             surf, shade, bvh_nodes, bvh_tris, cams, frame_stride);
}
#endif

// ======================================================================================
// Variant 3/4, kernel 2: the dual-ray machine over the surface pixels of the pre-pass.  Every
// pixel starts with a surface event at its cached primary hit, so no iteration is spent on
// primary rays and every lane enters the scan with a shadow and (usually) a path ray.
//   TILED = false (variant 3): each wave scans the triangles with wave-uniform scalar loads
//           (the whole Cornell scene stays in the scalar cache);
//   TILED = true  (variant 4, large meshes): the workgroup's waves scan in lockstep over
//           triangle tiles that the workgroup loads once, coalesced, into LDS -- the triangle
//           stream is read from L2/HBM once per workgroup instead of once per wave.
// ======================================================================================
// Variant 4 is held to 4 waves per SIMD (128 VGPRs, a few spills around the tile loop): 5 %
// faster on C5 than the 3 waves its natural 146-155 VGPRs give.
// The BVH path kernel traces one ray per lane per iteration (the variant-5 form): C5 297 ->
// 283 ms over the dual form, whose second traversal leaves the lanes without a path ray idle.
constexpr int kTiledMinWaves = 4;
// The generic nearest-hit scans of the non-tiled path kernels: every triangle in index order
// (wave-uniform face index, the records in SGPRs), one ray (scan_generic1) or the lane's two
// (scan_generic2; slot A keeps its face only for SINGLE); FAST as tri_stage2.
template <bool FAST>
__device__ __forceinline__ void scan_generic1(const TriRecord *__restrict__ tri, uint32_t n, f3 o,
                                              f3 d, float tmin, float &bt, int &best) {
#pragma unroll 1
    for (uint32_t i = 0; i < n; ++i) {
        const TriRecord T = tri[i];
        float t;
        if (tri_accept<FAST>(T, o, d, tmin, bt, t)) { bt = t; best = (int)i; }
    }
}
template <bool FAST, bool SINGLE>
__device__ __forceinline__ void scan_generic2(const TriRecord *__restrict__ tri, uint32_t n,
                                              f3 a_o, f3 a_d, f3 b_o, f3 b_d, float tmin,
                                              float &btA, int &bestA, float &btB, int &bestB) {
#pragma unroll 1
    for (uint32_t i = 0; i < n; ++i) {
        const TriRecord T = tri[i];
        float tA, tB;
#ifndef RVCP_SPEC_NO_SKIP
        if (!SINGLE) {
            // the shadow slot as the specialised scan runs it (rvcp_jit.cpp emit_scan): t and its
            // range mask first, the barycentric half only when some lane of the wave is in range
            // (every other lane would reject on the mask); the same operations on the same values
            const f3 s = mk(a_o.x - T.v0[0], a_o.y - T.v0[1], a_o.z - T.v0[2]);
            const f3 e1 = ld3(T.e1);
            const f3 s1 = cross(a_d, ld3(T.e2));
            const f3 s2 = cross(s, e1);
            const float f = FAST ? rcp_scan_fast(dot(s1, e1)) : rcp_scan(dot(s1, e1));
            const float t = f * dot(s2, ld3(T.e2));
            const bool q = (t >= tmin) & (t <= btA);
            if (__builtin_amdgcn_ballot_w64(q) != 0ull) {
                const float b1 = f * dot(s1, s);
                const float b2 = f * dot(s2, a_d);
                if ((b1 >= 0.0f) & (b2 >= 0.0f) & (b1 + b2 <= 1.0f) & q) btA = t;
            }
        } else
#endif
        if (tri_accept<FAST>(T, a_o, a_d, tmin, btA, tA)) {
            btA = tA;
            if (SINGLE) bestA = (int)i;
        }
        if (tri_accept<FAST>(T, b_o, b_d, tmin, btB, tB)) { btB = tB; bestB = (int)i; }
    }
}
// The tiled scans issue the first pretest halves of two triangles together (ILP for the
// latency-bound per-triangle chain; C5 -5 %); the one-slot schedule 5 too (3
// and 4 triangles per step measured equal to 2).
// The BVH hybrid's prefix (FrameArgs::bvh_prefix = K > 0: faces [0, K) are not in the BVH):
// the new rays of the wave (nA: the shadow ray a, nB: the path ray b) are tested against
// faces [0, K) first, with the specialised scan of the module (which covers exactly those
// faces) when every new ray is in its range, else with the generic test; each ray then enters
// the BVH with that nearest hit as its bound and candidate -- and the BVH's rule (smaller t,
// or equal t and larger face) combines them as the brute-force scan's order would.  The
// specialised dual scan keeps no face for the shadow slot (as in the brute-force dual scan):
// a prefix hit is face 0 for the order rule -- resolve A needs only hit / no hit -- and a
// nearest t of exactly t_max is settled by a generic re-scan that keeps the face.
// SPEC_A = false (SINGLE): the shadow slot may hold a path ray, which needs its face.
template <bool SPEC_A>
__device__ __forceinline__ void bvh_prefix_scan(const FrameArgs &A, const TriRecord *__restrict__ tri,
                                                bool nA, bool nB, f3 a_o, f3 a_d, f3 b_o, f3 b_d,
                                                float &btA, int &bestA, float &btB, int &bestB) {
    const uint32_t K = A.bvh_prefix;
    btA = A.t_max;
    bestA = -1;
    btB = A.t_max;
    bestB = -1;
#ifdef RVCP_SPEC_SCAN
    if (SPEC_A && A.t_min > 0.0f &&
        !__any((nA && !ray_in_range(a_o, a_d)) || (nB && !ray_in_range(b_o, b_d)))) {
        float sa = nA ? A.t_max : -1.0f;        // a lane without a new shadow ray: below t_min
        spec_scan2(a_o, a_d, b_o, b_d, A.t_min, sa, btB, bestB);
        const bool rescan = nA && sa == A.t_max;
        if (nA) { btA = sa; bestA = sa != A.t_max ? 0 : -1; }
        if (__builtin_expect(__any(rescan), 0)) {
            float t2 = A.t_max;
            int b2 = -1;
            for (uint32_t i = 0; i < K; ++i) {
                float t;
                if (tri_accept(tri[i], a_o, a_d, A.t_min, t2, t) && rescan) { t2 = t; b2 = (int)i; }
            }
            if (rescan) { btA = t2; bestA = b2; }
        }
        return;
    }
#endif
    for (uint32_t i = 0; i < K; ++i) {
        float t;
        if (nA && tri_accept(tri[i], a_o, a_d, A.t_min, btA, t)) { btA = t; bestA = (int)i; }
        if (nB && tri_accept(tri[i], b_o, b_d, A.t_min, btB, t)) { btB = t; bestB = (int)i; }
    }
}

// The variant-3 path kernel runs 5 waves per SIMD: 95 VGPRs without spills once the scan loop
// is not unrolled and the pixel's surface record is re-read per sample instead of held in
// registers (C3 5.93 -> 5.73 ms, C4 44.2 -> 41.3 ms, C2 unchanged, over 105 VGPRs / 4 waves;
// tools/ab.sh).  Forcing 6 waves spills 26 VGPRs and is slower.
constexpr int kPathMinWaves = 5;
// LDS_STATE: the light sample's pending state (a_p, nee_C, nee_dist: written at the surface
// event, read when the shadow ray resolves) and the pixel's running sum `acc` live in this
// lane's column of an LDS block (SoA, stride = the block size) instead of 10 VGPRs across the
// scan.
// POOL_W > 0 (schedule 10, with TILED): the workgroup of POOL_W waves pools its rays in LDS
// every iteration and scans them in 64-ray passes shared out over its waves.
template <bool TILED, bool BVH, bool SINGLE = false, bool LDS_STATE = false, int POOL_W = 0>
__device__ __forceinline__ void path_body(
    const FrameArgs &A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade, uint8_t (*tail_tab)[kWave], TriRecord *tile,
    const Bvh4Node *__restrict__ bvh_nodes = nullptr, const TriRecord *__restrict__ bvh_tris = nullptr,
    int32_t *bvh_stack = nullptr, float4 *compact_lds = nullptr, float *state_lds = nullptr,
    float4 *pool = nullptr, uint32_t *pool_count = nullptr)
{
    static_assert(POOL_W == 0 || TILED, "the workgroup ray pool is built for the tiled scan");
    constexpr int BLK = POOL_W ? POOL_W * kWave : kBlock;     // threads per workgroup
    float *const st = LDS_STATE ? state_lds + threadIdx.x : nullptr;   // st[f * BLK]
    auto st_put3 = [&](int f, f3 v) { st[f * BLK] = v.x; st[(f + 1) * BLK] = v.y; st[(f + 2) * BLK] = v.z; };
    auto st_get3 = [&](int f) { return mk(st[f * BLK], st[(f + 1) * BLK], st[(f + 2) * BLK]); };
    const uint32_t lane = lane_id();
    // this wave's index in the block, made wave-uniform (an SGPR) for the LDS row bases
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    clock_stamp(counters, lane, wv == 0, false);
    // the per-wave timeline (FrameArgs::timeline) exists in the debug build only (RVCP_TIMELINE,
    // also passed to its specialised modules): its clocks held across the kernel cost the
    // product kernel SGPRs, spilled into VGPR lanes read back inside the loop
#ifdef RVCP_TIMELINE
    const unsigned long long t_start = A.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const unsigned long long c_start = A.timeline ? __builtin_amdgcn_s_memtime() : 0ull;
    unsigned long long t_exhausted = 0ull;
#endif
    // RVCP_REGION_CLOCK=k (debug builds of the specialised module only): shader-clock cycles this wave
    // spent in region k and in its iterations as a whole, summed (timeline rec[6..7]); regions:
    // 1 the scans, 2 the settle loop, 3 the resolve step, 4 the unit-ball sample + BRDF update,
    // 5 the light sample (nee_sample)
    unsigned long long c_scan = 0ull, c_iter = 0ull;
#ifdef RVCP_REGION_CLOCK
#define RC_BEGIN(k) const unsigned long long rc_t##k = (RVCP_REGION_CLOCK == k) ? __builtin_amdgcn_s_memtime() : 0ull
#define RC_END(k) do { if (RVCP_REGION_CLOCK == k) c_scan += __builtin_amdgcn_s_memtime() - rc_t##k; } while (0)
#else
#define RC_BEGIN(k) do {} while (0)
#define RC_END(k) do {} while (0)
#endif
    // the queue runs over the pre-pass's compact list; its length is in counters[3]
    FrameArgs Q = A;
    Q.n_pixels = __builtin_amdgcn_readfirstlane(*(volatile unsigned int *)&counters[3]);
    {   // static chunks over the surface list, same rule as the host's (static_split)
        uint32_t waves, c;
        const uint32_t grid_waves = gridDim.x * (BLK / kWave);
        static_split(Q.n_pixels, grid_waves, A.n_simds, waves, c);
        if (A.spread_min && Q.n_pixels <= grid_waves * kChunk) {
            // small frame: every resident wave gets a share (latency hiding over lane count)
            c = (Q.n_pixels + grid_waves - 1) / grid_waves;
            if (c < A.spread_min) c = A.spread_min;
            if (c > kChunk) c = kChunk;
            waves = (Q.n_pixels + c - 1) / c;
        }
        Q.static_chunk = c;
        Q.static_chunks = c * waves;
    }
    Queue q = queue_init(Q);
    const float sppf = (float)A.spp;
    const float inv_spp = rcp_ieee(sppf);     // divs_y's shared reciprocal

    bool need_pixel = true, done = false, ended = false, surf_ev = false;
    // the pixel's surface record (cached primary hit, pixel index) is re-read from the list at
    // each sample start instead of being held in 10 VGPRs for the whole pixel
    uint32_t pslot = 0, k = 0, depth = 0;
    uint32_t trav_wave = 0, iters = 0;      // wave-uniform: traversals of all lanes, iterations
    float seed = 0.0f, ridx = 0.0f;
    f3 acc = mk(0, 0, 0), att = mk(1, 1, 1), col = mk(0, 0, 0);
    f3 S_pos = mk(0, 0, 0), S_nrm = mk(0, 0, 0), S_alb = mk(0, 0, 0);
    bool hasA = false;
    f3 a_o = mk(0, 0, 0), a_d = mk(0, 0, 1), a_p = mk(0, 0, 0), nee_C = mk(0, 0, 0);
    float nee_dist = 0.0f;
    bool hasB = false;
    f3 b_o = mk(0, 0, 0), b_d = mk(0, 0, 1);
    // BVH pool (BVH, !SINGLE): rays submitted to the pool and not yet resolved, the traversal
    // this lane carries into the next iteration, and whether this lane waits on a carried ray
    constexpr bool CARRY = BVH && !SINGLE;
    bool subA = false, subB = false;
    BvhCarry carry;

    for (;;) {
#ifdef RVCP_REGION_CLOCK
        const unsigned long long c_top = __builtin_amdgcn_s_memtime();
#endif
        RC_BEGIN(2);
        // ---- settle: end samples, take pixels, emit surface events ----
        for (;;) {
            if (ended) {                                            // color += L / SPP (:495)
                ended = false;
                if (LDS_STATE) acc = st_get3(7);
                acc = add(acc, divs_y(col, sppf, inv_spp));
                if (LDS_STATE) st_put3(7, acc);
                k += 1;
                if (k >= A.spp) {
                    store_acc(surf[pslot].pix, acc, out_lin);
                    need_pixel = true;
                } else {
                    depth = 0;
                    att = mk(1, 1, 1);
                    if (LDS_STATE) st_put3(10, att);
                    col = mk(0, 0, 0);
                    if (LDS_STATE) st_put3(13, col);
                    const SurfRecord r = surf[pslot];
                    S_pos = ld3(r.pos); S_nrm = ld3(r.nrm); S_alb = ld3(r.alb_pi);
                    surf_ev = true;
                }
            }
            {   // new pixels (wave-uniform control flow)
                bool got;
                uint32_t slot = 0;
                queue_take(q, __ballot(need_pixel && !done), lane, Q, counters, got, slot);
                if (got) {
                    const SurfRecord r = surf[slot];
                    pslot = slot;
                    seed = r.seed;
                    ridx = 0.0f;
                    k = 0;
                    acc = mk(0, 0, 0);
                    if (LDS_STATE) st_put3(7, acc);
                    depth = 0;
                    att = mk(1, 1, 1);
                    if (LDS_STATE) st_put3(10, att);
                    col = mk(0, 0, 0);
                    if (LDS_STATE) st_put3(13, col);
                    S_pos = ld3(r.pos); S_nrm = ld3(r.nrm); S_alb = ld3(r.alb_pi);
                    need_pixel = false;
                    surf_ev = true;
                } else if (need_pixel && q.exhausted) {
                    done = true;
                }
            }
            bool need_dir = false;
            if (surf_ev) {                                          // :431-462
                surf_ev = false;
                if (LDS_STATE) att = st_get3(10);
                f3 ws;
                RC_BEGIN(5);
                const bool nee_ok = nee_sample(A, lights, S_alb, S_pos, S_nrm, att, seed, ridx,
                                               nee_C, nee_dist, ws);
                RC_END(5);
                if (nee_ok) {
                    a_o = add(S_pos, muls(ws, A.eps));
                    a_d = ws;
                    a_p = S_pos;
                    hasA = true;
                    if (LDS_STATE) {
                        st_put3(0, a_p);
                        st_put3(3, nee_C);
                        st[6 * BLK] = nee_dist;
                    }
                }
                need_dir = !(rnd(seed, ridx) > A.rr);               // Russian roulette :462
                if (!need_dir && !hasA) ended = true;
            }
            f3 p = mk(0, 0, 0);
            RC_BEGIN(4);
            coop_unit_sphere(need_dir, seed, ridx, p, lane, tail_tab[wv]);
            if (need_dir) {                                         // :464-478
                f3 wi;
                brdf_finish(A, S_alb, S_nrm, p, att, wi);
                if (LDS_STATE) st_put3(10, att);
                depth += 1;
                if (!(depth >= A.max_bounces || att_stop(A, att))) {
                    b_o = add(S_pos, muls(wi, A.eps));
                    b_d = wi;
                    hasB = true;
                }
                if (!hasA && !hasB) ended = true;
            }
            RC_END(4);
            if (!__any(ended)) break;
        }
        RC_END(2);
        // The shading point is dead until the next surface event sets it again (resolve B, or
        // a sample / pixel start): say so, so that it is not held in 9 VGPRs across the scan.
        S_pos = mk(0, 0, 0);
        S_nrm = mk(0, 0, 0);
        S_alb = mk(0, 0, 0);
        if (LDS_STATE) {       // likewise the attenuation and the sample's colour (LDS columns)
            att = mk(0, 0, 0);
            col = mk(0, 0, 0);
        }
        // The scan's view of the lane's rays.  SINGLE (variant 5): one ray per lane per
        // iteration -- the shadow ray A while it is pending, else the path ray B; a B left
        // pending is traced on the next iteration, without a new surface event.
        const bool sA = SINGLE ? (hasA || hasB) : hasA;
        const bool sB = SINGLE ? false : hasB;
        const f3 s_ao = (SINGLE && !hasA) ? b_o : a_o;
        const f3 s_ad = (SINGLE && !hasA) ? b_d : a_d;
        const uint64_t mA = __ballot(sA), mB = __ballot(sB);
        const bool wave_active = (mA | mB) != 0ull;
        // POOL_W: this wave's first A and B slots in the workgroup's ray pool and the pool's
        // size R (its A rays first, wave by wave, then its B rays)
        uint32_t pool_baseA = 0, pool_baseB = 0, pool_R = 0;
        if (POOL_W) {
            // every wave of the workgroup takes part in every iteration until the whole group
            // has no ray left (the pool is filled and scanned between workgroup barriers)
            if (lane == 0) {
                pool_count[2 * wv] = (uint32_t)__builtin_popcountll(mA);
                pool_count[2 * wv + 1] = (uint32_t)__builtin_popcountll(mB);
            }
            __syncthreads();
            uint32_t RA = 0, RB = 0;
#pragma unroll
            for (int v = 0; v < POOL_W; ++v) {
                const uint32_t ca = pool_count[2 * v], cb = pool_count[2 * v + 1];
                pool_baseA += (uint32_t)v < wv ? ca : 0u;
                pool_baseB += (uint32_t)v < wv ? cb : 0u;
                RA += ca;
                RB += cb;
            }
            pool_R = __builtin_amdgcn_readfirstlane(RA + RB);
            pool_baseA = __builtin_amdgcn_readfirstlane(pool_baseA);
            pool_baseB = __builtin_amdgcn_readfirstlane(pool_baseB + RA);
            if (pool_R == 0u) break;
        } else if (TILED) {
            // every wave of the workgroup keeps loading tiles until the whole group is done
            if (!__syncthreads_or(wave_active ? 1 : 0)) break;
        } else if (!wave_active) {
            break;
        }
        if (wave_active) iters += 1;
        // CARRY: a lane waiting on a carried ray keeps hasA / hasB without new traversals
        const bool newA = CARRY ? hasA && !subA : sA, newB = CARRY ? hasB && !subB : sB;
        trav_wave += CARRY ? (uint32_t)__builtin_popcountll(__ballot(newA)) +
                                 (uint32_t)__builtin_popcountll(__ballot(newB))
                           : (uint32_t)__builtin_popcountll(mA) + (uint32_t)__builtin_popcountll(mB);
        bool frozen = false;
#ifdef RVCP_TIMELINE
        if (A.timeline && q.exhausted && t_exhausted == 0ull) t_exhausted = __builtin_amdgcn_s_memrealtime();
#endif

        int bestA = -1, bestB = -1;
        float btA = A.t_max, btB = A.t_max;
        RC_BEGIN(1);
        const uint32_t na = (uint32_t)__builtin_popcountll(mA);
        const uint32_t nr = na + (uint32_t)__builtin_popcountll(mB);
        const bool tail = wave_active && (q.exhausted || A.early_tail) && nr <= kWave / 2 && !BVH &&
                          !POOL_W;
        if (TILED) {
            // ---- LDS-tiled scan (optionally with the tail partition below) ----
            // The scan's operands: slot 0 (so0, sd0; lanes m0) and slot 1 (so1, sd1; lanes m1)
            // are the lane's A and B rays, or with POOL_W the wave's passes of the workgroup
            // ray pool; `ttail`: R lanes per ray (o, d), each scanning every R-th triangle.
            // Workgroup ray pool (schedule 10): ray j of the pool is two float4s, (o, t) and
            // (d, face); the R rays are scanned in ceil(R / 64) passes of 64, pass p by wave p
            // mod POOL_W, as that wave's slots, so the workgroup's waves scan what it holds
            // instead of two slots per lane whether or not they hold a ray (the tiles are
            // streamed once per iteration either way).  When R is at most half the
            // workgroup's lanes, every ray gets R >= 2 lanes that scan every R-th triangle of
            // each tile (the tail partition).  Each ray meets the same triangles with the same
            // test wherever it is scanned, so every nearest hit is unchanged.
            f3 so0 = s_ao, sd0 = s_ad, so1 = b_o, sd1 = b_d;
            uint64_t m0 = mA, m1 = mB;
            // a slot's shadow ray leaves the scan's gates once a hit already blocks its light
            // sample (shadow_stop; -inf: a path ray, never); a wave whose slots are all settled
            // skips the tests of the remaining tiles (it still loads them with the workgroup)
#ifdef RVCP_NO_SHADOW_STOP
            const float my_stop = -__builtin_inff();
#else
            const float my_stop = hasA ? shadow_stop(A.eps, A.t_min, a_p, nee_dist) : -__builtin_inff();
#endif
            float stop0 = my_stop, stop1 = -__builtin_inff();
            bool ttail = tail;
            uint32_t R = 1, part = 0;
            bool worker = false;
            f3 o = s_ao, d = s_ad;
            uint32_t jA = 0, jB = 0, pj0 = 0, pj1 = 0;
            if (POOL_W) {
                // push the rays (as in the non-tiled pool above); the pool's passes become
                // this wave's slots, or every ray gets R lanes when the pool is small
                jA = pool_baseA + rank_in(mA);
                jB = pool_baseB + rank_in(mB);
                if (sA) {
                    pool[2 * jA] = make_float4(s_ao.x, s_ao.y, s_ao.z, my_stop);
                    pool[2 * jA + 1] = make_float4(s_ad.x, s_ad.y, s_ad.z, 0.0f);
                }
                if (sB) {
                    pool[2 * jB] = make_float4(b_o.x, b_o.y, b_o.z, -__builtin_inff());
                    pool[2 * jB + 1] = make_float4(b_d.x, b_d.y, b_d.z, 0.0f);
                }
                __syncthreads();
                if (pool_R * 2u <= (uint32_t)(POOL_W * kWave)) {
                    uint32_t lgK = 1;
                    while (lgK < 6u && (pool_R << (lgK + 1)) <= (uint32_t)(POOL_W * kWave)) lgK += 1;
                    R = 1u << lgK;
                    const uint32_t g = wv * kWave + lane;
                    pj0 = g >> lgK;
                    part = g & (R - 1u);
                    worker = pj0 < pool_R;
                    const uint32_t jj = worker ? pj0 : 0u;
                    const float4 ro = pool[2 * jj], rd = pool[2 * jj + 1];
                    o = mk(ro.x, ro.y, ro.z);
                    d = mk(rd.x, rd.y, rd.z);
                    ttail = true;
                    m0 = m1 = 0ull;
                } else {
                    ttail = false;
                    pj0 = wv * kWave + lane;
                    pj1 = (wv + POOL_W) * kWave + lane;
                    const bool v0 = pj0 < pool_R;
                    const bool v1 = pj1 < pool_R;
                    const uint32_t i0 = v0 ? pj0 : 0u, i1 = v1 ? pj1 : 0u;
                    const float4 o0r = pool[2 * i0], d0r = pool[2 * i0 + 1];
                    const float4 o1r = pool[2 * i1], d1r = pool[2 * i1 + 1];
                    so0 = mk(o0r.x, o0r.y, o0r.z);
                    sd0 = mk(d0r.x, d0r.y, d0r.z);
                    so1 = mk(o1r.x, o1r.y, o1r.z);
                    sd1 = mk(d1r.x, d1r.y, d1r.z);
                    stop0 = o0r.w;
                    stop1 = o1r.w;
                    m0 = __ballot(v0);
                    m1 = __ballot(v1);
                }
            } else if (tail) {
                R = 2;
                while (nr * R * 2 <= (uint32_t)kWave) R *= 2;
                uint8_t *tab = tail_tab[wv];
                if (sA) tab[rank_in(mA)] = (uint8_t)lane;
                if (sB) tab[na + rank_in(mB)] = (uint8_t)lane;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t j = lane / R;
                part = lane % R;
                worker = j < nr;
                const int owner = worker ? (int)tab[j] : (int)lane;
                const bool isA = j < na;
                const f3 oa = mk(__shfl(s_ao.x, owner), __shfl(s_ao.y, owner), __shfl(s_ao.z, owner));
                const f3 da = mk(__shfl(s_ad.x, owner), __shfl(s_ad.y, owner), __shfl(s_ad.z, owner));
                const f3 ob = mk(__shfl(b_o.x, owner), __shfl(b_o.y, owner), __shfl(b_o.z, owner));
                const f3 db = mk(__shfl(b_d.x, owner), __shfl(b_d.y, owner), __shfl(b_d.z, owner));
                o = isA ? oa : ob;
                d = isA ? da : db;
            }
            float bt = A.t_max;
            int best = -1;
            if (POOL_W) {        // slot results accumulate in btA/bestA (slot 0), btB/bestB (1)
                btA = btB = A.t_max;
                bestA = bestB = -1;
            }
            uint64_t a0 = m0, a1 = m1;      // the slots' lanes still scanning
            for (uint32_t base = 0; base < A.n_faces; base += kTile) {
                const uint32_t n = A.n_faces - base < kTile ? A.n_faces - base : kTile;
                const float4 *src = reinterpret_cast<const float4 *>(tri + base);
                float4 *dst = reinterpret_cast<float4 *>(tile);
                for (uint32_t e = threadIdx.x; e < 3 * n; e += BLK) dst[e] = src[e];
                __syncthreads();
                if (ttail) {
                    if (worker) {
                        for (uint32_t i = part; i < n; i += R) {
                            float t;
                            if (tri_accept(tile[i], o, d, A.t_min, bt, t)) { bt = t; best = (int)(base + i); }
                        }
                    }
                } else if ((a0 | a1) != 0ull) {
                    // Two-stage exact test: stage 2 (1/den, t, b1, b2, the
                    // compares) only when some lane may accept.  (A software-pipelined read of
                    // the next triangle costs 12 VGPRs and was slower at 4 waves/SIMD.)
                    // Two triangles per step: the first pretest halves of both (slots A and B)
                    // are four independent chains issued together; their results stay live
                    // and the gates then run per triangle, in index order.
                    // (SINGLE scans one slot, two triangles per step too)
                    constexpr uint32_t kStep = 2u;
                    uint32_t i = 0;
                    for (; i + kStep <= n; i += kStep) {
                        TriRecord Tp[kStep];
                        TriPartA Pa[kStep], Pb[kStep];
                        uint64_t ga[kStep], gb[kStep];
#pragma unroll
                        for (uint32_t h = 0; h < kStep; ++h) { Tp[h] = tile[i + h]; gb[h] = 0ull; }
#pragma unroll
                        for (uint32_t h = 0; h < kStep; ++h) {
                            Pa[h] = tri_stage1a(Tp[h], so0, sd0);
                            ga[h] = __builtin_amdgcn_ballot_w64(tri_maybe_a(Pa[h])) & a0;
                            if (!SINGLE) {
                                Pb[h] = tri_stage1a(Tp[h], so1, sd1);
                                gb[h] = __builtin_amdgcn_ballot_w64(tri_maybe_a(Pb[h])) & a1;
                            }
                        }
#pragma unroll
                        for (uint32_t h = 0; h < kStep; ++h) {
                            const TriRecord &T = Tp[h];
                            if (ga[h] != 0ull) {
                                const TriPart PA = tri_stage1b(T, Pa[h], sd0);
                                if ((__builtin_amdgcn_ballot_w64(__builtin_fabsf(PA.n2) <= Pa[h].m) & ga[h]) != 0ull) {
                                    float tA;
                                    if (tri_stage2(T, PA, A.t_min, btA, tA)) { btA = tA; bestA = (int)(base + i + h); }
                                }
                            }
                            if (!SINGLE && gb[h] != 0ull) {
                                const TriPart PB = tri_stage1b(T, Pb[h], sd1);
                                if ((__builtin_amdgcn_ballot_w64(__builtin_fabsf(PB.n2) <= Pb[h].m) & gb[h]) != 0ull) {
                                    float tB;
                                    if (tri_stage2(T, PB, A.t_min, btB, tB)) { btB = tB; bestB = (int)(base + i + h); }
                                }
                            }
                        }
                    }
                    for (; i < n; ++i) {          // the last triangles of a tile
                        const TriRecord T = tile[i];
                        // the gates are lane masks ANDed in scalar registers (ballot of one
                        // compare each): __any(sA && p) materialised the predicate in a VGPR
                        // and compared it again, 2 VALU per gate (C5 schedule 4: -7 %)
                        const TriPartA PaA = tri_stage1a(T, so0, sd0);
                        const uint64_t gA = __builtin_amdgcn_ballot_w64(tri_maybe_a(PaA)) & a0;
                        if (gA != 0ull) {
                            const TriPart PA = tri_stage1b(T, PaA, sd0);
                            if ((__builtin_amdgcn_ballot_w64(__builtin_fabsf(PA.n2) <= PaA.m) & gA) != 0ull) {
                                float tA;
                                if (tri_stage2(T, PA, A.t_min, btA, tA)) { btA = tA; bestA = (int)(base + i); }
                            }
                        }
                        if (!SINGLE) {
                            const TriPartA PaB = tri_stage1a(T, so1, sd1);
                            const uint64_t gB = __builtin_amdgcn_ballot_w64(tri_maybe_a(PaB)) & a1;
                            if (gB != 0ull) {
                                const TriPart PB = tri_stage1b(T, PaB, sd1);
                                if ((__builtin_amdgcn_ballot_w64(__builtin_fabsf(PB.n2) <= PaB.m) & gB) != 0ull) {
                                    float tB;
                                    if (tri_stage2(T, PB, A.t_min, btB, tB)) { btB = tB; bestB = (int)(base + i); }
                                }
                            }
                        }
                    }
                    a0 &= ~__builtin_amdgcn_ballot_w64(btA <= stop0);
                    if (!SINGLE) a1 &= ~__builtin_amdgcn_ballot_w64(btB <= stop1);
                }
                __syncthreads();
            }
            if (ttail) {
                for (uint32_t off = R >> 1; off >= 1; off >>= 1) {
                    const float ot = __shfl_xor(bt, (int)off);
                    const int ob = __shfl_xor(best, (int)off);
                    if (ot < bt || (ot == bt && ob > best)) { bt = ot; best = ob; }
                }
            }
            if (POOL_W) {
                float *const poolf = reinterpret_cast<float *>(pool);
                if (ttail) {
                    if (worker && part == 0u) {
                        poolf[8 * pj0 + 3] = bt;
                        poolf[8 * pj0 + 7] = __int_as_float(best);
                    }
                } else {
                    if ((m0 >> lane) & 1ull) {
                        poolf[8 * pj0 + 3] = btA;
                        poolf[8 * pj0 + 7] = __int_as_float(bestA);
                    }
                    if ((m1 >> lane) & 1ull) {
                        poolf[8 * pj1 + 3] = btB;
                        poolf[8 * pj1 + 7] = __int_as_float(bestB);
                    }
                }
                __syncthreads();
                // this lane's own results (its rays stay in registers: the tiled kernel's
                // budget is not the limit here)
                const uint32_t cap = (uint32_t)(POOL_W * 2 * kWave) - 1u;
                const uint32_t ia = jA < cap ? jA : cap, ib = jB < cap ? jB : cap;
                const float ta = poolf[8 * ia + 3], tb = poolf[8 * ib + 3];
                const int ba = __float_as_int(poolf[8 * ia + 7]), bb = __float_as_int(poolf[8 * ib + 7]);
                btA = ta; bestA = ba;
                btB = tb; bestB = bb;
            } else if (tail) {
                const int srcA = sA ? (int)(rank_in(mA) * R) : (int)lane;
                const int srcB = sB ? (int)((na + rank_in(mB)) * R) : (int)lane;
                const float tA_ = __shfl(bt, srcA), tB_ = __shfl(bt, srcB);
                const int iA_ = __shfl(best, srcA), iB_ = __shfl(best, srcB);
                if (sA) { btA = tA_; bestA = iA_; }
                if (sB) { btB = tB_; bestB = iB_; }
            }
        } else if (BVH) {
            // ---- opt-in BVH: each lane traverses for its own rays, or the wave's rays are
            // pooled over its lanes (bvh_pool) ----
            lds_i32 *stk = (lds_i32 *)bvh_stack;
            if (!SINGLE) {
                // the hybrid's prefix faces first (bvh_prefix_scan), for the rays new this call
                float pbtA = A.t_max, pbtB = A.t_max;
                int pbestA = -1, pbestB = -1;
                if (A.bvh_prefix)
                    bvh_prefix_scan<true>(A, tri, newA, newB, s_ao, s_ad, b_o, b_d, pbtA, pbestA,
                                          pbtB, pbestB);
                float4 *pl = pool + wv * 72;            // res: 64 float4 (128 float2), tab: 8 float4
                bvh_pool(bvh_nodes, bvh_tris, A.bvh_root, stk, reinterpret_cast<uint8_t *>(pl + 64),
                         reinterpret_cast<float2 *>(pl), lane, newA, newB, s_ao, s_ad, b_o, b_d,
                         A.t_min, A.t_max, !q.exhausted, carry, subA, subB, frozen, btA, bestA,
                         btB, bestB, A.bvh_n4, A.bvh_slots, pbtA, pbestA, pbtB, pbestB,
#ifdef RVCP_NO_SHADOW_STOP     // A/B: every shadow ray traversed to its nearest hit
                         -__builtin_inff());
#else
                         newA ? shadow_stop(A.eps, A.t_min, a_p, nee_dist) : -__builtin_inff());
#endif
            } else
            {
            if (A.bvh_prefix)
                bvh_prefix_scan<false>(A, tri, sA, sB, s_ao, s_ad, b_o, b_d, btA, bestA, btB, bestB);
            if (sA) bvh_nearest<true>(bvh_nodes, bvh_tris, A.bvh_root, stk, s_ao, s_ad, A.t_min, btA, bestA, A.bvh_n4, A.bvh_slots);
            if (sB) bvh_nearest<true>(bvh_nodes, bvh_tris, A.bvh_root, stk, b_o, b_d, A.t_min, btB, bestB, A.bvh_n4, A.bvh_slots);
            }
        } else if (tail) {
            // ---- tail: R lanes per ray, each scanning every R-th triangle ----
            // The frame queue is empty, so what is left are the serial sample chains of the
            // last pixels.  The sequential scan keeps (min t, largest index among equal t)
            // (:288-295), so partial scans over disjoint face subsets combined with that same
            // order give the identical nearest hit.
            uint32_t R = 2;
            while (nr * R * 2 <= (uint32_t)kWave) R *= 2;
            uint8_t *tab = tail_tab[wv];
            if (hasA) tab[rank_in(mA)] = (uint8_t)lane;
            if (hasB) tab[na + rank_in(mB)] = (uint8_t)lane;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t j = lane / R, part = lane % R;
            const bool worker = j < nr;
            const int owner = worker ? (int)tab[j] : (int)lane;
            const bool isA = j < na;
            f3 o, d;
            {
                const f3 oa = mk(__shfl(a_o.x, owner), __shfl(a_o.y, owner), __shfl(a_o.z, owner));
                const f3 da = mk(__shfl(a_d.x, owner), __shfl(a_d.y, owner), __shfl(a_d.z, owner));
                const f3 ob = mk(__shfl(b_o.x, owner), __shfl(b_o.y, owner), __shfl(b_o.z, owner));
                const f3 db = mk(__shfl(b_d.x, owner), __shfl(b_d.y, owner), __shfl(b_d.z, owner));
                o = isA ? oa : ob;
                d = isA ? da : db;
            }
            float bt = A.t_max;
            int best = -1;
            if (worker) {
                if (A.rcp_fast && !__any(worker && !dir_fast_ok(d))) {
                    for (uint32_t i = part; i < A.n_faces; i += R) {
                        float t;
                        if (tri_accept<true>(tri[i], o, d, A.t_min, bt, t)) { bt = t; best = (int)i; }
                    }
                } else {
                    for (uint32_t i = part; i < A.n_faces; i += R) {
                        float t;
                        if (tri_accept(tri[i], o, d, A.t_min, bt, t)) { bt = t; best = (int)i; }
                    }
                }
            }
            for (uint32_t off = R >> 1; off >= 1; off >>= 1) {
                const float ot = __shfl_xor(bt, (int)off);
                const int ob = __shfl_xor(best, (int)off);
                if (ot < bt || (ot == bt && ob > best)) { bt = ot; best = ob; }
            }
            const int srcA = hasA ? (int)(rank_in(mA) * R) : (int)lane;
            const int srcB = hasB ? (int)((na + rank_in(mB)) * R) : (int)lane;
            const float tA_ = __shfl(bt, srcA), tB_ = __shfl(bt, srcB);
            const int iA_ = __shfl(best, srcA), iB_ = __shfl(best, srcB);
            if (hasA) { btA = tA_; bestA = iA_; }
            if (hasB) { btB = tB_; bestB = iB_; }
        } else if (!TILED && wave_active && nr <= (uint32_t)kWave) {
            // ---- compact: at most 64 rays, one per lane, one slot instead of two ----
            // Ray j (A rays of the lanes in lane order, then B rays) goes to lane j through
            // this wave's LDS rows, lane j tests it against every triangle, and the nearest hits
            // go back the same way.  Each ray meets the same triangles in the same order, so
            // every nearest hit is unchanged.
            float4 *rows = compact_lds + wv * (2 * kWave);
            if (hasA) {
                const uint32_t j = rank_in(mA);
                rows[2 * j] = make_float4(a_o.x, a_o.y, a_o.z, 0.0f);
                rows[2 * j + 1] = make_float4(a_d.x, a_d.y, a_d.z, 0.0f);
            }
            if (hasB) {
                const uint32_t j = na + rank_in(mB);
                rows[2 * j] = make_float4(b_o.x, b_o.y, b_o.z, 0.0f);
                rows[2 * j + 1] = make_float4(b_d.x, b_d.y, b_d.z, 0.0f);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the lane index re-derived here (opaque to the compiler) so that its row address
            // is not held live across the whole loop -- at 6 waves/SIMD it was spilled
            uint32_t lane_r;
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0"
                         : "=v"(lane_r));
            const float4 ro = rows[2 * lane_r], rd = rows[2 * lane_r + 1];
            const f3 o = mk(ro.x, ro.y, ro.z), d = mk(rd.x, rd.y, rd.z);
            float bt = A.t_max;
            int best = -1;
#ifdef RVCP_SPEC_SCAN
            if (!__any(lane_r < nr && !ray_in_range(o, d))) {
                spec_scan1(o, d, A.t_min, bt, best);
            } else
#endif
            if (A.rcp_fast && !__any(lane_r < nr && !dir_fast_ok(d)))
                scan_generic1<true>(tri, A.n_faces, o, d, A.t_min, bt, best);
            else
                scan_generic1<false>(tri, A.n_faces, o, d, A.t_min, bt, best);
            // lanes >= nr traced stale rows; their results are never read
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            rows[2 * lane_r] = make_float4(bt, __int_as_float(best), 0.0f, 0.0f);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (hasA) {
                const float4 r = rows[2 * rank_in(mA)];
                btA = r.x;
                bestA = __float_as_int(r.y);
            }
            if (hasB) {
                const float4 r = rows[2 * (na + rank_in(mB))];
                btB = r.x;
                bestB = __float_as_int(r.y);
            }
        } else {
            // ---- scan: both rays against every triangle (wave-uniform face index) ----
#ifdef RVCP_SPEC_SCAN
            if (!__any((hasA && !ray_in_range(a_o, a_d)) || (hasB && !ray_in_range(b_o, b_d)))) {
                // the shadow ray's nearest face is not needed, only whether it hit (resolve
                // A): a nearest t other than t_max is a hit; t_max itself (a miss, or a hit at
                // exactly t_max -- neither occurs in a closed room) is settled by the generic
                // scan of the wave's shadow rays, which finds the same nearest hit
                // a lane without a shadow ray takes no part in the shadow slot's skippable
                // blocks: its mask is false whatever its stale ray (btA below t_min)
                if (!hasA) btA = -1.0f;
                spec_scan2(a_o, a_d, b_o, b_d, A.t_min, btA, btB, bestB);
            } else
#endif
            {
            // the generic loop keeps no face index for the shadow ray either (as spec_scan2),
            // and a lane without a shadow ray takes no part in its skips (btA below t_min)
            if (!SINGLE && !hasA) btA = -1.0f;
            if (A.rcp_fast && !__any((hasA && !dir_fast_ok(a_d)) || (hasB && !dir_fast_ok(b_d))))
                scan_generic2<true, SINGLE>(tri, A.n_faces, a_o, a_d, b_o, b_d, A.t_min, btA, bestA, btB, bestB);
            else
                scan_generic2<false, SINGLE>(tri, A.n_faces, a_o, a_d, b_o, b_d, A.t_min, btA, bestA, btB, bestB);
            }
            if (!SINGLE) {
                // The shadow ray's nearest face is not needed, only whether it hit (resolve A):
                // a nearest t other than t_max is a hit; t_max itself (a miss, or a hit at
                // exactly t_max -- neither occurs in a closed room) is settled by a re-scan of
                // the wave's shadow rays that keeps the face, which finds the same nearest hit.
                bestA = btA != A.t_max ? 0 : -1;
                if (__builtin_expect(__any(hasA && btA == A.t_max), 0)) {
                    btA = A.t_max;
                    bestA = -1;
                    for (uint32_t i = 0; i < A.n_faces; ++i) {
                        float tA;
                        if (tri_accept(tri[i], a_o, a_d, A.t_min, btA, tA)) { btA = tA; bestA = (int)i; }
                    }
                }
            }
        }

        if (SINGLE && !hasA) {          // the lane traced its path ray
            btB = btA;
            bestB = bestA;
        }
        RC_END(1);
        RC_BEGIN(3);

        // ---- resolve A: visibility of the light sample (:447-459) ----
        if (LDS_STATE) col = st_get3(13);
        if (hasA && !frozen) {
            if (LDS_STATE) {
                a_p = st_get3(0);
                nee_C = st_get3(3);
                nee_dist = st[6 * BLK];
            }
            const f3 hp = bestA >= 0 ? add(a_o, muls(a_d, btA))
                                     : mk(__builtin_inff(), __builtin_inff(), __builtin_inff());
            const float dist_blocked = len(sub(hp, a_p));
            if (__builtin_fabsf(nee_dist - dist_blocked) < A.eps) {
                col = add(col, nee_C);
                if (LDS_STATE) st_put3(13, col);
            }
        }
        // ---- resolve B: next bounce (:421-429) ----
        const bool defer_B = SINGLE && hasA && hasB;    // B was not traced this iteration
        if (frozen) {
            // waiting on a carried ray: nothing resolves, the rays stay pending
        } else if (hasB && !defer_B) {
            if (bestB < 0) {
                col = add(col, mk(0.1f, 0.1f, 0.1f));
                if (LDS_STATE) st_put3(13, col);
                ended = true;
            } else {
                f3 hpos, hn;
                FaceShade fs;
                hit_shade(tri, shade, bestB, b_o, b_d, btB, hpos, hn, fs);
                if (fs.ty == kLight) {
                    ended = true;       // depth >= 1: no emission term (:426)
                } else {
                    S_pos = hpos; S_nrm = hn; S_alb = ld3(fs.alb_pi);
                    surf_ev = true;
                }
            }
        } else if (hasA && !hasB) {
            ended = true;       // the path ended at its last surface event (RR / depth / att)
        }
        if (!frozen) {
            hasA = false;
            if (!defer_B) hasB = false;
        }
        RC_END(3);
#ifdef RVCP_REGION_CLOCK
        c_iter += __builtin_amdgcn_s_memtime() - c_top;
#endif
    }
    flush_wave_counters(counters, lane, trav_wave, iters);
    clock_stamp(counters, lane, wv == 0, true);
#ifdef RVCP_TIMELINE
    if (A.timeline && lane == 0) {
        const uint32_t w = (blockIdx.x * BLK + threadIdx.x) / kWave;
        unsigned long long *rec = A.timeline + 8ull * w;
        rec[6] = c_scan;
        rec[7] = c_iter;
        rec[0] = t_start;
        rec[1] = t_exhausted;
        rec[2] = __builtin_amdgcn_s_memrealtime();
        rec[3] = iters;
        rec[4] = c_start;                              // shader-clock ticks (s_memtime)
        rec[5] = __builtin_amdgcn_s_memtime();
    }
#endif
}

#ifndef RVCP_JIT
template <int MIN_WAVES>
__global__ __launch_bounds__(kBlock, MIN_WAVES) void games101_path_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];   // tail: ray rank -> owner lane
    __shared__ float4 compact_lds[kBlock / kWave * 2 * kWave];  // compact scan: rays, then hits
    __shared__ float state_lds[kStateCols * kBlock];   // LDS_STATE columns
    path_body<false, false, false, true>(
        A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf, shade, tail_tab,
        nullptr, nullptr, nullptr, nullptr, compact_lds, state_lds);
}

// Opt-in BVH (RVCP_ACCEL_BVH): the variant-3 machine with per-lane BVH traversal in place of
// the brute-force scan.
// (Measured and not kept: private scratch stacks, the path state in LDS columns, 5 waves per SIMD
// (96 VGPRs with two-triangle leaf chunks): all slower)
__global__ __launch_bounds__(kBlock, 4) void games101_bvh_path_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade, const Bvh4Node *__restrict__ bvh_nodes,
    const TriRecord *__restrict__ bvh_tris)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ int32_t bvh_stack[kBvhStack * kBlock];     // traversal stacks, column per thread
    __shared__ float4 bvh_pool_lds[(kBlock / kWave) * 72];  // per wave: 128 results + 128-B owner table
    path_body<false, true, false>(A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf,
                           shade, tail_tab, nullptr, bvh_nodes, bvh_tris,
                           bvh_stack + threadIdx.x, nullptr, nullptr, bvh_pool_lds);
}

__global__ __launch_bounds__(kBlock, kTiledMinWaves) void games101_tiled_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ TriRecord tile[kTile];
    path_body<true, false>(A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf,
                           shade, tail_tab, tile);
}

// Schedule 10: schedule 4 with the workgroup ray pool (path_body POOL_W): the workgroup's rays
// are scanned against each LDS tile in full 64-ray passes shared out over its 4 waves.
__global__ __launch_bounds__(kTiledPoolWaves * kWave, kTiledMinWaves) void games101_tiled_pool_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kTiledPoolWaves][kWave];
    __shared__ TriRecord tile[kTile];
    __shared__ float4 pool[2 * kTiledPoolWaves * 2 * kWave];
    __shared__ uint32_t pool_count[2 * kTiledPoolWaves];
    path_body<true, false, false, false, kTiledPoolWaves>(
        A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf, shade, tail_tab,
        tile, nullptr, nullptr, nullptr, nullptr, nullptr, pool, pool_count);
}

// Variant 5: the LDS-tiled scan with one ray per lane per iteration (no empty ray slots).
__global__ __launch_bounds__(kBlock, kTiledMinWaves) void games101_tiled_single_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ TriRecord tile[kTile];
    path_body<true, false, true>(A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf,
                           shade, tail_tab, tile);
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

// The frame's tone map + UNORM8 store after the v3-family kernels (store_acc above): the
// threshold table in LDS, one pixel per lane.
constexpr uint32_t kToneBlock = 256;
__global__ __launch_bounds__(kToneBlock) void tonemap_kernel(const float *__restrict__ lin, uint32_t n,
                                                             const float *__restrict__ gamma_t,
                                                             uint32_t *__restrict__ out_rgba)
{
    __shared__ float T[257];
    T[threadIdx.x] = gamma_t[threadIdx.x];
    if (threadIdx.x == 0) T[256] = gamma_t[256];
    __syncthreads();
    for (uint32_t i = blockIdx.x * kToneBlock + threadIdx.x; i < n; i += gridDim.x * kToneBlock)
        out_rgba[i] = pack_rgba(mk(lin[3 * (size_t)i], lin[3 * (size_t)i + 1], lin[3 * (size_t)i + 2]), T);
}

__global__ void fill_kernel(uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
                            uint32_t n, uint32_t rgba)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        out_rgba[i] = rgba;
        if (out_lin) { out_lin[3 * i] = 0.0f; out_lin[3 * i + 1] = 0.0f; out_lin[3 * i + 2] = 0.0f; }
    }
}

#endif  // RVCP_JIT
#if !defined(RVCP_JIT) || defined(RVCP_JIT_LEGACY)
// ======================================================================================
// Integrator RVCP_INTEGRATOR_LEGACY: ray_trace of assets/shaders/ray_tracer.comp
// (:618-694, main :802-822) -- spheres then triangles, Lambertian / metal / dielectric
// scattering, no light sampling, UNORM store without gamma.  Same machine as variant 1: one
// ray per lane per iteration, the RNG-independent primary hit traced once per pixel and reused
// by every sample, the per-lane rejection loops of random_in_unit_sphere run cooperatively.
// ======================================================================================
namespace {

// GLSL reflect(I, N) = I - 2 dot(N, I) N
__device__ __forceinline__ f3 reflect_glsl(f3 I, f3 N) { return sub(I, muls(N, 2.0f * dot(N, I))); }

// GLSL refract(I, N, eta)
__device__ __forceinline__ f3 refract_glsl(f3 I, f3 N, float eta) {
    const float d = dot(N, I);
    const float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk(0, 0, 0);
    return sub(muls(I, eta), muls(N, eta * d + sqrt_c(k)));
}

// fresnel_schlick, :544-551; pow(x, 5.0) := ((x*x)*(x*x))*x
__device__ __forceinline__ float fresnel_schlick(float cosine, float ratio) {
    float r0 = (1.0f - ratio) / (1.0f + ratio);
    r0 = r0 * r0;
    const float x = 1.0f - cosine;
    return r0 + (1.0f - r0) * (x * x * (x * x) * x);
}

// is_intersect_with_sphere + is_intersect_with_quadratic_equation (:260-321) under the
// nearest-hit rule of get_intersection_with_scene (:376-381): true iff the shader would take
// this sphere as the new nearest hit, whose time is written to t_out.  a = dot(d, d) and
// two_a = 2 a are per-ray constants (the shader recomputes the same values per sphere).
// FAST: the two roots (-b +- sq) / two_a as Markstein quotients from y = RN(1 / two_a)
// (rcp_ieee, once per ray): q = x y, r = fma(-two_a, q, x) (exact), t = fma(r, y, q) =
// RN(x / two_a) whenever 2^-60 <= |x| <= 2^60 with two_a in [2^-30, 2^30].  Outside that
// range both the IEEE root and this one lie below 2^-30 or above 2^30 in magnitude (or are
// NaN), so with t_min >= 2^-29 and t_max < 2^29 both are rejected, and the root order of the
// swap differs at most between two rejected roots: the decision and the accepted t are the
// IEEE ones.  The caller checks the ranges per wave.
__device__ __forceinline__ float quot_markstein(float x, float s, float y) {
    const float q = x * y;
    return __builtin_fmaf(__builtin_fmaf(-s, q, x), y, q);
}
template <bool FAST>
__device__ __forceinline__ bool sphere_accept(f3 ce, float radius, f3 o, f3 d, float a,
                                              float two_a, float y, float tmin, float bt,
                                              float &t_out) {
    const f3 co = mk(o.x - ce.x, o.y - ce.y, o.z - ce.z);
    const float b = 2.0f * dot(d, co);
    const float c = dot(co, co) - radius * radius;
    const float delta = b * b - 4.0f * a * c;
    // no lane's line meets the sphere (delta < 0 or NaN everywhere): every lane rejects it
    // below (!(delta < 0) fails, or NaN roots fail the compares), so the wave skips the
    // square root, the roots and the compares
    if (!__any(delta >= 0.0f)) { t_out = bt; return false; }
    // the root matters only where delta >= 0: a lane with delta < 0 (or NaN) rejects the sphere
    // whatever sq is (NaN from either form), so only delta >= 0 outside sqrt_fast_ok's range
    // takes the IEEE sequence -- not every wave in which some lane misses the sphere
    float sq = sqrt_fast_core(delta);
    if (__builtin_expect((delta >= 0.0f) & !sqrt_fast_ok(delta), 0)) sq = __builtin_sqrtf(delta);
#ifndef RVCP_SPHERE_SWAP_FORM     // (A/B only: the swap form below for the FAST roots too)
    if (FAST) {
        // The swap below always leaves the "- sq" root first: with two_a > 0 (FAST: two_a in
        // [2^-30, 2^30]) and sq >= 0, RN(-b - sq) <= RN(-b + sq), and the Markstein quotient is
        // the IEEE one, monotonic in the numerator, wherever the numerator lies in
        // [2^-60, 2^60]; a root outside that range is below 2^-30 or above 2^30 in magnitude
        // (or NaN: the quotient overflows past 2^98) in both forms and fails tmin <= t <= bt
        // either way.  So the shader's choice (the smaller root if it is in [tmin, bt], else the
        // larger one if that is) is: the smaller root if it is >= tmin, else the larger one,
        // accepted iff it lies in [tmin, bt] (a smaller root above bt leaves a larger one above
        // bt too; a NaN root fails its compares, as the IEEE root it stands for, beyond 2^30,
        // fails them).  4 compares / selects instead of 8.
        const float ts = quot_markstein(-b - sq, two_a, y);
        const float tl = quot_markstein(-b + sq, two_a, y);
        const float tc = (tmin <= ts) ? ts : tl;
        t_out = tc;
        return !(delta < 0.0f) & (tmin <= tc) & (tc <= bt);
    }
#endif
    float t0 = FAST ? quot_markstein(-b + sq, two_a, y) : (-b + sq) / two_a;
    float t1 = FAST ? quot_markstein(-b - sq, two_a, y) : (-b - sq) / two_a;
    if (t0 > t1) { const float tmp = t0; t0 = t1; t1 = tmp; }
    const bool h0 = (tmin <= t0) & (t0 <= bt);
    const bool h1 = (tmin <= t1) & (t1 <= bt);
    t_out = h0 ? t0 : t1;
    return !(delta < 0.0f) & (h0 | h1);
}

constexpr int L_IDLE = 0, L_TRACE = 1, L_SCATTER = 2, L_END = 3;

// The sphere half of get_intersection_with_scene (:369-381) for the tracing lanes (`active`);
// FAST as sphere_accept, chosen per wave by the caller.
template <bool FAST>
__device__ __forceinline__ void legacy_spheres(const FrameArgs &A, const rvcp_sphere_t *__restrict__ sph,
                                               f3 ro, f3 rd, float a, float two_a, float rtmin,
                                               float &bt, int &best) {
    const float y = FAST ? rcp_ieee(two_a) : 0.0f;
#ifdef RVCP_SPEC_SPHERES
    // the scene-specialised module (rvcp_jit.cpp jit_sphere_source): the uploaded spheres as
    // literals, X(index, center x, y, z, radius) in index order -- the loop unrolled, no record
    // loads, the radius' square folded; the same operations on the same values
    (void)A;
    (void)sph;
#define RVCP_SPHERE_TEST(i, cx, cy, cz, r)                                                        \
    {                                                                                             \
        float t;                                                                                  \
        if (sphere_accept<FAST>(mk(cx, cy, cz), r, ro, rd, a, two_a, y, rtmin, bt, t)) {          \
            bt = t;                                                                               \
            best = (i);                                                                           \
        }                                                                                         \
    }
    RVCP_SPEC_SPHERES(RVCP_SPHERE_TEST)
#undef RVCP_SPHERE_TEST
#else
    for (uint32_t i = 0; i < A.n_spheres; ++i) {
        float t;
        if (sphere_accept<FAST>(ld3(sph[i].center), sph[i].radius, ro, rd, a, two_a, y, rtmin, bt, t)) {
            bt = t;
            best = (int)i;
        }
    }
#endif
}

// The hit record of the nearest hit `best` (spheres first, then faces) of ray (ro, rd) at time
// bt: position, the normal against the ray and whether the ray hit the front face
// (:314-319 spheres, :348-363 faces), and the material.
__device__ __forceinline__ void legacy_hit(const FrameArgs &A, const TriRecord *__restrict__ tri,
                                           const FaceShade *__restrict__ shade,
                                           const rvcp_sphere_t *__restrict__ sph, int best, f3 ro,
                                           f3 rd, float bt, f3 &hpos, f3 &hn, uint32_t &hm,
                                           bool &ho) {
    ho = true;
    hpos = add(ro, muls(rd, bt));
    // The vector each kind of hit normalises -- hpos - centre (:314), or the interpolated vertex
    // normal (:352-356) -- is chosen per lane and normalised once after the branch: a wave
    // whose lanes hit both kinds runs one normalize instead of two (the same operations on
    // the same value per lane).
    const bool is_sphere = (uint32_t)best < A.n_spheres;
    f3 nv;
    bool inside = false;
    if (is_sphere) {                                            // :314-319
        const rvcp_sphere_t S = sph[best];
        const f3 ce = ld3(S.center);
        nv = sub(hpos, ce);
        const f3 oc = sub(ro, ce);
        inside = dot(oc, oc) < S.radius * S.radius;
        hm = S.material_id;
#ifdef RVCP_HIT_SPLIT_NORMALIZE     // (A/B only: a normalize in each branch, as before round 6)
        hn = normalize(nv);
#endif
    } else {                                                    // :348-363
        const int fi = best - (int)A.n_spheres;
        const TriRecord T = tri[fi];
        const FaceShade fs = shade[fi];
        const f3 s = mk(ro.x - T.v0[0], ro.y - T.v0[1], ro.z - T.v0[2]);
        const f3 s1 = cross(rd, ld3(T.e2));
        const f3 s2 = cross(s, ld3(T.e1));
        const float f = rcp_ieee(dot(s1, ld3(T.e1)));
        const float b1 = f * dot(s1, s);
        const float b2 = f * dot(s2, rd);
        nv = add(add(muls(ld3(fs.n0), 1.0f - b1 - b2), muls(ld3(fs.n1), b1)), muls(ld3(fs.n2), b2));
        hm = fs.mat;
#ifdef RVCP_HIT_SPLIT_NORMALIZE
        hn = normalize(nv);
#endif
    }
#ifndef RVCP_HIT_SPLIT_NORMALIZE
    hn = normalize(nv);
#endif
    if (is_sphere ? inside : dot(hn, rd) > 0.0f) { hn = neg(hn); ho = false; }
}

// kLegacyDefer: the most lanes left ending a sample that sit out one trace (below).  16
// measured best: sphere room 0.367 -> 0.345 ms, mode 2 on the C3 frame 2.237 -> 2.156 ms per
// frame (profiles/history/r03v_m2_defer_sweep.log; 8, 24, 32, 40 and 64 less good).
#ifndef RVCP_LEGACY_DEFER
#define RVCP_LEGACY_DEFER 16
#endif
constexpr int kLegacyDefer = RVCP_LEGACY_DEFER;

}  // namespace

__device__ __forceinline__ void legacy_body(
    const FrameArgs &A, const TriRecord *__restrict__ tri, const FaceShade *__restrict__ shade,
    const rvcp_sphere_t *__restrict__ sph, const rvcp_material_t *__restrict__ mats,
    const float *__restrict__ unorm_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters,
    uint8_t (*coop_tab)[kWave], StartSlot (*start_slots)[kWave], float *prim_lds = nullptr)
{
    uint8_t *tab = coop_tab[threadIdx.x / kWave];
    const uint32_t lane = lane_id();
    const bool first_wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave) == 0;
    clock_stamp(counters, lane, first_wave, false);
    Queue q = queue_init(A);
#if RVCP_LEGACY_PREFILL
    StartSlot *slots = start_slots[threadIdx.x / kWave];
    uint32_t q_base = q.next;                       // the static chunk, prefilled here
    prefill_starts(A, q_base, q.end - q.next, lane, slots);
#endif
    const float sppf = (float)A.spp;
    const float inv_spp = rcp_ieee(sppf);     // divs_y's shared reciprocal
    const float inv_rr = rcp_ieee(A.rr);
    // RR = 1.0 (ray_tracer.comp's own setting): rand() < 1 (v_fract_f32 never returns 1), so
    // the roulette never ends a path and only advances the rand() index, and att / 1.0 = att
    // exactly -- neither the sine nor the division is computed (wave-uniform)
    const bool rr_one = A.rr == 1.0f;

    // debug timeline (FrameArgs::timeline) and RVCP_REGION_CLOCK=k as in path_body; regions:
    // 1 the trace (spheres + faces), 2 the settle loop, 3 the hit record, 4 the scatter block,
    // 5 taking new pixels (queue + srand + sample_ray)
#ifdef RVCP_TIMELINE
    const unsigned long long t_start = A.timeline ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const unsigned long long c_start = A.timeline ? __builtin_amdgcn_s_memtime() : 0ull;
#endif
    unsigned long long c_scan = 0ull, c_iter = 0ull;
    int st = L_IDLE;
    bool need_pixel = true, done = false, primary = false;
    uint32_t pix = 0, k = 0, left = 0, trav = 0, iters = 0;
    float seed = 0.0f, ridx = 0.0f;
    f3 acc = mk(0, 0, 0), att = mk(1, 1, 1), col = mk(0, 0, 0);
#ifdef RVCP_LEGACY_LDS_PRIMARY
    // the cached primary hit in this lane's LDS column (prim_lds[f * kBlock], f = 0..10:
    // position, normal, direction, material | front-face bit 31) instead of 11 VGPRs held for
    // the whole pixel: it is written once per pixel and read once per sample
    float *const pcol = prim_lds + threadIdx.x;
    auto prim_put = [&](f3 p, f3 n, f3 d, uint32_t m, bool out) {
        pcol[0 * kBlock] = p.x; pcol[1 * kBlock] = p.y; pcol[2 * kBlock] = p.z;
        pcol[3 * kBlock] = n.x; pcol[4 * kBlock] = n.y; pcol[5 * kBlock] = n.z;
        pcol[6 * kBlock] = d.x; pcol[7 * kBlock] = d.y; pcol[8 * kBlock] = d.z;
        pcol[9 * kBlock] = __uint_as_float(m | (out ? 0x80000000u : 0u));
    };
#else
    (void)prim_lds;
    f3 P_pos = mk(0, 0, 0), P_nrm = mk(0, 0, 0), P_dir = mk(0, 0, 1);   // cached primary hit
    uint32_t P_mat = 0;
    bool P_out = true;
#endif
    f3 H_pos = mk(0, 0, 0), H_nrm = mk(0, 0, 0), H_dir = mk(0, 0, 1);   // hit being scattered
    uint32_t H_mat = 0;
    bool H_out = true;
    f3 ro = mk(0, 0, 0), rd = mk(0, 0, 1);
    float rtmin = 0.0f, rtmax = 0.0f;

    for (;;) {
#ifdef RVCP_REGION_CLOCK
        const unsigned long long c_top = __builtin_amdgcn_s_memtime();
#endif
        RC_BEGIN(2);
        // ============ settle: advance every lane until it has a ray or is done ============
        for (;;) {
            if (st == L_END) {                                      // color += ray_trace (:817)
                acc = add(acc, col);
                k += 1;
                if (k >= A.spp) {                                   // :819-821
                    store_acc(batch_out(A, pix), divs_y(acc, sppf, inv_spp), out_lin);
                    need_pixel = true;
                    st = L_IDLE;
                } else {                                            // next sample, cached hit
                    att = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    left = A.max_bounces - 1u;
#ifdef RVCP_LEGACY_LDS_PRIMARY
                    H_pos = mk(pcol[0 * kBlock], pcol[1 * kBlock], pcol[2 * kBlock]);
                    H_nrm = mk(pcol[3 * kBlock], pcol[4 * kBlock], pcol[5 * kBlock]);
                    H_dir = mk(pcol[6 * kBlock], pcol[7 * kBlock], pcol[8 * kBlock]);
                    const uint32_t mo = __float_as_uint(pcol[9 * kBlock]);
                    H_mat = mo & 0x7FFFFFFFu;
                    H_out = (mo >> 31) != 0u;
#else
                    H_pos = P_pos; H_nrm = P_nrm; H_dir = P_dir; H_mat = P_mat; H_out = P_out;
#endif
                    st = L_SCATTER;
                }
            }
            RC_BEGIN(5);
            {   // take new pixels from the frame queue (wave-uniform control flow)
                bool got;
                uint32_t np = pix;
#if RVCP_LEGACY_PREFILL
                queue_take_started(q, __ballot(need_pixel && !done), lane, A, counters, slots,
                                   q_base, got, np, seed, ridx, ro, rd, rtmin, rtmax);
#else
                queue_take(q, __ballot(need_pixel && !done), lane, A, counters, got, np);
#endif
                if (got) {
                    pix = np;
#if !RVCP_LEGACY_PREFILL
                    start_any(A, pix, seed, ridx, ro, rd, rtmin, rtmax);
#endif
                    primary = true;
                    need_pixel = false;
                    k = 0;
                    acc = mk(0, 0, 0);
                    att = mk(1, 1, 1);
                    col = mk(0, 0, 0);
                    st = L_TRACE;
                } else if (need_pixel && q.exhausted) {
                    done = true;
                }
            }
            RC_END(5);
            RC_BEGIN(4);
            if (__any(st == L_SCATTER)) {
                // material_scatter (:585-602), then the tail of the bounce loop (:668-686)
                const bool sc = st == L_SCATTER;
                uint32_t ty = 0xFFFFFFFFu;
                f3 alb = mk(0, 0, 0);
                float fuzz = 0.0f, ior = 1.0f;
                if (sc) {
                    const rvcp_material_t &M = mats[H_mat];
                    ty = M.ty;
                    alb = ld3(M.albedo);
                    fuzz = M.fuzz;
                    ior = M.refraction_ratio;
                }
                f3 dir = mk(0, 0, 0);
                f3 refl = mk(0, 0, 0);
                if (A.has_metal) {      // (only metal reads it; a scene-wide uniform test)
                    refl = reflect_glsl(H_dir, H_nrm);                      // metal :526-527
                    if (dot(refl, H_nrm) < 0.0f) refl = neg(refl);
                }
                bool pend = sc && (ty == 0u || ty == 1u);
                while (__any(pend)) {
                    f3 p = mk(0, 0, 0);
                    coop_unit_sphere(pend, seed, ridx, p, lane, tab);
                    if (pend) {
                        const f3 u = normalize(p);          // random_in_unit_sphere_surface :225
                        if (ty == 0u) {                     // lambertian_scatter :491-513
                            dir = normalize(add(H_nrm, u));
                            if (__builtin_fabsf(dir.x) < A.eps && __builtin_fabsf(dir.y) < A.eps &&
                                __builtin_fabsf(dir.z) < A.eps)
                                dir = H_nrm;
                            pend = false;
                        } else {                            // metal_scatter :528-530
                            dir = normalize(add(refl, muls(u, fuzz)));
                            pend = dot(dir, H_nrm) < 0.0f;
                        }
                    }
                }
                if (sc && ty == 2u) {                                       // :553-581
                    const float ratio = H_out ? (1.0f / ior) : ior;
                    const float cos_t = dot(neg(H_dir), H_nrm);
                    const float sin_t = sqrt_c(1.0f - cos_t * cos_t);
                    bool refracted = ratio * sin_t <= 1.0f;
                    if (refracted) refracted = rnd(seed, ridx) >= fresnel_schlick(cos_t, ratio);
                    dir = refracted ? refract_glsl(H_dir, H_nrm, ratio) : reflect_glsl(H_dir, H_nrm);
                }
                if (sc) {
                    const f3 natt = (ty == 0u || ty == 1u) ? alb
                                  : (ty == 2u ? mk(1, 1, 1) : mk(0, 0, 0));    // unknown: 0 (:655)
                    att = mulv(att, natt);                                  // :667
                    rd = dir;
                    ro = add(H_pos, muls(dir, A.t_min));                    // :668-670
                    rtmin = A.t_min;
                    rtmax = A.t_max;
                    if (att.x < A.eps && att.y < A.eps && att.z < A.eps) {  // :673-676
                        st = L_END;
                    } else if (rr_one ? (ridx = ridx + 1.0f, false)          // :679-681
                                      : rnd(seed, ridx) >= A.rr) {
                        st = L_END;
                    } else {
                        if (!rr_one) att = divs_y(att, A.rr, inv_rr);        // :683
                        if (left == 0u) {
                            st = L_END;                                     // :633
                        } else {
                            left -= 1u;                                     // :634
                            st = L_TRACE;
                        }
                    }
                }
            }
            RC_END(4);
            if (!__any(st == L_END)) break;
            // Lanes whose sample ended in this scatter (bounce limit) sit out one trace when
            // few of them did and other lanes have rays: their next sample's scatter then runs
            // inside the next settle with the whole wave's instead of in a nearly empty pass
            // now.  Timing only: each lane's own sequence of operations is unchanged.
            if (__any(st == L_TRACE) && __popcll(__ballot(st == L_END)) <= kLegacyDefer) break;
        }
        RC_END(2);
        if (!__any(st == L_TRACE)) break;
        iters += 1;
        RC_BEGIN(1);

        // ============ trace: get_intersection_with_scene, spheres then faces (:369-393) ============
        int best = -1;
        float bt = rtmax;
        const float a = dot(rd, rd), two_a = 2.0f * a;
        // the sphere roots by Markstein quotients when every tracing lane is in range (above)
        const bool fast = A.t_max < 0x1p29f &&
                          __all(st != L_TRACE || ((two_a >= 0x1p-30f) & (two_a <= 0x1p30f) &
                                                  (rtmin >= 0x1p-29f)));
#ifdef RVCP_SPEC_SCAN
        const bool spec = __all(st != L_TRACE || (ray_in_range(ro, rd) && rtmin > 0.0f));
#endif
        const bool rfast = A.rcp_fast && __all(st != L_TRACE || dir_fast_ok(rd));
        if (st == L_TRACE) {
            trav += 1;
            if (fast) legacy_spheres<true>(A, sph, ro, rd, a, two_a, rtmin, bt, best);
            else legacy_spheres<false>(A, sph, ro, rd, a, two_a, rtmin, bt, best);
#ifdef RVCP_SPEC_SCAN
            if (spec) {
                // the scene-specialised scan (§4.7), exact for finite rays with t_min > 0
                int bf = -1;
                spec_scan1(ro, rd, rtmin, bt, bf);
                if (bf >= 0) best = (int)A.n_spheres + bf;
            } else
#endif
            if (rfast) {
#pragma unroll 2
            for (uint32_t i = 0; i < A.n_faces; ++i) {
                float t;
                if (tri_accept<true>(tri[i], ro, rd, rtmin, bt, t)) { bt = t; best = (int)(A.n_spheres + i); }
            }
            } else {
#pragma unroll 2
            for (uint32_t i = 0; i < A.n_faces; ++i) {
                float t;
                if (tri_accept(tri[i], ro, rd, rtmin, bt, t)) { bt = t; best = (int)(A.n_spheres + i); }
            }
            }
        }

        RC_END(1);
        RC_BEGIN(3);
        // ============ hit record + emission / miss (:636-661) ============
        if (st == L_TRACE) {
            if (best < 0) {
                col = add(col, mulv(att, mk(0, 0, 0)));   // sample_infinite_light = 0 (:600-606)
                st = L_END;
            } else {
                f3 hpos, hn;
                uint32_t hm;
                bool ho;
                legacy_hit(A, tri, shade, sph, best, ro, rd, bt, hpos, hn, hm, ho);
                const rvcp_material_t &M = mats[hm];
                if (M.ty == kLight) {                                       // :656-660
                    col = add(col, mulv(att, ld3(M.albedo)));
                    st = L_END;
                } else {
                    H_pos = hpos; H_nrm = hn; H_dir = rd; H_mat = hm; H_out = ho;
                    st = L_SCATTER;
                }
            }
            if (primary) {
                primary = false;
                if (st == L_END) {
                    // miss / light: every sample returns this same color without touching the
                    // RNG; sum it SPP times in order (:816-818)
                    for (uint32_t i = 0; i < A.spp; ++i) acc = add(acc, col);
                    store_acc(batch_out(A, pix), divs_y(acc, sppf, inv_spp), out_lin);
                    need_pixel = true;
                    st = L_IDLE;
                } else {
#ifdef RVCP_LEGACY_LDS_PRIMARY
                    prim_put(H_pos, H_nrm, H_dir, H_mat, H_out);
#else
                    P_pos = H_pos; P_nrm = H_nrm; P_dir = H_dir; P_mat = H_mat; P_out = H_out;
#endif
                    left = A.max_bounces - 1u;
                }
            }
        }
        RC_END(3);
#ifdef RVCP_REGION_CLOCK
        c_iter += __builtin_amdgcn_s_memtime() - c_top;
#endif
    }
    flush_counters(counters, lane, trav, iters);
    clock_stamp(counters, lane, first_wave, true);
#ifdef RVCP_TIMELINE
    if (A.timeline && lane == 0) {
        const uint32_t w = (blockIdx.x * kBlock + threadIdx.x) / kWave;
        unsigned long long *rec = A.timeline + 8ull * w;
        rec[0] = t_start;
        rec[1] = 0ull;
        rec[2] = __builtin_amdgcn_s_memrealtime();
        rec[3] = iters;
        rec[4] = c_start;
        rec[5] = __builtin_amdgcn_s_memtime();
        rec[6] = c_scan;
        rec[7] = c_iter;
    }
#endif
}

#ifndef RVCP_JIT
#ifndef RVCP_LEGACY_MIN_WAVES
#define RVCP_LEGACY_MIN_WAVES 1
#endif
__global__ __launch_bounds__(kBlock, RVCP_LEGACY_MIN_WAVES) void legacy_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const FaceShade *__restrict__ shade,
    const rvcp_sphere_t *__restrict__ sph, const rvcp_material_t *__restrict__ mats,
    const float *__restrict__ unorm_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters)
{
    __shared__ uint8_t coop_tab[kBlock / kWave][kWave];
    __shared__ StartSlot start_slots[kBlock / kWave][kWave];
    legacy_body(A, tri, shade, sph, mats, unorm_t, out_rgba, out_lin, counters, coop_tab,
                start_slots);
}
#else
// mode 2 with the scene-specialised triangle scan (rvcp_jit.cpp, RVCP_JIT_LEGACY)
#ifndef RVCP_LEGACY_MIN_WAVES
#define RVCP_LEGACY_MIN_WAVES 1
#endif
extern "C" __global__ __launch_bounds__(kBlock, RVCP_LEGACY_MIN_WAVES) void rvcp_spec_legacy_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const FaceShade *__restrict__ shade,
    const rvcp_sphere_t *__restrict__ sph, const rvcp_material_t *__restrict__ mats,
    const float *__restrict__ unorm_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters)
{
    __shared__ uint8_t coop_tab[kBlock / kWave][kWave];
    __shared__ StartSlot start_slots[kBlock / kWave][kWave];
#ifdef RVCP_LEGACY_LDS_SCENE
    // scenes of at most 64 spheres, materials and faces (rvcp_jit.cpp, lds_fits): the per-lane
    // gathers of the hit record, the spheres and the scatter's material read LDS copies
    // instead of global memory (sphere room -3.5 %, mode 2 on the C3 frame -2 %)
    // (sized to the uploaded scene: the module's RVCP_LDS_FACES / _SPHERES / _MATS, rvcp_jit.cpp
    // jit_legacy_source, so that the block's LDS leaves room for more resident blocks)
#ifndef RVCP_LDS_FACES
#define RVCP_LDS_FACES 64
#define RVCP_LDS_SPHERES 64
#define RVCP_LDS_MATS 64
#endif
    __shared__ TriRecord sh_tri[RVCP_LDS_FACES];
    __shared__ FaceShade sh_shade[RVCP_LDS_FACES];
    __shared__ rvcp_sphere_t sh_sph[RVCP_LDS_SPHERES];
    __shared__ rvcp_material_t sh_mat[RVCP_LDS_MATS];
    {
        auto cp = [](float4 *dst, const float4 *src, uint32_t n) {
            for (uint32_t e = threadIdx.x; e < n; e += kBlock) dst[e] = src[e];
        };
        // (the module is built for this scene, so the counts fit; the minima only keep the
        // copies inside the arrays)
        const uint32_t nf = min(A.n_faces, (uint32_t)RVCP_LDS_FACES);
        const uint32_t ns = min(A.n_spheres, (uint32_t)RVCP_LDS_SPHERES);
        const uint32_t nm = min(A.n_mats, (uint32_t)RVCP_LDS_MATS);
        cp(reinterpret_cast<float4 *>(sh_tri), reinterpret_cast<const float4 *>(tri), 3u * nf);
        cp(reinterpret_cast<float4 *>(sh_shade), reinterpret_cast<const float4 *>(shade), 4u * nf);
        cp(reinterpret_cast<float4 *>(sh_sph), reinterpret_cast<const float4 *>(sph), 2u * ns);
        cp(reinterpret_cast<float4 *>(sh_mat), reinterpret_cast<const float4 *>(mats), 2u * nm);
        __syncthreads();
    }
    // (the sphere loop's wave-uniform records read from global memory by scalar loads instead,
    // beside the LDS copies for the per-lane gathers: 0.2855 vs 0.2814 ms, profiles/history/r04i_ab_m2c.log)
#ifdef RVCP_LEGACY_LDS_PRIMARY
    __shared__ float prim_lds[10 * kBlock];
#else
    float *const prim_lds = nullptr;
#endif
    legacy_body(A, sh_tri, sh_shade, sh_sph, sh_mat, unorm_t, out_rgba, out_lin, counters, coop_tab,
                start_slots, prim_lds);
#else
    legacy_body(A, tri, shade, sph, mats, unorm_t, out_rgba, out_lin, counters, coop_tab,
                start_slots);
#endif
}
#endif
#endif  // !RVCP_JIT || RVCP_JIT_LEGACY
#ifdef RVCP_JIT
// Scene-specialised path kernels (rvcp_jit.cpp compiles this file with hipRTC, RVCP_JIT and
// RVCP_SPEC_SCAN set): schedules 3 and 6 with the scan unrolled over the uploaded scene
// (DESIGN.md §4.7).  extern "C" so that the host finds them by name in the module.
#ifdef RVCP_JIT_BVH
// The BVH hybrid (FrameArgs::bvh_prefix): the module's scan covers the scene's
// first bvh_prefix faces; the BVH path kernel and pre-pass test them with it, then the BVH.
extern "C" __global__ __launch_bounds__(kBlock, 4) void rvcp_spec_bvh_path_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade, const Bvh4Node *__restrict__ bvh_nodes,
    const TriRecord *__restrict__ bvh_tris)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ int32_t bvh_stack[kBvhStack * kBlock];     // traversal stacks, column per thread
    __shared__ float4 bvh_pool_lds[(kBlock / kWave) * 72];  // per wave: 128 results + 128-B owner table
    path_body<false, true, false>(A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf,
                           shade, tail_tab, nullptr, bvh_nodes, bvh_tris,
                           bvh_stack + threadIdx.x, nullptr, nullptr, bvh_pool_lds);
}
extern "C" __global__ __launch_bounds__(kPrimaryBlock) void rvcp_spec_bvh_primary_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const float *__restrict__ gamma_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters,
    SurfRecord *__restrict__ surf, const FaceShade *__restrict__ shade,
    const Bvh4Node *__restrict__ bvh_nodes, const TriRecord *__restrict__ bvh_tris,
    const float *__restrict__ cams, uint32_t frame_stride)
{
    primary_body<true, true>(A, tri, faces, verts, mats, gamma_t, out_rgba, out_lin, counters,
                             surf, shade, bvh_nodes, bvh_tris, cams, frame_stride);
}
#endif
// the pre-pass with the specialised scan (rvcp_launch_games101_v3's spec_pre_fn)
extern "C" __global__ __launch_bounds__(kPrimaryBlock) void rvcp_spec_primary_kernel(
    FrameArgs A, const TriRecord *__restrict__ tri, const rvcp_face_t *__restrict__ faces,
    const rvcp_vertex_t *__restrict__ verts, const MatRecord *__restrict__ mats,
    const float *__restrict__ gamma_t, uint32_t *__restrict__ out_rgba,
    float *__restrict__ out_lin, unsigned long long *__restrict__ counters,
    SurfRecord *__restrict__ surf, const FaceShade *__restrict__ shade,
    const Bvh4Node *__restrict__ bvh_nodes, const TriRecord *__restrict__ bvh_tris,
    const float *__restrict__ cams, uint32_t frame_stride)
{
    primary_body<false, true>(A, tri, faces, verts, mats, gamma_t, out_rgba, out_lin, counters,
                              surf, shade, bvh_nodes, bvh_tris, cams, frame_stride);
}
extern "C" __global__ __launch_bounds__(kBlock, kPathMinWaves) void rvcp_spec_path_kernel5(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ float4 compact_lds[kBlock / kWave * 2 * kWave];
    __shared__ float state_lds[kStateCols * kBlock];
    // The scene's triangle and shading records (at most 64 faces in this module) are copied
    // into LDS once per workgroup, so the hit record's per-lane gathers and the tail
    // partition's triangle reads are LDS reads: a small frame's serial chain waits on them
    // every iteration (C2 one frame alone 0.492 -> 0.485 ms, its path kernel 0.470 -> 0.459;
    // C3 unchanged, profiles/history/r04g_ab_c2lds*.log).  31.5 KB per workgroup: 5 per CU still fit.
    __shared__ TriRecord sh_tri[kJitMaxFaces];
    __shared__ FaceShade sh_shade[kJitMaxFaces];
    static_assert(5 * (sizeof(tail_tab) + sizeof(compact_lds) + sizeof(state_lds) + sizeof(sh_tri) +
                       sizeof(sh_shade)) <= 160 * 1024, "5 workgroups per CU");
    {
        const float4 *src = reinterpret_cast<const float4 *>(tri);
        float4 *dst = reinterpret_cast<float4 *>(sh_tri);
        for (uint32_t e = threadIdx.x; e < 3u * A.n_faces; e += kBlock) dst[e] = src[e];
        const float4 *src2 = reinterpret_cast<const float4 *>(shade);
        float4 *dst2 = reinterpret_cast<float4 *>(sh_shade);
        for (uint32_t e = threadIdx.x; e < 4u * A.n_faces; e += kBlock) dst2[e] = src2[e];
        __syncthreads();
    }
#ifdef RVCP_SPEC_REG_STATE
    // A/B: the path state in registers instead of LDS columns (fewer LDS round trips on a
    // small frame's serial chain)
    path_body<false, false, false, false>(
        A, sh_tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf, sh_shade, tail_tab,
        nullptr, nullptr, nullptr, nullptr, compact_lds, state_lds);
#else
    path_body<false, false, false, true>(
        A, sh_tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf, sh_shade, tail_tab,
        nullptr, nullptr, nullptr, nullptr, compact_lds, state_lds);
#endif
}
extern "C" __global__ __launch_bounds__(kBlock, 6) void rvcp_spec_path_kernel6(
    FrameArgs A, const TriRecord *__restrict__ tri, const MatRecord *__restrict__ mats,
    const LightRecord *__restrict__ lights, const float *__restrict__ gamma_t,
    uint32_t *__restrict__ out_rgba, float *__restrict__ out_lin,
    unsigned long long *__restrict__ counters, const SurfRecord *__restrict__ surf,
    const FaceShade *__restrict__ shade)
{
    __shared__ uint8_t tail_tab[kBlock / kWave][kWave];
    __shared__ float4 compact_lds[kBlock / kWave * 2 * kWave];
    __shared__ float state_lds[kStateCols * kBlock];
    path_body<false, false, false, true>(
        A, tri, mats, lights, gamma_t, out_rgba, out_lin, counters, surf, shade, tail_tab,
        nullptr, nullptr, nullptr, nullptr, compact_lds, state_lds);
}
#endif  // RVCP_JIT
}  // namespace rvcp

#ifndef RVCP_JIT

extern "C" int rvcp_launch_games101(const rvcp::FrameArgs *args, const rvcp::TriRecord *tri,
                                    const void *faces, const void *verts,
                                    const rvcp::MatRecord *mats, const rvcp::LightRecord *lights,
                                    const float *gamma_t, uint32_t *out_rgba, float *out_lin,
                                    unsigned long long *counters, uint32_t grid_blocks,
                                    void *stream)
{
    auto kern = args->variant == 2 ? rvcp::games101_dual_kernel : rvcp::games101_kernel;
    hipLaunchKernelGGL(kern, dim3(grid_blocks), dim3(rvcp::kBlock), 0, (hipStream_t)stream,
                       *args, tri, (const rvcp_face_t *)faces, (const rvcp_vertex_t *)verts, mats,
                       lights, gamma_t, out_rgba, out_lin, counters);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_launch_games101_v3(const rvcp::FrameArgs *args, uint32_t n_frames,
                                       uint32_t frame_stride, const rvcp::TriRecord *tri,
                                       const void *faces, const void *verts,
                                       const rvcp::MatRecord *mats,
                                       const rvcp::LightRecord *lights, const float *gamma_t,
                                       uint32_t *out_rgba, float *out_lin,
                                       unsigned long long *counters, rvcp::SurfRecord *surf,
                                       const rvcp::FaceShade *shade,
                                       const rvcp::Bvh4Node *bvh_nodes,
                                       const rvcp::TriRecord *bvh_tris,
                                       uint32_t grid_blocks, void *stream, void *main_event,
                                       void *spec_path_fn, const float *cams, void *spec_pre_fn)
{
    const uint32_t pre_blocks = (args->n_pixels + rvcp::kPrimaryBlock - 1) / rvcp::kPrimaryBlock;
    auto pre = args->accel ? rvcp::games101_primary_kernel<true> : rvcp::games101_primary_kernel<false>;
    // the frames' pre-passes append to one surface list (the path kernel reads each record's
    // pixel and seed, so the list's order is free): a batch with its cameras in device memory
    // in one launch, one frame per grid row, else one launch per frame
    if (spec_pre_fn) {
        // the specialised pre-pass (same parameters as games101_primary_kernel; with the BVH:
        // the hybrid's, rvcp_spec_bvh_primary_kernel)
        const bool batch = cams && n_frames > 1;
        for (uint32_t k = 0; k < (batch ? 1u : n_frames); ++k) {
            rvcp::FrameArgs a = args[k];
            const void *p_faces = faces, *p_verts = verts;
            const rvcp::Bvh4Node *p_nodes = bvh_nodes;
            const rvcp::TriRecord *p_btris = bvh_tris;
            const float *p_cams = batch ? cams : nullptr;
            uint32_t p_stride = batch ? frame_stride : 0u;
            void *params[] = {&a, &tri, &p_faces, &p_verts, &mats, &gamma_t, &out_rgba, &out_lin,
                              &counters, &surf, &shade, &p_nodes, &p_btris, &p_cams, &p_stride};
            if (hipModuleLaunchKernel((hipFunction_t)spec_pre_fn, pre_blocks, batch ? n_frames : 1u,
                                      1, rvcp::kPrimaryBlock, 1, 1, 0, (hipStream_t)stream, params,
                                      nullptr) != hipSuccess)
                return -2;
        }
    } else if (cams && n_frames > 1)
        hipLaunchKernelGGL(pre, dim3(pre_blocks, n_frames), dim3(rvcp::kPrimaryBlock), 0,
                           (hipStream_t)stream, args[0], tri, (const rvcp_face_t *)faces,
                           (const rvcp_vertex_t *)verts, mats, gamma_t, out_rgba, out_lin, counters,
                           surf, shade, bvh_nodes, bvh_tris, cams, frame_stride);
    else
        for (uint32_t k = 0; k < n_frames; ++k)
            hipLaunchKernelGGL(pre, dim3(pre_blocks), dim3(rvcp::kPrimaryBlock), 0,
                               (hipStream_t)stream, args[k], tri, (const rvcp_face_t *)faces,
                               (const rvcp_vertex_t *)verts, mats, gamma_t, out_rgba, out_lin,
                               counters, surf, shade, bvh_nodes, bvh_tris, (const float *)nullptr,
                               0u);
    if (main_event && hipEventRecord((hipEvent_t)main_event, (hipStream_t)stream) != hipSuccess)
        return -2;
    if (spec_path_fn && args->accel) {
        // the BVH hybrid's path kernel (rvcp_spec_bvh_path_kernel, games101_bvh_path_kernel's
        // signature)
        rvcp::FrameArgs a = *args;
        void *params[] = {&a, &tri, &mats, &lights, &gamma_t, &out_rgba, &out_lin, &counters,
                          &surf, &shade, &bvh_nodes, &bvh_tris};
        if (hipModuleLaunchKernel((hipFunction_t)spec_path_fn, grid_blocks, 1, 1, rvcp::kBlock,
                                  1, 1, 0, (hipStream_t)stream, params, nullptr) != hipSuccess)
            return -2;
    } else if (spec_path_fn) {
        // the scene-specialised schedule 3 / 6 kernel of rvcp_jit.cpp (same signature)
        rvcp::FrameArgs a = *args;
        void *params[] = {&a, &tri, &mats, &lights, &gamma_t, &out_rgba, &out_lin, &counters,
                          &surf, &shade};
        if (hipModuleLaunchKernel((hipFunction_t)spec_path_fn, grid_blocks, 1, 1, rvcp::kBlock,
                                  1, 1, 0, (hipStream_t)stream, params, nullptr) != hipSuccess)
            return -2;
    } else if (args->accel)
        hipLaunchKernelGGL(rvcp::games101_bvh_path_kernel, dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                           (hipStream_t)stream, *args, tri, mats, lights, gamma_t, out_rgba,
                           out_lin, counters, surf, shade, bvh_nodes, bvh_tris);
    else if (args->variant == 10)
        hipLaunchKernelGGL(rvcp::games101_tiled_pool_kernel, dim3(grid_blocks), dim3(rvcp::kTiledPoolWaves * rvcp::kWave), 0,
                           (hipStream_t)stream, *args, tri, mats, lights, gamma_t, out_rgba,
                           out_lin, counters, surf, shade);
    else if (args->variant == 5)
        hipLaunchKernelGGL(rvcp::games101_tiled_single_kernel, dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                           (hipStream_t)stream, *args, tri, mats, lights, gamma_t, out_rgba,
                           out_lin, counters, surf, shade);
    else if (args->variant == 4)
        hipLaunchKernelGGL(rvcp::games101_tiled_kernel, dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                           (hipStream_t)stream, *args, tri, mats, lights, gamma_t, out_rgba,
                           out_lin, counters, surf, shade);
    else
        hipLaunchKernelGGL(args->variant == 6 ? rvcp::games101_path_kernel<6>
                                              : rvcp::games101_path_kernel<rvcp::kPathMinWaves>,
                           dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                           (hipStream_t)stream, *args, tri, mats, lights, gamma_t, out_rgba,
                           out_lin, counters, surf, shade);
    if (hipGetLastError() != hipSuccess) return -2;
    // the frame's UNORM8 store from the linear colours (out_lin is never null here); a batch's
    // frames lie frame_stride pixels apart (the rows of a smaller shard's slot are padding)
    const uint32_t n_tone = n_frames > 1 ? n_frames * frame_stride : args->n_pixels;
    uint32_t tb = (n_tone + rvcp::kToneBlock - 1) / rvcp::kToneBlock;
    if (tb > 8192u) tb = 8192u;
    hipLaunchKernelGGL(rvcp::tonemap_kernel, dim3(tb), dim3(rvcp::kToneBlock), 0, (hipStream_t)stream,
                       out_lin, n_tone, gamma_t, out_rgba);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" void rvcp_static_split(uint32_t n, uint32_t grid_waves, uint32_t n_simds,
                                  uint32_t *waves, uint32_t *chunk)
{
    rvcp::static_split(n, grid_waves, n_simds, *waves, *chunk);
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
    const uint32_t blocks = n ? ((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096) : 1;
    hipLaunchKernelGGL(rvcp::fill_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       out_rgba, out_lin, n, rgba);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_games101_occupancy(int variant, int *blocks_per_cu)
{
    int b = 0;
    const hipError_t e = variant == rvcp::kOccupancyBvh
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_bvh_path_kernel, rvcp::kBlock, 0)
        : variant == 5
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_tiled_single_kernel, rvcp::kBlock, 0)
        : variant == 4
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_tiled_kernel, rvcp::kBlock, 0)
        : variant == 10
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_tiled_pool_kernel, rvcp::kTiledPoolWaves * rvcp::kWave, 0)
        : variant == 6
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_path_kernel<6>, rvcp::kBlock, 0)
        : variant == 3
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_path_kernel<rvcp::kPathMinWaves>, rvcp::kBlock, 0)
        : variant == 2
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_dual_kernel, rvcp::kBlock, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::games101_kernel, rvcp::kBlock, 0);
    if (e != hipSuccess) return -2;
    *blocks_per_cu = b;
    return 0;
}

extern "C" int rvcp_launch_legacy(const rvcp::FrameArgs *args, const rvcp::TriRecord *tri,
                                  const rvcp::FaceShade *shade, const void *spheres,
                                  const void *materials, const float *unorm_t, uint32_t *out_rgba,
                                  float *out_lin, unsigned long long *counters,
                                  uint32_t grid_blocks, void *stream, void *spec_legacy_fn)
{
    if (spec_legacy_fn) {
        // the mode-2 kernel with the scene-specialised triangle scan (rvcp_jit.cpp)
        rvcp::FrameArgs a = *args;
        void *params[] = {&a, &tri, &shade, &spheres, &materials, &unorm_t, &out_rgba, &out_lin,
                          &counters};
        if (hipModuleLaunchKernel((hipFunction_t)spec_legacy_fn, grid_blocks, 1, 1, rvcp::kBlock,
                                  1, 1, 0, (hipStream_t)stream, params, nullptr) != hipSuccess)
            return -2;
    } else {
        hipLaunchKernelGGL(rvcp::legacy_kernel, dim3(grid_blocks), dim3(rvcp::kBlock), 0,
                           (hipStream_t)stream, *args, tri, shade, (const rvcp_sphere_t *)spheres,
                           (const rvcp_material_t *)materials, unorm_t, out_rgba, out_lin, counters);
        if (hipGetLastError() != hipSuccess) return -2;
    }
    // the frame's UNORM8 store (no gamma in mode 2) from the linear colours (a batch's frames
    // frame_stride pixels apart)
    const uint32_t n_tone = args->batch_cams ? args->n_pixels / args->frame_pixels * args->frame_stride
                                             : args->n_pixels;
    uint32_t tb = (n_tone + rvcp::kToneBlock - 1) / rvcp::kToneBlock;
    if (tb > 8192u) tb = 8192u;
    hipLaunchKernelGGL(rvcp::tonemap_kernel, dim3(tb), dim3(rvcp::kToneBlock), 0, (hipStream_t)stream,
                       out_lin, n_tone, unorm_t, out_rgba);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int rvcp_legacy_occupancy(int *blocks_per_cu)
{
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rvcp::legacy_kernel, rvcp::kBlock, 0) !=
        hipSuccess)
        return -2;
    *blocks_per_cu = b;
    return 0;
}
#endif  // RVCP_JIT
