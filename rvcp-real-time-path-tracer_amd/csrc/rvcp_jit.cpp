// rvcp_jit.cpp -- scene-specialised path kernels.
//
// The brute-force nearest-hit scan of the path kernels (schedules 3 and 6) tests every ray
// against every triangle with the exact operation sequence of the numeric contract (DESIGN.md
// §3.1, §3.5): ~42 VALU instructions per test, read from a triangle record in SGPRs.  For a
// small scene (the reference's Cornell box: 32 triangles) this module generates, at upload,
// source code in which every triangle's test is written out with its v0 / e1 / e2 as literals
// and every product with an exact-zero triangle component dropped (axis-aligned walls and box
// faces have a third of their edge components zero), compiles rvcp_kernels.hip around it with
// hipRTC for gfx950, and hands the host the two kernels.
//
// Why the result is bit-identical to the generic scan (for rays within ray_in_range and
// t_min > 0; the kernel falls back to the generic loop for a wave holding any other ray, and
// the host uses the generic kernels when ray_t_min <= 0 or a coordinate is out of range):
//  * a dropped term is a product c * x with c = +0 or -0 and x finite, i.e. a zero (x is
//    finite because nothing overflows: the scene is specialised only within jit_scene_in_range's
//    bounds and a wave uses the scan only when its rays pass ray_in_range); removing a
//    zero addend from a correctly rounded sum or fma changes at most the sign of a zero result;
//  * so every intermediate equals the generic one up to the sign of zero, and the values that
//    reach a decision are: f = 1/den (den = +-0 gives f = +-inf, and then t = +-inf or NaN is
//    rejected by t >= t_min > 0 or t <= bt either way), b1, b2 (compared with >= 0 and
//    b1 + b2 <= 1, blind to the sign of zero), t (an accepted t >= t_min > 0 is non-zero, so
//    its bits are the generic ones);
//  * a triangle whose denominator is identically zero is never accepted and is omitted; a
//    vanished b1 or b2 drops its ">= 0" test, which a finite f would pass and an infinite f
//    rejects through t anyway;
//  * triangles are tested in index order with the shader's "t <= bt" rule, as the loop does.
//
// hipRTC is loaded at run time (dlopen), like RCCL: without it, or if compilation fails, the
// context keeps the generic kernels (frames are the same either way).
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <map>
#include <string>
#include <vector>

#include "rvcp_internal.h"
#include "rvcp_jit.h"
#include "build/rvcp_jit_src.h"   // kJitSrcKernels, kJitSrcInternal, kJitSrcAbi (Makefile)

namespace rvcp {
namespace {

// ------------------------------------------------------------------ hipRTC, dlopen()ed --
typedef int rtc_result;
typedef void *rtc_program;
struct RtcApi {
    bool ok = false;
    std::string why;
    rtc_result (*create)(rtc_program *, const char *, const char *, int, const char *const *,
                         const char *const *) = nullptr;
    rtc_result (*compile)(rtc_program, int, const char *const *) = nullptr;
    rtc_result (*log_size)(rtc_program, size_t *) = nullptr;
    rtc_result (*log)(rtc_program, char *) = nullptr;
    rtc_result (*code_size)(rtc_program, size_t *) = nullptr;
    rtc_result (*code)(rtc_program, char *) = nullptr;
    rtc_result (*destroy)(rtc_program *) = nullptr;
    rtc_result (*version)(int *, int *) = nullptr;     // optional: part of the disk-cache key
};

const RtcApi &rtc()
{
    static RtcApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"libhiprtc.so", "libhiprtc.so.7", "/opt/rocm/lib/libhiprtc.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!h) {
            api.why = "libhiprtc not found";
            return;
        }
        api.create = (decltype(api.create))dlsym(h, "hiprtcCreateProgram");
        api.compile = (decltype(api.compile))dlsym(h, "hiprtcCompileProgram");
        api.log_size = (decltype(api.log_size))dlsym(h, "hiprtcGetProgramLogSize");
        api.log = (decltype(api.log))dlsym(h, "hiprtcGetProgramLog");
        api.code_size = (decltype(api.code_size))dlsym(h, "hiprtcGetCodeSize");
        api.code = (decltype(api.code))dlsym(h, "hiprtcGetCode");
        api.destroy = (decltype(api.destroy))dlsym(h, "hiprtcDestroyProgram");
        api.version = (decltype(api.version))dlsym(h, "hiprtcVersion");
        api.ok = api.create && api.compile && api.log_size && api.log && api.code_size &&
                 api.code && api.destroy;
        if (!api.ok) api.why = "libhiprtc lacks a required symbol";
    });
    return api;
}

// ------------------------------------------------------------------ source generator ----
// A value of the generated expression graph: an exact zero, a named float, or a non-zero
// literal (the triangle's own float, written as its bit pattern), each with a sign: the value
// is -|x| when `neg` is set.  Signs are carried, not computed -- RN(-x) = -RN(x), so a
// product or fma with negated operands is the negation of the one with positive operands
// (exactly, up to the sign of a zero result, which the header's argument already allows) --
// and `key` spells the magnitude's whole expression with commutative operands in a fixed
// order, so that equal expressions anywhere in the scan are computed once: the shared
// denominator of an axis-aligned quad's two triangles, the products d.y * c they repeat, ...
//
// `grain`: every value is an integer multiple of 2^grain (kNoGrain: not known).  A literal's is
// its lowest set bit; a ray direction component's is kDirGrain, which the kernel's per-wave
// check dir_grain_ok establishes (every component 0 or at least 2^-40 in magnitude, so a multiple
// of its ulp >= 2^-63); o's is not known.  The exact product, sum or fma of multiples of 2^ga and
// 2^gb is a multiple of 2^(ga + gb) resp. 2^min(ga, gb), and rounding to float keeps a multiple of
// 2^g (g >= -149) a multiple of 2^g, non-zero values at least 2^g in magnitude (2^g is a float
// and rounding is monotone).  `mag`: |value| <= 2^mag (ray_in_range: |d_i| <= 16, |o_i| <=
// 2^41; a product 2^(ma + mb), a sum or fma 2^(max + 1), rounding being monotone).  So a
// non-zero denominator with grain >= -126 and mag <= 126 is a normal number whose reciprocal is
// normal, and the kernel's 1/den needs no class check (rcp_scan_fast).
constexpr int kNoGrain = -100000;
constexpr int kNoMag = 100000;
constexpr int kDirGrain = -63;             // dir_grain_ok's bound 2^-40, 23 fraction bits
constexpr int kDirMag = 4, kOrgMag = 41;   // ray_in_range's |d|_1 <= 16, |o|_1 <= 2^41
struct Val {
    enum Kind { kZero, kVar, kLit } kind = kZero;
    std::string name;       // kVar: the variable holding the magnitude
    float lit = 0.0f;       // kLit: the magnitude (> 0)
    bool neg = false;
    std::string key = "0";  // the magnitude's expression
    int grain = kNoGrain;
    int mag = kNoMag;
};
int mag_mul(int a, int b) { return (a == kNoMag || b == kNoMag) ? kNoMag : a + b; }
int mag_sum(int a, int b) { return (a == kNoMag || b == kNoMag) ? kNoMag : std::max(a, b) + 1; }

int grain_of(float x)       // the exponent of x's lowest set bit (x finite, non-zero)
{
    int e = 0;
    const float m = std::frexp(std::fabs(x), &e);    // x = m 2^e, m in [0.5, 1)
    uint32_t s = (uint32_t)std::ldexp(m, 24);        // exact for normal x
    if (s == 0) return kNoGrain;
    int g = e - 24;
    while ((s & 1u) == 0) { s >>= 1; g += 1; }
    return g < -149 ? kNoGrain : g;
}
int grain_mul(int a, int b) { return (a == kNoGrain || b == kNoGrain || a + b < -149) ? kNoGrain : a + b; }
int grain_min(int a, int b) { return (a == kNoGrain || b == kNoGrain) ? kNoGrain : std::min(a, b); }

std::string lit_text(float x)
{
    uint32_t bits;
    std::memcpy(&bits, &x, 4);
    char buf[48];
    std::snprintf(buf, sizeof buf, "RVCP_F32(0x%08xu)", bits);
    return buf;
}

Val zero() { return Val{}; }
Val var(const std::string &n, int grain = kNoGrain, int mag = kNoMag)
{
    Val v;
    v.kind = Val::kVar;
    v.name = n;
    v.key = n;
    v.grain = grain;
    v.mag = mag;
    return v;
}
Val lit_or_zero(float x)
{
    if (x == 0.0f) return zero();          // +0 and -0: dropped terms (see the header)
    Val v;
    v.kind = Val::kLit;
    v.lit = std::fabs(x);
    v.neg = std::signbit(x);
    v.key = lit_text(v.lit);
    v.grain = grain_of(x);
    int e = 0;
    (void)std::frexp(v.lit, &e);           // |x| < 2^e
    v.mag = e;
    return v;
}
Val negate(Val v)
{
    if (v.kind != Val::kZero) v.neg = !v.neg;
    return v;
}
Val magnitude(Val v)
{
    v.neg = false;
    return v;
}
std::string signed_key(const Val &v) { return (v.neg ? "-" : "+") + v.key; }

struct Gen {
    std::string out;
    int n = 0;
    // expressions already computed by an earlier test of the same scan: key -> variable (the
    // scan's temporaries are declared at function scope, so a later test can use them)
    std::map<std::string, std::string> *seen = nullptr;

    std::string prefix;
    std::string text(const Val &v) const
    {
        if (v.kind == Val::kLit) return lit_text(v.neg ? -v.lit : v.lit);
        return v.neg ? "(-" + v.name + ")" : v.name;
    }
    // (the grain is a function of the key, so a value found in `seen` has the one given here)
    Val tmp(const std::string &expr, const std::string &key, int grain = kNoGrain,
            int mag = kNoMag)
    {
        if (seen) {
            const auto it = seen->find(key);
            if (it != seen->end()) {
                Val v = var(it->second, grain, mag);
                v.key = key;
                return v;
            }
        }
        const std::string name = prefix + "r" + std::to_string(n++);
        out += "    const float " + name + " = " + expr + ";\n";
        if (seen) (*seen)[key] = name;
        Val v = var(name, grain, mag);
        v.key = key;
        return v;
    }
    // |a| * |b| (commutative: operands in key order), carrying the sign
    Val mul(const Val &a, const Val &b)
    {
        if (a.kind == Val::kZero || b.kind == Val::kZero) return zero();
        const bool swap = b.key < a.key;
        const Val &x = swap ? b : a, &y = swap ? a : b;
        Val r = tmp(text(magnitude(x)) + " * " + text(magnitude(y)), "m(" + x.key + "," + y.key + ")",
                    grain_mul(a.grain, b.grain), mag_mul(a.mag, b.mag));
        r.neg = a.neg != b.neg;
        return r;
    }
    Val neg(const Val &a) { return negate(a); }
    // fma(a, b, c) = s * fma(|a|, |b|, s * c) with s the product's sign
    Val fma(const Val &a, const Val &b, const Val &c)
    {
        if (a.kind == Val::kZero || b.kind == Val::kZero) return c;
        if (c.kind == Val::kZero) return mul(a, b);
        const bool sp = a.neg != b.neg;
        const Val cc = sp ? negate(c) : c;
        const bool swap = b.key < a.key;
        const Val &x = swap ? b : a, &y = swap ? a : b;
        Val r = tmp("__builtin_fmaf(" + text(magnitude(x)) + ", " + text(magnitude(y)) + ", " +
                        text(cc) + ")",
                    "f(" + x.key + "," + y.key + "," + signed_key(cc) + ")",
                    grain_min(grain_mul(a.grain, b.grain), c.grain),
                    mag_sum(mag_mul(a.mag, b.mag), c.mag));
        r.neg = sp;
        return r;
    }
    Val sub(const Val &a, const Val &b)       // a - b; x - (+-0) == x exactly, so b = 0 drops
    {
        if (b.kind == Val::kZero) return a;
        return tmp(text(a) + " - " + text(b), "s(" + signed_key(a) + "," + signed_key(b) + ")",
                   grain_min(a.grain, b.grain), mag_sum(a.mag, b.mag));
    }
    // dot = fma(z, z', fma(y, y', x*x')), cross_i = fma(a_j, b_k, -(a_k*b_j)): DESIGN.md §3.1
    Val dot(const Val *a, const Val *b) { return fma(a[2], b[2], fma(a[1], b[1], mul(a[0], b[0]))); }
    // component k of a x b; a component of a whose partners in b are both zero is not read
    // (it may be a placeholder zero: the terms it would enter are dropped anyway)
    Val cross_at(const Val *a, const Val *b, int k)
    {
        const int i = (k + 1) % 3, j = (k + 2) % 3;
        return fma(a[i], b[j], neg(mul(a[j], b[i])));
    }
    void cross(const Val *a, const Val *b, Val *r)
    {
        for (int k = 0; k < 3; k++) r[k] = cross_at(a, b, k);
    }
};

// Per ray: the t of its previous test and the name of that test's range mask, tmin <= t <= bt
// evaluated before it.  The next test of the ray with the same t (the other triangle of an
// axis-aligned quad: one plane, one denominator, one t) reuses the mask: between the two tests
// bt changed only if the first accepted, and then to t itself, so t <= bt holds before the
// second exactly when it held before the first (2 of the 5 compares of a quad's second test).
struct RangeMask {
    std::string t, name;
    // tests of this ray with this t whose acceptance is still to be applied (emit_scan's quad
    // regions): their acceptance flags and face indices, in order
    std::vector<std::pair<std::string, uint32_t>> pending;
};

// One triangle's test for ray `r` ("" / "A" / "B"), split into its arithmetic (`decl`: every
// value that does not depend on the running nearest hit, temporaries named <prefix>r<k>, then
// the range mask, which reads the nearest hit as the previous commit left it) and its
// acceptance (`accept`: the update); false when it can never accept.
//
// `inner` (the dual scan's shadow slot, emit_scan): the arithmetic is split at the range mask.
// `decl` gets what t and the mask need (s, s1 = d x e2, den, s2 = s x e1, dot(s2, e2), f, t,
// mask), `*inner` the rest (n1, n2, b1, b2, the compares) -- code the caller places inside a
// wave-uniform `if (RVCP_SPEC_ANY(mask))`, so its temporaries go to `inner_seen` and never to
// `seen` (a later test must not name a value a skipped block did not compute).  The same
// operations on the same values as the unsplit order, so the same results.
bool emit_triangle(std::string &decl, std::string &accept, const TriRecord &T, uint32_t index,
                   const char *r, std::map<std::string, std::string> &seen,
                   std::map<std::string, RangeMask> &prev, bool *reused = nullptr,
                   bool defer = false, std::string *inner = nullptr,
                   std::map<std::string, std::string> *inner_seen = nullptr, bool eager = false)
{
    Gen g;
    g.seen = &seen;
    g.prefix = "t" + std::to_string(index) + r + "_";
    const std::string R(r);
    Val o[3] = {var("o" + R + ".x", kNoGrain, kOrgMag), var("o" + R + ".y", kNoGrain, kOrgMag),
                var("o" + R + ".z", kNoGrain, kOrgMag)};
    Val d[3] = {var("d" + R + ".x", kDirGrain, kDirMag), var("d" + R + ".y", kDirGrain, kDirMag),
                var("d" + R + ".z", kDirGrain, kDirMag)};
    Val v0[3], e1[3], e2[3];
    for (int k = 0; k < 3; k++) {
        v0[k] = lit_or_zero(T.v0[k]);
        e1[k] = lit_or_zero(T.e1[k]);
        e2[k] = lit_or_zero(T.e2[k]);
    }
    Val s[3], s1[3], s2[3];
    Val n1, n2, den, tt;
    // `inner`: s, s1 = d x e2 and s2 = s x e1 component by component, as t and the mask need
    // them (den reads the components of s1 where e1 is non-zero, dot(s2, e2) those of s2 where
    // e2 is), so that the ones only n1 and n2 read are computed after the split, inside the
    // skippable block -- the same operations on the same operands in either order
    bool have_s[3] = {}, have_s1[3] = {}, have_s2[3] = {};
    auto S = [&](int k) {
        if (!have_s[k]) { s[k] = g.sub(o[k], v0[k]); have_s[k] = true; }
        return s[k];
    };
    auto S1 = [&](int k) {
        if (!have_s1[k]) { s1[k] = g.cross_at(d, e2, k); have_s1[k] = true; }
        return s1[k];
    };
    auto S2 = [&](int k) {
        if (!have_s2[k]) {
            const int i = (k + 1) % 3, j = (k + 2) % 3;
            Val a[3];
            if (e1[j].kind != Val::kZero) a[i] = S(i);
            if (e1[i].kind != Val::kZero) a[j] = S(j);
            s2[k] = g.cross_at(a, e1, k);
            have_s2[k] = true;
        }
        return s2[k];
    };
    const bool lazy = inner && !eager;      // eager: the round-5 (r05h) order, an A/B knob
    if (lazy) {
        Val s1p[3];
        for (int k = 0; k < 3; k++) s1p[k] = e1[k].kind != Val::kZero ? S1(k) : zero();
        den = g.dot(s1p, e1);                                                  // :254
    } else {
        for (int k = 0; k < 3; k++) S(k);                                      // :249
        g.cross(d, e2, s1);                                                    // :250
        have_s1[0] = have_s1[1] = have_s1[2] = true;
        den = g.dot(s1, e1);                                                   // :254
    }
    if (den.kind == Val::kZero) {
        decl += g.out;          // its temporaries may be named by a later test (`seen`)
        return false;
    }
    if (lazy) {
        Val s2p[3];
        for (int k = 0; k < 3; k++) s2p[k] = e2[k].kind != Val::kZero ? S2(k) : zero();
        tt = g.dot(s2p, e2);
    } else {
        g.cross(s, e1, s2);                                                    // :251
        have_s2[0] = have_s2[1] = have_s2[2] = true;
        if (!inner) {
            n1 = g.dot(s1, s);
            n2 = g.dot(s2, d);
        }
        tt = g.dot(s2, e2);
    }
    // the reciprocal of the signed denominator (its sign stays inside: v_rcp's symmetry is
    // not relied on); without the class check when the denominator is zero or a normal number
    // whose reciprocal is normal (grain >= -126, mag <= 126: see Val)
    const char *rcp = den.grain != kNoGrain && den.grain >= -126 && den.mag <= 126
                          ? "RVCP_SPEC_RCP_FAST(" : "RVCP_SPEC_RCP(";
    const Val f = g.tmp(rcp + g.text(den) + ")", "r(" + signed_key(den) + ")");   // :254
    // t = f * dot(s2, e2) (:255); a vanished dot leaves t = +-0 or NaN, rejected by
    // t >= t_min > 0 in both forms
    const std::string t = tt.kind == Val::kZero ? std::string("0.0f") : g.text(g.mul(f, tt));
    size_t split_at = std::string::npos;
    if (inner) {
        // the rest after the mask: into *inner, its temporaries into inner_seen (a copy of the
        // values visible here plus its own)
        split_at = g.out.size();
        *inner_seen = seen;
        g.seen = inner_seen;
        Val s1f[3], sf[3], s2f[3];
        for (int k = 0; k < 3; k++) s1f[k] = S1(k);
        for (int k = 0; k < 3; k++) sf[k] = s1f[k].kind != Val::kZero ? S(k) : zero();
        n1 = g.dot(s1f, sf);
        for (int k = 0; k < 3; k++) s2f[k] = S2(k);
        n2 = g.dot(s2f, d);
    }
    std::string cond;
    auto add = [&](const std::string &c) { cond += (cond.empty() ? "" : " & ") + c; };
    std::string b1, b2;
    if (n1.kind != Val::kZero) b1 = g.text(g.mul(f, n1));                     // :256
    if (n2.kind != Val::kZero) b2 = g.text(g.mul(f, n2));                     // :257
    if (!b1.empty()) add("(" + b1 + " >= 0.0f)");
    if (!b2.empty()) add("(" + b2 + " >= 0.0f)");
    if (!b1.empty() && !b2.empty()) add("(" + b1 + " + " + b2 + " <= 1.0f)");
    else if (!b1.empty()) add("(" + b1 + " <= 1.0f)");
    else if (!b2.empty()) add("(" + b2 + " <= 1.0f)");
    if (inner) {
        decl += g.out.substr(0, split_at);
        *inner += g.out.substr(split_at);
    } else {
        decl += g.out;
    }
    RangeMask &pm = prev[R];
    if (reused) *reused = !pm.name.empty() && pm.t == t;
    if (pm.name.empty() || pm.t != t) {
        pm.t = t;
        pm.name = g.prefix + "q";
        decl += "    const bool " + pm.name + " = (" + t + " >= tmin) & (" + t + " <= bt" + R + ");\n";
    }
    add(pm.name);
    // the dual scan's shadow ray (slot A) needs the nearest t and whether there was a hit, not
    // the face: only its t is kept (btA != t_max after the scan means a hit;
    // the caller resolves btA == t_max, a miss or a hit at exactly t_max, with the generic scan)
    if (defer) {
        // the next test of this ray has the same t: keep the flag, apply both together
        const std::string c = g.prefix + "c";
        accept += "        " + c + " = " + cond + ";\n";
        (inner ? *inner : decl) += "    bool " + c + ";\n";
        pm.pending.emplace_back(c, index);
        return true;
    }
    if (!pm.pending.empty()) {
        // the last test of a run with one t: bt takes t if any test of the run accepted, the
        // face is the last accepting one (the order the sequential updates would leave)
        const std::string c = g.prefix + "c";
        std::string any = c, best = "best" + R;
        for (const auto &pc : pm.pending) {
            any += " | " + pc.first;
            best = "(" + pc.first + " ? " + std::to_string(pc.second) + " : " + best + ")";
        }
        accept += "        const bool " + c + " = " + cond + ";\n";
        accept += "        if (" + any + ") bt" + R + " = " + t + ";\n";
        if (R != "A")
            accept += "        best" + R + " = " + c + " ? " + std::to_string(index) + " : " + best + ";\n";
        pm.pending.clear();
        return true;
    }
    if (R == "A")
        accept += "        if (" + cond + ") btA = " + t + ";\n";
    else
        accept += "        if (" + cond + ") { bt" + R + " = " + t + "; best" + R + " = " +
                  std::to_string(index) + "; }\n";
    return true;
}

// One test per commit: RVCP_SPEC_COMMIT(t, i) after each test makes its result final before
// the next test starts (without it the compiler interleaves all unrolled tests and spills
// hundreds of registers), in the order (0, A), (0, B), (1, A), ... of the dual scan.  Groups of
// two or four tests between commits (their arithmetic first, then the acceptances in order)
// measured within +-1 % and were removed: a range mask (RangeMask) must read
// the nearest hit after the previous test's acceptance, which a group's shared prologue does
// not.
//
// Except inside a quad (round 4): a test whose ray's next test reuses its range mask (the same
// t, RangeMask) is not committed on its own -- the two tests of each ray and the other ray's
// tests between them form one region, so the compiler can merge the two acceptances of a ray
// (both write the same t) into one select of bt.
void emit_scan(std::string &out, const TriRecord *tri, uint32_t n, const char *const *rays,
               int n_rays, unsigned opts = 0)
{
    const bool skip_b = (opts & kScanSkipB) != 0, eager = (opts & kScanEagerSplit) != 0;
    const uint32_t N = n * (uint32_t)n_rays;
    std::vector<char> used(N), reused(N);
    {   // dry run: which tests are emitted and which reuse their ray's previous range mask
        std::map<std::string, std::string> seen;
        std::map<std::string, RangeMask> prev;
        for (uint32_t u = 0; u < N; u++) {
            std::string decl, accept;
            bool ru = false;
            used[u] = emit_triangle(decl, accept, tri[u / (uint32_t)n_rays], u / (uint32_t)n_rays,
                                    rays[u % (uint32_t)n_rays], seen, prev, &ru);
            reused[u] = used[u] && ru;
        }
    }
    std::map<std::string, std::string> seen;
    std::map<std::string, RangeMask> prev;
    // this ray's next emitted test after u, and whether it shares u's range mask
    auto next_used = [&](uint32_t u) {
        uint32_t v = u + (uint32_t)n_rays;
        while (v < N && !used[v]) v += (uint32_t)n_rays;
        return v;
    };
    auto defers = [&](uint32_t u) {
        const uint32_t v = next_used(u);
        return used[u] && v < N && reused[v];
    };
    // The single-ray scan (and the dual scan's path slot B): one test per commit region, or
    // a run of tests sharing one range mask (an axis-aligned quad) in one region.
    auto emit_plain = [&](uint32_t u) {
        std::string decl, accept;
        const std::string R(rays[u % (uint32_t)n_rays]);
        const bool defer = defers(u);
        emit_triangle(decl, accept, tri[u / (uint32_t)n_rays], u / (uint32_t)n_rays, R.c_str(),
                      seen, prev, nullptr, defer);
        out += decl;
        if (!used[u]) return;
        out += "    {\n" + accept + "    }\n";
        if (defer) return;
        out += R == "A" ? "    RVCP_SPEC_COMMIT1(btA);\n"
                        : "    RVCP_SPEC_COMMIT(bt" + R + ", best" + R + ");\n";
    };
    if (n_rays == 1) {
        for (uint32_t u = 0; u < N; u++) emit_plain(u);
        return;
    }
    // The dual scan: per triangle (run), the shadow slot A, then the path slot B.  Slot A's
    // tests are emitted as runs of tests sharing one range mask, each split at the mask: the
    // first test's t and mask, then `if (RVCP_SPEC_ANY(mask)) { the rest of the run }`.  A
    // wave whose shadow rays all have t outside [t_min, btA] skips the barycentric half of the
    // run -- every one of them would reject it (the mask is part of every acceptance), so the
    // result is unchanged.  Shadow rays all end on a luminous face, which the scan tests first
    // in the Cornell box (faces 0, 1), so btA is that short distance for most of the scan and
    // the walls, floor and ceiling behind it are out of range for the whole wave.
    // a run of one ray's tests, split at the first test's mask into a skippable block
    auto emit_split_run = [&](const std::vector<uint32_t> &run, const char *R) {
        std::map<std::string, std::string> inner_seen;
        std::string head, body, accept;
        for (size_t k = 0; k < run.size(); k++) {
            const uint32_t u = run[k];
            const bool defer = k + 1 < run.size();
            std::string decl, inner, acc;
            if (k == 0) {
                emit_triangle(decl, acc, tri[u / 2], u / 2, R, seen, prev, nullptr, defer,
                              &inner, &inner_seen, eager);
                head += decl;
                body += inner;
            } else {
                emit_triangle(decl, acc, tri[u / 2], u / 2, R, inner_seen, prev, nullptr, defer);
                body += decl;
            }
            accept += acc;
        }
        const std::string &mask = prev[R].name;
        const std::string r(R);
        out += head;
        out += "    if (RVCP_SPEC_ANY(" + mask + ")) {\n" + body + "    {\n" + accept + "    }\n    }\n";
        out += r == "A" ? "    RVCP_SPEC_COMMIT1(btA);\n" : "    RVCP_SPEC_COMMIT(bt" + r + ", best" + r + ");\n";
    };
    for (uint32_t i = 0; i < n;) {
        const uint32_t uA = 2 * i;
        if (!used[uA]) {                  // den identically zero: omitted for both rays
            emit_plain(uA);
            emit_plain(uA + 1);
            i += 1;
            continue;
        }
        std::vector<uint32_t> run = {uA};
        while (defers(run.back())) run.push_back(next_used(run.back()));
        emit_split_run(run, "A");
        // slot B: the same triangles, as before (or split too: skip_b, an experiment knob --
        // path rays rarely leave a whole wave out of range, and the split costs slot B the
        // sharing of values across tests)
        if (skip_b) {
            std::vector<uint32_t> runB;
            for (uint32_t u : run) runB.push_back(u + 1);
            emit_split_run(runB, "B");
        } else {
            for (uint32_t u : run) emit_plain(u + 1);
        }
        // (triangles of the run's span that slot A omitted are omitted for B too)
        i = run.back() / 2 + 1;
    }
}

}  // namespace

// Grain and magnitude alone (Val without the expression text): the same zero-dropping rules as
// Gen::mul / Gen::fma / Gen::cross / Gen::dot -- the keys and names only serve the generator's
// common subexpressions and never change a bound -- so the scene rule costs a few integer
// operations per triangle instead of building each test's strings (100k triangles
// took 0.3 s of upload that way).
namespace {
struct GrainMag {
    bool zero = true;
    int grain = kNoGrain;
    int mag = kNoMag;
};
GrainMag gm_lit(float x)           // lit_or_zero's grain and magnitude, without its key text
{
    if (x == 0.0f) return {};
    int e = 0;
    (void)std::frexp(std::fabs(x), &e);            // |x| < 2^e
    return {false, grain_of(x), e};
}
GrainMag gm_mul(const GrainMag &a, const GrainMag &b)
{
    if (a.zero || b.zero) return {};
    return {false, grain_mul(a.grain, b.grain), mag_mul(a.mag, b.mag)};
}
GrainMag gm_fma(const GrainMag &a, const GrainMag &b, const GrainMag &c)
{
    if (a.zero || b.zero) return c;
    if (c.zero) return gm_mul(a, b);
    return {false, grain_min(grain_mul(a.grain, b.grain), c.grain),
            mag_sum(mag_mul(a.mag, b.mag), c.mag)};
}
}  // namespace

bool scan_rcp_fast_scene(const TriRecord *tri, uint32_t n)
{
    // the generic test's den = dot(cross(d, e2), e1) equals the zero-dropped expression's value
    // (a product with a zero factor is an exact zero, an fma with one adds nothing) as long as
    // nothing overflows, so its grain and magnitude bounds (Val) hold for it: ask that s1 and den
    // stay within 2^126 (no overflow, so no inf x 0 either) and that a non-zero den is at least
    // 2^-126, for every ray passing dir_fast_ok
    const GrainMag d{false, kDirGrain, kDirMag};     // every direction component (dir_grain_ok)
    for (uint32_t i = 0; i < n; i++) {
        GrainMag e1[3], e2[3], s1[3];
        for (int k = 0; k < 3; k++) {
            if (!std::isfinite(tri[i].e1[k]) || !std::isfinite(tri[i].e2[k])) return false;
            e1[k] = gm_lit(tri[i].e1[k]);
            e2[k] = gm_lit(tri[i].e2[k]);
        }
        // cross_i = fma(a_j, b_k, -(a_k * b_j)) with a = d (Gen::cross)
        s1[0] = gm_fma(d, e2[2], gm_mul(d, e2[1]));
        s1[1] = gm_fma(d, e2[0], gm_mul(d, e2[2]));
        s1[2] = gm_fma(d, e2[1], gm_mul(d, e2[0]));
        for (int k = 0; k < 3; k++)
            if (!s1[k].zero && s1[k].mag > 126) return false;
        // dot = fma(z, z', fma(y, y', x * x')) (Gen::dot)
        const GrainMag den = gm_fma(s1[2], e1[2], gm_fma(s1[1], e1[1], gm_mul(s1[0], e1[0])));
        if (den.zero) continue;                      // identically zero: f = NaN, rejected
        if (den.grain == kNoGrain || den.grain < -126 || den.mag > 126) return false;
    }
    return true;
}

// The string-building form the rule was first written in (Gen over Val), kept as the CPU tests'
// second opinion on scan_rcp_fast_scene (rvcp_internal_scan_rcp_fast_scene_ref).
bool scan_rcp_fast_scene_ref(const TriRecord *tri, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++) {
        Gen g;
        Val d[3] = {var("d.x", kDirGrain, kDirMag), var("d.y", kDirGrain, kDirMag),
                    var("d.z", kDirGrain, kDirMag)};
        Val e1[3], e2[3], s1[3];
        for (int k = 0; k < 3; k++) {
            if (!std::isfinite(tri[i].e1[k]) || !std::isfinite(tri[i].e2[k])) return false;
            e1[k] = lit_or_zero(tri[i].e1[k]);
            e2[k] = lit_or_zero(tri[i].e2[k]);
        }
        g.cross(d, e2, s1);
        for (int k = 0; k < 3; k++)
            if (s1[k].kind != Val::kZero && s1[k].mag > 126) return false;
        const Val den = g.dot(s1, e1);
        if (den.kind == Val::kZero) continue;
        if (den.grain == kNoGrain || den.grain < -126 || den.mag > 126) return false;
    }
    return true;
}

bool jit_scene_in_range(const TriRecord *tri, uint32_t n)
{
    // the premise of the zero-dropping (header): with |v0| <= 2^40, |e1|, |e2| <= 2^41 and the
    // kernel's per-wave ray check (|o|_1 <= 2^41, |d|_1 <= 16) no intermediate overflows
    for (uint32_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++)
            if (!(std::fabs(tri[i].v0[k]) <= 0x1p40f) || !(std::fabs(tri[i].e1[k]) <= 0x1p41f) ||
                !(std::fabs(tri[i].e2[k]) <= 0x1p41f))
                return false;
    return true;
}

std::string jit_scan_source(const TriRecord *tri, uint32_t n, unsigned opts)
{
    // RVCP_F32(bits): the triangle's float by its bit pattern; RVCP_SPEC_COMMIT(t, i): the
    // test's result is final here (on the GPU an empty asm on the two registers plus a
    // scheduling barrier, so the unrolled scan stays one test deep in registers; the CPU
    // check in tests/test_jit_cpu.py compiles the same text with plain C definitions)
    std::string out = "// generated by rvcp_jit.cpp: the scan of DESIGN.md §4.7 over " +
                      std::to_string(n) + " triangles\n";
    out += "__device__ __forceinline__ void spec_scan1(f3 o, f3 d, float tmin, float &bt, "
           "int &best) {\n";
    static const char *const one[] = {""}, *const two[] = {"A", "B"};
    emit_scan(out, tri, n, one, 1);
    out += "}\n";
    out += "__device__ __forceinline__ void spec_scan2(f3 oA, f3 dA, f3 oB, f3 dB, float tmin, "
           "float &btA, float &btB, int &bestB) {\n";
    emit_scan(out, tri, n, two, 2, opts);
    out += "}\n";
    return out;
}

// Mode 2's spheres (RVCP_JIT_LEGACY modules): the uploaded records as an X-macro over
// (index, center x, y, z, radius) with the floats as bit patterns, which legacy_spheres expands
// into its unrolled sphere tests (rvcp_kernels.hip).  Empty for no spheres or more than
// kJitMaxSpheres (the kernel then keeps its loop over the records).
std::string jit_sphere_source(const rvcp_sphere_t *sph, uint32_t n)
{
    if (n == 0 || n > kJitMaxSpheres || !sph) return std::string();
    std::string out = "// the scene's " + std::to_string(n) + " spheres (rvcp_jit.cpp jit_sphere_source)\n"
                      "#define RVCP_SPEC_SPHERES(X)";
    for (uint32_t i = 0; i < n; i++) {
        out += " \\\n    X(" + std::to_string(i);
        for (float v : {sph[i].center[0], sph[i].center[1], sph[i].center[2], sph[i].radius})
            out += ", " + lit_text(v);
        out += ")";
    }
    return out + "\n";
}

// Mode 2 with the scene in LDS (RVCP_LEGACY_LDS_SCENE): the LDS copies sized to the scene
// (every one at least 1 entry) and the cached primary hit in LDS columns
// (RVCP_LEGACY_LDS_PRIMARY, rvcp_kernels.hip legacy_body) -- the block's LDS then stays small
// enough for the resident blocks its registers allow.
std::string jit_legacy_lds_source(uint32_t n_faces, uint32_t n_spheres, uint32_t n_materials)
{
    auto at_least_1 = [](uint32_t v) { return std::to_string(v ? v : 1u); };
    std::string out = "#define RVCP_LDS_FACES " + at_least_1(n_faces) + "\n#define RVCP_LDS_SPHERES " +
                      at_least_1(n_spheres) + "\n#define RVCP_LDS_MATS " + at_least_1(n_materials) + "\n";
#ifndef RVCP_NO_LDS_PRIMARY         // (A/B variant only, tools/build_variant.sh)
    out += "#define RVCP_LEGACY_LDS_PRIMARY 1\n";
#endif
    return out;
}

// ------------------------------------------------------------------ compile + cache -----
namespace {

}  // namespace

// Extra hipRTC options: only the debug build of the library (-DRVCP_DEBUG_KNOBS, tools/) reads
// them, from RVCP_JIT_FLAGS (separated by spaces or commas).  Options that would change the
// numeric contract (contraction, fast math) are refused; the options are part of the module
// cache key (jit_path_kernels), so changing them within a process recompiles.
std::vector<std::string> jit_extra_flags()
{
    std::vector<std::string> extra;
#ifdef RVCP_DEBUG_KNOBS
    if (const char *e = std::getenv("RVCP_JIT_FLAGS")) {
        std::string cur;
        for (const char *c = e;; c++) {
            if (*c == ' ' || *c == ',' || *c == '\0') {
                if (!cur.empty()) {
                    if (cur.find("fp-contract") == std::string::npos &&
                        cur.find("fast-math") == std::string::npos &&
                        cur.find("ffast") == std::string::npos &&
                        cur.find("unsafe") == std::string::npos)
                        extra.push_back(cur);
                    else
                        std::fprintf(stderr, "rvcp: ignoring JIT option %s (numeric contract)\n", cur.c_str());
                }
                cur.clear();
                if (!*c) break;
            } else {
                cur += *c;
            }
        }
    }
#endif
    return extra;
}

// Experiment knobs (debug build only, like jit_extra_flags): split the dual scan's path slot B
// into skippable runs as well (RVCP_DEBUG_SPEC_SKIP_B=1); compute the shadow slot's s1 and s2
// whole before its split, as round 5's first form did (RVCP_DEBUG_SPEC_EAGER=1).
unsigned jit_scan_opts()
{
    unsigned opts = 0;
#ifdef RVCP_DEBUG_KNOBS
    const char *e = std::getenv("RVCP_DEBUG_SPEC_SKIP_B");
    if (e && *e == '1') opts |= kScanSkipB;
    e = std::getenv("RVCP_DEBUG_SPEC_EAGER");
    if (e && *e == '1') opts |= kScanEagerSplit;
#endif
    return opts;
}

std::vector<std::string> jit_options(bool legacy, int legacy_waves, bool lds_scene, bool bvh);

namespace {

uint64_t fnv1a(const std::string &s)
{
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

struct CacheEntry {
    int device;
    uint64_t hash;
    std::string scan;
    std::shared_ptr<JitKernels> kernels;
};
std::mutex g_mu;
std::list<CacheEntry> g_cache;            // most recently used first
constexpr size_t kCacheEntries = 16;

// ---- on-disk code-object cache (rvcp_set_code_cache_dir) ----
// One file per module, <fnv1a(key) in hex>.rvcpco:
//   "RVCPCO01" | u64 key bytes | u64 code bytes | u64 fnv1a(code) | u64 fnv1a(key) | key | code
// The key is the whole input of the compile: the hipRTC version, the options, the hash and
// length of every embedded source (kernels, headers) and the generated scan text itself, so an
// entry is used only for exactly the module it was compiled as; a file whose header, lengths,
// key or code checksum disagree -- or whose code the runtime refuses -- is rejected, recompiled
// and rewritten.  Writes go to a temporary file renamed into place (readers never see half a
// file; concurrent writers of one key write the same bytes).
constexpr char kCoMagic[8] = {'R', 'V', 'C', 'P', 'C', 'O', '0', '1'};
std::string g_cache_dir;                  // "" = disk cache off
bool g_cache_dir_set = false;             // rvcp_set_code_cache_dir was called
std::atomic<uint64_t> g_disk_loads{0}, g_disk_compiles{0}, g_disk_rejects{0};

std::string default_cache_dir()
{
    const char *x = std::getenv("XDG_CACHE_HOME");
    if (x && *x == '/') return std::string(x) + "/rvcp-mi355x";
    const char *h = std::getenv("HOME");
    if (h && *h == '/') return std::string(h) + "/.cache/rvcp-mi355x";
    return std::string();
}

std::string cache_dir()          // with g_mu held
{
    if (!g_cache_dir_set) {
        g_cache_dir = default_cache_dir();
        g_cache_dir_set = true;
    }
    return g_cache_dir;
}

bool make_dirs(const std::string &dir)
{
    if (dir.empty()) return false;
    for (size_t i = 1; i <= dir.size(); i++) {
        if (i == dir.size() || dir[i] == '/') {
            const std::string p = dir.substr(0, i);
            if (::mkdir(p.c_str(), 0700) != 0 && errno != EEXIST) return false;
        }
    }
    struct stat st;
    return ::stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::string code_key(const std::string &scan, const std::vector<std::string> &opts)
{
    int maj = -1, mnr = -1;
    if (rtc().version) (void)rtc().version(&maj, &mnr);
    std::string k = "rvcp code object\nhiprtc " + std::to_string(maj) + "." + std::to_string(mnr) + "\n";
    for (const std::string &o : opts) k += o + "\n";
    for (const char *src : {kJitSrcKernels, kJitSrcInternal, kJitSrcAbi, kJitSrcSqrt}) {
        const std::string s(src);
        k += "src " + std::to_string(s.size()) + " " + std::to_string(fnv1a(s)) + "\n";
    }
    return k + scan;
}

std::string hex64(uint64_t v)
{
    char b[17];
    std::snprintf(b, sizeof(b), "%016llx", (unsigned long long)v);
    return b;
}

uint64_t fnv1a_bytes(const char *p, size_t n)
{
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; i++) {
        h ^= (unsigned char)p[i];
        h *= 1099511628211ull;
    }
    return h;
}

// The entry for `key` in `dir`: 1 = code read and verified, 0 = no entry, -1 = entry rejected
int disk_read(const std::string &dir, const std::string &key, std::vector<char> &code)
{
    const std::string path = dir + "/" + hex64(fnv1a(key)) + ".rvcpco";
    std::FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return 0;
    std::vector<char> buf;
    char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    std::fclose(f);
    uint64_t hdr[4];
    if (buf.size() < 8 + sizeof(hdr) || std::memcmp(buf.data(), kCoMagic, 8) != 0) return -1;
    std::memcpy(hdr, buf.data() + 8, sizeof(hdr));
    const size_t off = 8 + sizeof(hdr);
    // (the lengths are compared without forming off + hdr[0] + hdr[1], which a damaged or
    // crafted header could wrap past 2^64 onto the file size)
    if (hdr[0] != key.size() || hdr[1] == 0 || buf.size() - off < hdr[0] ||
        buf.size() - off - hdr[0] != hdr[1] ||
        hdr[3] != fnv1a(key) || std::memcmp(buf.data() + off, key.data(), key.size()) != 0)
        return -1;
    const char *c = buf.data() + off + hdr[0];
    if (fnv1a_bytes(c, hdr[1]) != hdr[2] || hdr[1] < 4 || std::memcmp(c, "\x7f" "ELF", 4) != 0)
        return -1;
    code.assign(c, c + hdr[1]);
    return 1;
}

void disk_write(const std::string &dir, const std::string &key, const std::vector<char> &code)
{
    if (!make_dirs(dir)) return;
    static std::atomic<unsigned> seq{0};
    const std::string path = dir + "/" + hex64(fnv1a(key)) + ".rvcpco";
    const std::string tmp = path + ".tmp." + std::to_string((long)::getpid()) + "." + std::to_string(seq++);
    std::FILE *f = std::fopen(tmp.c_str(), "wb");
    if (!f) return;
    const uint64_t hdr[4] = {key.size(), code.size(), fnv1a_bytes(code.data(), code.size()), fnv1a(key)};
    bool ok = std::fwrite(kCoMagic, 1, 8, f) == 8 && std::fwrite(hdr, 1, sizeof(hdr), f) == sizeof(hdr) &&
              std::fwrite(key.data(), 1, key.size(), f) == key.size() &&
              std::fwrite(code.data(), 1, code.size(), f) == code.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());
}

}  // namespace

// The module's code object: from the disk cache when it holds a verified entry for exactly this
// compile (from_disk = true), else compiled with hipRTC and stored.  force_compile: the caller
// found the disk entry unusable (the runtime refused it) -- count it rejected, compile, overwrite.
// With g_mu held.
int jit_cached_code(const std::string &scan, std::vector<char> &code, std::string &err,
                    bool legacy, int legacy_waves, bool lds_scene, bool bvh, bool *from_disk,
                    bool force_compile)
{
    *from_disk = false;
    const std::string dir = cache_dir();
    std::string key;
    if (!dir.empty()) {
        key = code_key(scan, jit_options(legacy, legacy_waves, lds_scene, bvh));
        if (force_compile) {
            g_disk_rejects++;
        } else {
            const int r = disk_read(dir, key, code);
            if (r == 1) {
                g_disk_loads++;
                *from_disk = true;
                return 0;
            }
            if (r < 0) g_disk_rejects++;
        }
    }
    if (jit_compile_code(scan, code, err, legacy, legacy_waves, lds_scene, bvh) != 0) return -1;
    g_disk_compiles++;
    if (!dir.empty()) disk_write(dir, key, code);
    return 0;
}

JitKernels::~JitKernels()
{
    if (module) {
        int cur = -1;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        (void)hipModuleUnload(module);
        if (cur >= 0) (void)hipSetDevice(cur);
    }
}

// The hipRTC options of a module: the flags of the static build (Makefile), on which the
// numeric contract depends, and the module's variant defines.
std::vector<std::string> jit_options(bool legacy, int legacy_waves, bool lds_scene, bool bvh)
{
    std::vector<std::string> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17",
                                     "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
                                     "-fno-fast-math", "-fno-slp-vectorize", "-DRVCP_JIT",
                                     "-DRVCP_SPEC_SCAN=\"rvcp_spec_scan.inc\""};
    if (legacy) opts.push_back("-DRVCP_JIT_LEGACY");
    if (bvh) opts.push_back("-DRVCP_JIT_BVH");
#ifdef RVCP_TIMELINE
    opts.push_back("-DRVCP_TIMELINE");      // the debug library's modules keep the per-wave timeline
#endif
    if (legacy && legacy_waves > 0) opts.push_back("-DRVCP_LEGACY_MIN_WAVES=" + std::to_string(legacy_waves));
    if (legacy && lds_scene) opts.push_back("-DRVCP_LEGACY_LDS_SCENE");
    for (const std::string &x : jit_extra_flags()) opts.push_back(x);
    return opts;
}

int jit_compile_code(const std::string &scan, std::vector<char> &code, std::string &err,
                     bool legacy, int legacy_waves, bool lds_scene, bool bvh)
{
    const RtcApi &api = rtc();
    if (!api.ok) {
        err = api.why;
        return -1;
    }
    const char *hdr_src[] = {kJitSrcInternal, kJitSrcAbi, kJitSrcSqrt, scan.c_str()};
    const char *hdr_name[] = {"rvcp_internal.h", "../../include/rvcp.h", "rvcp_sqrt.h", "rvcp_spec_scan.inc"};
    rtc_program prog = nullptr;
    if (api.create(&prog, kJitSrcKernels, "rvcp_kernels.hip", 4, hdr_src, hdr_name) != 0) {
        err = "hiprtcCreateProgram failed";
        return -1;
    }
    const std::vector<std::string> opt_s = jit_options(legacy, legacy_waves, lds_scene, bvh);
    std::vector<const char *> opts;
    for (const std::string &x : opt_s) opts.push_back(x.c_str());
    const int rc = api.compile(prog, (int)opts.size(), opts.data());
    if (rc != 0) {
        size_t ls = 0;
        api.log_size(prog, &ls);
        std::string log(ls, '\0');
        if (ls) api.log(prog, &log[0]);
        err = "hipRTC compile failed: " + log.substr(0, 4000);
        api.destroy(&prog);
        return -1;
    }
    size_t cs = 0;
    api.code_size(prog, &cs);
    code.assign(cs, 0);
    if (cs) api.code(prog, code.data());
    api.destroy(&prog);
    return cs ? 0 : -1;
}

std::shared_ptr<JitKernels> jit_path_kernels(int device, const TriRecord *tri, uint32_t n,
                                             std::string &err, bool legacy, bool sphereless,
                                             bool lds_fits, bool bvh, const rvcp_sphere_t *spheres,
                                             uint32_t n_spheres, uint32_t n_materials)
{
    // Mode 2 on a scene without spheres (the Cornell frame): 6 waves per SIMD measured 2.5 %
    // faster than 5, with spheres 5 % slower (profiles/history/r02_legacy_waves_ab.log).  With the
    // scene in LDS (lds_fits): the sphere room 0.288 -> 0.278 ms at 5 waves (4 and 6: 0.305,
    // 0.308; 5 waves without LDS 0.290), the Cornell frame 1.867 -> 1.831 ms at 6
    // (profiles/history/r04d_ab_m2.log, r04e_ab_m2b.log).
    // (debug build: RVCP_JIT_LEGACY_WAVES overrides; 0 = the compiler's choice)
    const bool lds_scene = legacy && lds_fits;
#ifndef RVCP_SPHERELESS_LEGACY_WAVES   // (A/B variants only, tools/build_variant.sh)
#define RVCP_SPHERELESS_LEGACY_WAVES 6
#endif
    int legacy_waves = legacy && sphereless ? RVCP_SPHERELESS_LEGACY_WAVES : lds_scene ? 5 : 0;
#ifdef RVCP_DEBUG_KNOBS
    if (const char *e = std::getenv("RVCP_JIT_LEGACY_WAVES")) legacy_waves = std::atoi(e);
#endif
    std::string key_flags;
    for (const std::string &x : jit_extra_flags()) key_flags += " " + x;
    const std::string scan = jit_scan_source(tri, n, jit_scan_opts()) +
        (legacy ? "// +legacy " + std::to_string(legacy_waves) + (lds_scene ? " lds" : "") + "\n"
#ifndef RVCP_NO_SPHERE_LITERALS     // (A/B variant only, tools/build_variant.sh)
                      + jit_sphere_source(spheres, n_spheres)
#endif
                      + (lds_scene ? jit_legacy_lds_source(n, n_spheres, n_materials) : std::string())
                : std::string()) +
        (key_flags.empty() ? std::string() : "// +flags" + key_flags + "\n") +
        (bvh ? "// +bvh\n" : "");
    const uint64_t h = fnv1a(scan);
    std::lock_guard<std::mutex> lock(g_mu);
    for (auto it = g_cache.begin(); it != g_cache.end(); ++it) {
        if (it->device == device && it->hash == h && it->scan == scan) {
            g_cache.splice(g_cache.begin(), g_cache, it);
            return g_cache.front().kernels;
        }
    }
    if (hipSetDevice(device) != hipSuccess) {
        err = "hipSetDevice failed";
        return nullptr;
    }
    // the module's kernels from its code object; "" or what is missing
    auto load = [&](JitKernels &k, const std::vector<char> &code) -> std::string {
        if (hipModuleLoadData(&k.module, code.data()) != hipSuccess) {
            k.module = nullptr;
            return "hipModuleLoadData failed";
        }
        if (hipModuleGetFunction(&k.path5, k.module, "rvcp_spec_path_kernel5") != hipSuccess ||
            hipModuleGetFunction(&k.path6, k.module, "rvcp_spec_path_kernel6") != hipSuccess)
            return "specialised kernels missing from the module";
        if (hipModuleGetFunction(&k.primary, k.module, "rvcp_spec_primary_kernel") != hipSuccess)
            return "specialised pre-pass kernel missing from the module";
        if (bvh && (hipModuleGetFunction(&k.bvh_path, k.module, "rvcp_spec_bvh_path_kernel") != hipSuccess ||
                    hipModuleGetFunction(&k.bvh_primary, k.module, "rvcp_spec_bvh_primary_kernel") != hipSuccess))
            return "specialised BVH kernels missing from the module";
        if (legacy && hipModuleGetFunction(&k.legacy, k.module, "rvcp_spec_legacy_kernel") != hipSuccess)
            return "specialised mode-2 kernel missing from the module";
        return std::string();
    };
    std::vector<char> code;
    bool from_disk = false;
    if (jit_cached_code(scan, code, err, legacy, legacy_waves, lds_scene, bvh, &from_disk, false) != 0)
        return nullptr;
    const uint64_t key_hash = fnv1a(code_key(scan, jit_options(legacy, legacy_waves, lds_scene, bvh)));
    auto k = std::make_shared<JitKernels>();
    k->device = device;
    k->key_hash = key_hash;
    std::string why = load(*k, code);
    if (!why.empty() && from_disk) {
        // a verified entry the runtime still refuses (another ROCm, another device): not
        // trusted -- compiled afresh and the entry overwritten
        k = std::make_shared<JitKernels>();
        k->device = device;
        k->key_hash = key_hash;
        if (jit_cached_code(scan, code, err, legacy, legacy_waves, lds_scene, bvh, &from_disk, true) != 0)
            return nullptr;
        why = load(*k, code);
    }
    if (!why.empty()) {
        err = why;
        return nullptr;
    }
    int bpc = 0;
    if (legacy && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k->legacy, kBlock, 0) == hipSuccess)
        k->blocks_per_cu_legacy = bpc;
    if (bvh && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k->bvh_path, kBlock, 0) == hipSuccess)
        k->blocks_per_cu_bvh = bpc;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k->path5, kBlock, 0) == hipSuccess)
        k->blocks_per_cu5 = bpc;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k->path6, kBlock, 0) == hipSuccess)
        k->blocks_per_cu6 = bpc;
    g_cache.push_front(CacheEntry{device, h, scan, k});
    if (g_cache.size() > kCacheEntries) g_cache.pop_back();
    return k;
}

}  // namespace rvcp

// Self-test hook: may the generic scans of a scene with these n triangle records take 1/den
// without the class check (scan_rcp_fast_scene; 1 / 0)?
extern "C" int rvcp_internal_scan_rcp_fast_scene(const void *tri_records, uint32_t n)
{
    return rvcp::scan_rcp_fast_scene(static_cast<const rvcp::TriRecord *>(tri_records), n) ? 1 : 0;
}

extern "C" int rvcp_internal_scan_rcp_fast_scene_ref(const void *tri_records, uint32_t n)
{
    return rvcp::scan_rcp_fast_scene_ref(static_cast<const rvcp::TriRecord *>(tri_records), n) ? 1 : 0;
}

// Self-test hook: would upload specialise a scene with these n triangle records (1 / 0)?
extern "C" int rvcp_internal_jit_scene_in_range(const void *tri_records, uint32_t n)
{
    return rvcp::jit_scene_in_range(static_cast<const rvcp::TriRecord *>(tri_records), n) ? 1 : 0;
}

// Self-test hooks for the CPU test suite (not part of rvcp.h): generate and compile the
// specialised module for n triangle records without a GPU (`legacy`: with the mode-2 kernel).
// Returns 0 and the code-object size, or -1 with the message in err (err_cap bytes).
// (with n_spheres sphere records: a mode-2 module with the spheres as literals, as upload
// builds it for a scene with spheres -- rvcp_internal_jit_compile_check_spheres)
static int jit_compile_check(const void *tri_records, uint32_t n, int legacy, const void *spheres,
                             uint32_t n_spheres, size_t *code_bytes, char *err, size_t err_cap)
{
    try {
        std::string e;
        std::vector<char> code;
        std::string scan = rvcp::jit_scan_source(static_cast<const rvcp::TriRecord *>(tri_records), n);
        if (legacy) scan += rvcp::jit_sphere_source(static_cast<const rvcp_sphere_t *>(spheres), n_spheres);
        const int rc = rvcp::jit_compile_code(scan, code, e, legacy != 0);
        if (code_bytes) *code_bytes = code.size();
        if (err && err_cap) {
            std::strncpy(err, e.c_str(), err_cap - 1);
            err[err_cap - 1] = '\0';
        }
        return rc;
    } catch (...) {
        return -1;
    }
}

extern "C" int rvcp_internal_jit_compile_check_mode(const void *tri_records, uint32_t n,
                                                     int legacy, size_t *code_bytes, char *err,
                                                     size_t err_cap)
{
    return jit_compile_check(tri_records, n, legacy, nullptr, 0, code_bytes, err, err_cap);
}

extern "C" int rvcp_internal_jit_compile_check_spheres(const void *tri_records, uint32_t n,
                                                        const void *spheres, uint32_t n_spheres,
                                                        size_t *code_bytes, char *err,
                                                        size_t err_cap)
{
    return jit_compile_check(tri_records, n, 1, spheres, n_spheres, code_bytes, err, err_cap);
}

extern "C" int rvcp_internal_jit_compile_check(const void *tri_records, uint32_t n,
                                                size_t *code_bytes, char *err, size_t err_cap)
{
    return rvcp_internal_jit_compile_check_mode(tri_records, n, 0, code_bytes, err, err_cap);
}

// The generated scan source for n triangle records (for inspection): writes at most cap bytes
// including the terminator and returns the full length.
extern "C" size_t rvcp_internal_jit_scan_source_opt(const void *tri_records, uint32_t n,
                                                    int opts, char *out, size_t cap)
{
    try {
        const std::string s = rvcp::jit_scan_source(
            static_cast<const rvcp::TriRecord *>(tri_records), n, (unsigned)opts);
        if (out && cap) {
            std::strncpy(out, s.c_str(), cap - 1);
            out[cap - 1] = '\0';
        }
        return s.size();
    } catch (...) {
        return 0;
    }
}

// Self-test hook: the sphere X-macro of a mode-2 module for n sphere records (rvcp_sphere_t);
// the length without the terminator, written into out when it fits cap bytes.
extern "C" size_t rvcp_internal_jit_sphere_source(const void *spheres, uint32_t n, char *out,
                                                   size_t cap)
{
    try {
        const std::string s = rvcp::jit_sphere_source(static_cast<const rvcp_sphere_t *>(spheres), n);
        if (out && cap > s.size()) std::memcpy(out, s.c_str(), s.size() + 1);
        return s.size();
    } catch (...) {
        return 0;
    }
}

extern "C" size_t rvcp_internal_jit_scan_source(const void *tri_records, uint32_t n, char *out,
                                                size_t cap)
{
    return rvcp_internal_jit_scan_source_opt(tri_records, n, 0, out, cap);
}

// ---- the on-disk code-object cache's C-ABI (rvcp.h) ----
extern "C" int rvcp_set_code_cache_dir(const char *dir)
{
    try {
        std::lock_guard<std::mutex> lock(rvcp::g_mu);
        rvcp::g_cache_dir = dir ? std::string(dir) : std::string();
        while (rvcp::g_cache_dir.size() > 1 && rvcp::g_cache_dir.back() == '/') rvcp::g_cache_dir.pop_back();
        rvcp::g_cache_dir_set = true;
        return 0;
    } catch (...) {
        return -5;      // RVCP_E_NOMEM: the only thing that can throw here
    }
}

extern "C" int rvcp_code_cache_counts(uint64_t out[3])
{
    if (!out) return -1;
    out[0] = rvcp::g_disk_loads.load();
    out[1] = rvcp::g_disk_compiles.load();
    out[2] = rvcp::g_disk_rejects.load();
    return 0;
}

// Self-test hook for the CPU suite (not part of rvcp.h): the specialised module's code object
// for n triangle records through the on-disk cache, without a GPU (no module load).  Returns 0
// with *from_disk and *code_bytes, or -1 with the message in err.
extern "C" int rvcp_internal_jit_cached_code(const void *tri_records, uint32_t n, int legacy,
                                             int *from_disk, size_t *code_bytes, char *err,
                                             size_t err_cap)
{
    try {
        std::string e;
        std::vector<char> code;
        const std::string scan =
            rvcp::jit_scan_source(static_cast<const rvcp::TriRecord *>(tri_records), n);
        bool disk = false;
        int rc;
        {
            std::lock_guard<std::mutex> lock(rvcp::g_mu);
            rc = rvcp::jit_cached_code(scan, code, e, legacy != 0, 0, false, false, &disk, false);
        }
        if (from_disk) *from_disk = disk ? 1 : 0;
        if (code_bytes) *code_bytes = code.size();
        if (err && err_cap) {
            std::strncpy(err, e.c_str(), err_cap - 1);
            err[err_cap - 1] = '\0';
        }
        return rc;
    } catch (...) {
        return -1;
    }
}
