/*
 * rvcp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, scalar CPU restatement of the path-tracing kernel that the reference's
 * `src/ray_tracer` dispatches: /root/reference/assets/shaders/ray_tracer_games101_branch.comp
 * (selected by src/ray_tracer/shader.rs:12).  It exists to check the HIP kernel and to time
 * the CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product (librvcp.so) never links, calls or falls back to it.
 *
 * It is written independently of the HIP kernel: it follows the GLSL function by function
 * (each function cites the shader line it restates) and shares with the kernel only the
 * numeric contract of DESIGN.md §3 (float32 everywhere, no implicit contraction, the
 * builtins dot and cross as explicit fma chains, IEEE
 * correctly-rounded + - * / sqrt, the software sin below, the gamma threshold table).
 *
 * Parity pinning: the reference ships no tests and no golden vectors.  The
 * only reference-produced output is the README screenshot (1024^2, SPP=30); this oracle is
 * pinned against its block means by tests/test_oracle_reference.py (fixture made by
 * tests/golden/make_readme_fixture.py).  Per-pixel parity with the NVIDIA/Vulkan original is
 * impossible because its sin() is driver-defined; the oracle therefore
 * pins the algorithm statistically and the HIP kernel bit-exactly against this file.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rvcp.h"

#if defined(__FP_FAST_FMA) || defined(__FAST_MATH__)
#if defined(__FAST_MATH__)
#error "the oracle must not be built with -ffast-math"
#endif
#endif

/* ------------------------------------------------------------------------------------- */
/* Constants: ray_tracer_games101_branch.comp:5-25                                         */
/* ------------------------------------------------------------------------------------- */
#define PI_F 3.1415926f          /* :6 (not M_PI) */
#define MATERIAL_LIGHT 3u        /* :25 */

typedef struct {
    uint32_t spp, max_bounces;
    float att_stop, t_min, t_max, rr, eps;
    int quirk;
    int integrator;          /* 0 = games101 (dispatched), 1 = ray_tracer.comp ray_trace */
    int unorm_rule;          /* rvcp_config_t.unorm_rule */
} params_t;

/* ------------------------------------------------------------------------------------- */
/* vec3 algebra with GLSL semantics, evaluated left to right, no contraction              */
/* ------------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
/* The builtins dot and cross are fused chains: GLSL leaves their internal
 * rounding to the implementation; arithmetic the shader writes out stays unfused. */
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross(v3 a, v3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)),
              fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float length(v3 a) { return sqrtf(dot(a, a)); }
/* GLSL normalize(v) restated as v * (1 / sqrt(dot(v, v))). */
static inline v3 normalize(v3 a) { return muls(a, 1.0f / sqrtf(dot(a, a))); }
static inline float fractf(float x) { return x - floorf(x); }     /* GLSL fract */
static inline v3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }

/* ------------------------------------------------------------------------------------- */
/* Software sin: q = rint(x / pi), Cody-Waite reduction by pi with fma,   */
/* one odd minimax polynomial on [-pi/2, pi/2], sign flipped for odd q.  Bit-identical     */
/* wherever fmaf/rintf/floorf are IEEE.                                                    */
/* ------------------------------------------------------------------------------------- */
float rvcp_oracle_sinf(float x)
{
    if (!(fabsf(x) < 1.0e30f)) return x - x;            /* NaN for inf/NaN */
    const float q = rintf(x * 0x1.45f306p-2f);          /* nearest multiple of pi */
    float r = fmaf(q, -0x1.921fb6p+1f, x);              /* x - q*float(pi) */
    r = fmaf(q, 0x1.777a5cp-24f, r);                    /* - q*(pi - float(pi)) */
    const float z = r * r;
    const float p = fmaf(fmaf(fmaf(0x1.5dbdfep-19f, z, -0x1.9f7p-13f), z, 0x1.110ed4p-7f), z,
                         -0x1.55554cp-3f);
    const float s = fmaf(p, z * r, r);
    const float odd = q - 2.0f * floorf(q * 0.5f);      /* q mod 2, exact */
    return odd != 0.0f ? -s : s;
}

/* ------------------------------------------------------------------------------------- */
/* RNG: ray_tracer_games101_branch.comp:151-168                                            */
/* ------------------------------------------------------------------------------------- */
typedef struct { float seed, index; } rng_t;

/* srand, :153-155 */
static inline void srand_glsl(rng_t *g, float time, float u, float v)
{
    float a = fractf(rvcp_oracle_sinf(time) * 43758.5453f);
    float b = fractf(rvcp_oracle_sinf(u) * 22578.5453f);
    float c = fractf(rvcp_oracle_sinf(v) * 114514.1919f);
    g->seed = fractf(a + b + c);
    g->index = 0.0f;     /* :152 global initialiser; one invocation per pixel */
}
/* _rand, :156-158 */
static inline float rand_of(float x) { return fractf(rvcp_oracle_sinf(x) * 43758.5453f); }
/* rand, :159-162 */
static inline float rand_next(rng_t *g)
{
    g->index = g->index + 1.0f;
    return rand_of(g->seed + g->index);
}

/* random_in_unit_sphere, :195-201 (rand3 evaluates x, y, z in order, :166-168) */
static v3 random_in_unit_sphere(rng_t *g)
{
    v3 p;
    do {
        float rx = rand_next(g), ry = rand_next(g), rz = rand_next(g);
        p = mk(2.0f * rx - 1.0f, 2.0f * ry - 1.0f, 2.0f * rz - 1.0f);
    } while (dot(p, p) >= 1.0f);
    return p;
}
/* random_in_unit_hemisphere(_surface), :207-214 */
static v3 random_in_unit_hemisphere_surface(rng_t *g, v3 n)
{
    v3 p = random_in_unit_sphere(g);
    v3 h = dot(p, n) > 0.0f ? p : neg(p);
    return normalize(h);
}

/* ------------------------------------------------------------------------------------- */
/* Scene view                                                                              */
/* ------------------------------------------------------------------------------------- */
typedef struct {
    const rvcp_material_t *mat; uint32_t n_mat;
    const rvcp_vertex_t *vtx; uint32_t n_vtx;
    const rvcp_face_t *face; uint32_t n_face;
    const uint32_t *lum; uint32_t n_lum;   /* packed u32 ids as uploaded */
    const rvcp_sphere_t *sph; uint32_t n_sph;   /* integrator mode 2 only */
} scene_t;

typedef struct { v3 o, d; float t_min, t_max; } ray_t;        /* :116-121 */
typedef struct {                                                /* :123-133 */
    float time; v3 pos, normal; uint32_t material_id; int outward;
} hit_t;

/* Luminous face id i as the shader reads it (:109-111). */
static inline uint32_t lum_face_id(const scene_t *s, uint32_t i, int quirk)
{
    if (!quirk) return s->lum[i];
    return (4u * i < s->n_lum) ? s->lum[4u * i] : 0u;
}

/* is_intersect_with_face, :238-280 */
static int is_intersect_with_face(const scene_t *sc, const ray_t *ray, const rvcp_face_t *f,
                                  hit_t *out)
{
    v3 v0 = ld3(sc->vtx[f->vertices[0]].position);
    v3 v1 = ld3(sc->vtx[f->vertices[1]].position);
    v3 v2 = ld3(sc->vtx[f->vertices[2]].position);
    v3 e1 = sub(v1, v0), e2 = sub(v2, v0), s = sub(ray->o, v0);
    v3 s1 = cross(ray->d, e2), s2 = cross(s, e1);
    float f_ = 1.0f / dot(s1, e1);
    float t = f_ * dot(s2, e2);
    float b1 = f_ * dot(s1, s);
    float b2 = f_ * dot(s2, ray->d);
    if (b1 < 0 || 1 < b1 || b2 < 0 || 1 < b2 || 1 < b1 + b2) return 0;
    if (t < ray->t_min || ray->t_max < t) return 0;
    v3 n0 = ld3(sc->vtx[f->vertices[0]].normal);
    v3 n1 = ld3(sc->vtx[f->vertices[1]].normal);
    v3 n2 = ld3(sc->vtx[f->vertices[2]].normal);
    v3 n = normalize(add(add(muls(n0, 1.0f - b1 - b2), muls(n1, b1)), muls(n2, b2)));
    out->time = t;
    out->pos = add(ray->o, muls(ray->d, t));
    out->normal = n;
    out->material_id = f->material_id;
    out->outward = 1;
    if (dot(n, ray->d) > 0.0f) { out->normal = neg(n); out->outward = 0; }
    return 1;
}

/* get_intersection_with_scene, :283-298.  A miss leaves every field but `time`
 * uninitialised in the shader; DESIGN.md §3.4 defines them (position = +inf, material 0). */
static hit_t get_intersection_with_scene(const scene_t *sc, ray_t ray, uint64_t *trav)
{
    hit_t inter;
    inter.time = ray.t_max + 1.0f;
    inter.pos = mk(INFINITY, INFINITY, INFINITY);
    inter.normal = mk(0, 0, 0);
    inter.material_id = 0;
    inter.outward = 1;
    for (uint32_t i = 0; i < sc->n_face; i++) {
        hit_t h;
        if (is_intersect_with_face(sc, &ray, &sc->face[i], &h)) {
            if (h.time <= ray.t_max) { ray.t_max = h.time; inter = h; }
        }
    }
    (*trav)++;
    return inter;
}

/* get_face_area, :302-307 */
static float get_face_area(const scene_t *sc, const rvcp_face_t *f)
{
    v3 v0 = ld3(sc->vtx[f->vertices[0]].position);
    v3 v1 = ld3(sc->vtx[f->vertices[1]].position);
    v3 v2 = ld3(sc->vtx[f->vertices[2]].position);
    return 0.5f * length(cross(sub(v1, v0), sub(v2, v0)));
}

/* sample_in_face, :311-329 */
static void sample_in_face(const scene_t *sc, const rvcp_face_t *f, rng_t *g, hit_t *inter)
{
    v3 v0 = ld3(sc->vtx[f->vertices[0]].position);
    v3 v1 = ld3(sc->vtx[f->vertices[1]].position);
    v3 v2 = ld3(sc->vtx[f->vertices[2]].position);
    float x = sqrtf(rand_next(g));
    float y = rand_next(g);
    inter->time = 0.0f;
    inter->pos = add(add(muls(v0, 1.0f - x), muls(v1, x * (1.0f - y))), muls(v2, x * y));
    inter->normal = normalize(ld3(sc->vtx[f->vertices[0]].normal));
    inter->material_id = f->material_id;
    inter->outward = 1;
}

/* sample_light_games101, :384-404.  Returns 0 when no light face exists (then `inter` is
 * uninitialised in the shader; DESIGN.md §3.4: the NEE term is skipped). */
static int sample_light_games101(const scene_t *sc, rng_t *g, int quirk, uint32_t n_lum_len,
                                 hit_t *inter, float *pdf_light)
{
    float emit_area_sum = 0;
    for (uint32_t i = 0; i < n_lum_len; i++)
        emit_area_sum += get_face_area(sc, &sc->face[lum_face_id(sc, i, quirk)]);
    float p = rand_next(g) * emit_area_sum;
    *pdf_light = 1.0f / emit_area_sum;
    emit_area_sum = 0.0f;
    for (uint32_t i = 0; i < n_lum_len; i++) {
        const rvcp_face_t *f = &sc->face[lum_face_id(sc, i, quirk)];
        emit_area_sum += get_face_area(sc, f);
        if (p <= emit_area_sum) { sample_in_face(sc, f, g, inter); return 1; }
    }
    return 0;
}

/* lambertian_brdf_eval, :338-350 */
static inline v3 lambertian_brdf_eval(const rvcp_material_t *m, v3 wi, v3 normal)
{
    float cos_theta = dot(normal, wi);
    if (cos_theta > 0.0f) return divs(ld3(m->albedo), PI_F);
    return mk(0, 0, 0);
}
/* lambertian_brdf_pdf, :358-365 */
static inline float lambertian_brdf_pdf(v3 wi, v3 normal)
{
    return dot(wi, normal) > 0.0f ? 0.5f / PI_F : 0.0f;
}

/* ray_trace_games101, :406-482 */
static v3 ray_trace_games101(const scene_t *sc, const params_t *P, rng_t *g, ray_t ray,
                             uint64_t *trav)
{
    v3 color = mk(0, 0, 0);
    v3 attenuation = mk(1, 1, 1);
    for (uint32_t depth = 0; depth < P->max_bounces; depth++) {
        if (attenuation.x < P->att_stop && attenuation.y < P->att_stop &&
            attenuation.z < P->att_stop) break;                                   /* :415 */

        hit_t inter_p = get_intersection_with_scene(sc, ray, trav);               /* :421 */
        if (inter_p.time > ray.t_max) { color = add(color, mk(0.1f, 0.1f, 0.1f)); break; }
        const rvcp_material_t *material_p = &sc->mat[inter_p.material_id];        /* :422 */
        if (material_p->ty == MATERIAL_LIGHT) {                                   /* :425 */
            if (depth == 0) color = add(color, mulv(attenuation, ld3(material_p->albedo)));
            break;
        }
        v3 p = inter_p.pos;

        hit_t inter_x;                                                            /* :434 */
        float pdf_light;
        if (sample_light_games101(sc, g, P->quirk, sc->n_lum, &inter_x, &pdf_light)) {
            const rvcp_material_t *material_x = &sc->mat[inter_x.material_id];
            float dist = length(sub(inter_x.pos, p));
            v3 ws = divs(sub(inter_x.pos, p), dist);
            ray_t shadow = { add(p, muls(ws, P->eps)), ws, P->t_min, P->t_max };  /* :441 */
            hit_t blocked = get_intersection_with_scene(sc, shadow, trav);
            float dist_blocked = length(sub(blocked.pos, p));
            if (fabsf(dist - dist_blocked) < P->eps) {                           /* :449 */
                v3 f = lambertian_brdf_eval(material_p, ws, inter_p.normal);
                v3 c = mulv(mulv(attenuation, ld3(material_x->albedo)), f);
                c = muls(c, dot(inter_p.normal, ws));
                c = muls(c, dot(inter_x.normal, neg(ws)));
                c = divs(c, dist * dist * pdf_light);   /* pow(dist, 2.0) := dist*dist */
                color = add(color, c);
            }
        }

        if (rand_next(g) > P->rr) break;                                          /* :462 */

        v3 wi = random_in_unit_hemisphere_surface(g, inter_p.normal);             /* :464 */
        v3 f = lambertian_brdf_eval(material_p, wi, inter_p.normal);
        float pdf = lambertian_brdf_pdf(wi, inter_p.normal);
        float denom = fmaxf(0.1f, pdf) * P->rr;
        v3 a = divs(muls(muls(f, 1.0f), dot(inter_p.normal, wi)), denom);
        attenuation = mulv(attenuation, a);                                       /* :465 */

        ray.o = add(inter_p.pos, muls(wi, P->eps));                               /* :473 */
        ray.d = wi;
        ray.t_min = P->t_min;
        ray.t_max = P->t_max;
    }
    return color;
}

/* ------------------------------------------------------------------------------------- */
/* Integrator mode 2: ray_tracer.comp (the file north_star names; compiled only by the     */
/* deprecated host, src/ray_tracer_deprecated/shader.rs:12).  RNG, sample_ray and          */
/* is_intersect_with_face are identical to the games101 shader (ray_tracer.comp:151-258,   */
/* :324-366).                                                                              */
/* ------------------------------------------------------------------------------------- */

/* is_intersect_with_quadratic_equation, ray_tracer.comp:260-297 */
static int quad_hit(float a, float b, float c, const ray_t *ray, hit_t *out)
{
    float delta = b * b - 4.0f * a * c;
    if (delta < 0.0f) return 0;                       /* sign(delta) < 0.0 */
    float sq = sqrtf(delta);
    float t0 = (-b + sq) / (2.0f * a);
    float t1 = (-b - sq) / (2.0f * a);
    if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
    float t;
    if (ray->t_min <= t0 && t0 <= ray->t_max) t = t0;
    else if (ray->t_min <= t1 && t1 <= ray->t_max) t = t1;
    else return 0;
    out->time = t;
    out->pos = add(ray->o, muls(ray->d, t));
    out->normal = mk(0, 0, 0);
    out->material_id = 0;
    out->outward = 1;
    return 1;
}

/* is_intersect_with_sphere, ray_tracer.comp:300-321 */
static int sphere_hit(const ray_t *ray, const rvcp_sphere_t *sp, hit_t *out)
{
    v3 ce = ld3(sp->center);
    v3 co = sub(ray->o, ce);
    float a = dot(ray->d, ray->d);
    float b = 2.0f * dot(ray->d, co);
    float c = dot(co, co) - sp->radius * sp->radius;
    if (!quad_hit(a, b, c, ray, out)) return 0;
    out->normal = normalize(sub(out->pos, ce));
    out->material_id = sp->material_id;
    v3 oc = sub(ray->o, ce);
    if (dot(oc, oc) < sp->radius * sp->radius) { out->normal = neg(out->normal); out->outward = 0; }
    return 1;
}

/* get_intersection_with_scene, ray_tracer.comp:369-393: spheres first, then faces */
static hit_t scene_hit_legacy(const scene_t *sc, ray_t ray, uint64_t *trav)
{
    hit_t inter;
    inter.time = ray.t_max + 1.0f;
    inter.pos = mk(INFINITY, INFINITY, INFINITY);
    inter.normal = mk(0, 0, 0);
    inter.material_id = 0;
    inter.outward = 1;
    for (uint32_t i = 0; i < sc->n_sph; i++) {
        hit_t h;
        if (sphere_hit(&ray, &sc->sph[i], &h) && h.time <= ray.t_max) { ray.t_max = h.time; inter = h; }
    }
    for (uint32_t i = 0; i < sc->n_face; i++) {
        hit_t h;
        if (is_intersect_with_face(sc, &ray, &sc->face[i], &h) && h.time <= ray.t_max) {
            ray.t_max = h.time;
            inter = h;
        }
    }
    (*trav)++;
    return inter;
}

/* GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N */
static inline v3 reflect_glsl(v3 I, v3 N) { return sub(I, muls(N, 2.0f * dot(N, I))); }
/* GLSL refract(I, N, eta) */
static inline v3 refract_glsl(v3 I, v3 N, float eta)
{
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk(0, 0, 0);
    return sub(muls(I, eta), muls(N, eta * d + sqrtf(k)));
}
/* fresnel_schlick, ray_tracer.comp:544-551; pow(x, 5.0) := ((x*x)*(x*x))*x */
static inline float fresnel_schlick(float cosine, float ratio)
{
    float r0 = (1.0f - ratio) / (1.0f + ratio);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    return r0 + (1.0f - r0) * (x * x * (x * x) * x);
}

/* material_scatter, ray_tracer.comp:491-602.  Unknown types leave attenuation 0 (:655). */
static void material_scatter(const rvcp_material_t *m, const ray_t *ray, const hit_t *h,
                             rng_t *g, const params_t *P, v3 *att, ray_t *nr)
{
    nr->o = h->pos; nr->t_min = P->t_min; nr->t_max = P->t_max; nr->d = mk(0, 0, 0);
    *att = mk(0, 0, 0);
    if (m->ty == 0) {                                   /* lambertian_scatter :491-513 */
        v3 u = normalize(random_in_unit_sphere(g));
        v3 dir = normalize(add(h->normal, u));
        if (fabsf(dir.x) < P->eps && fabsf(dir.y) < P->eps && fabsf(dir.z) < P->eps) dir = h->normal;
        *att = ld3(m->albedo);
        nr->d = dir;
    } else if (m->ty == 1) {                            /* metal_scatter :517-540 */
        v3 refl = reflect_glsl(ray->d, h->normal);
        if (dot(refl, h->normal) < 0.0f) refl = neg(refl);
        v3 dir;
        do {
            v3 u = normalize(random_in_unit_sphere(g));
            dir = normalize(add(refl, muls(u, m->fuzz)));
        } while (dot(dir, h->normal) < 0.0f);
        *att = ld3(m->albedo);
        nr->d = dir;
    } else if (m->ty == 2) {                            /* dielectric_scatter :553-581 */
        float ratio = h->outward ? (1.0f / m->refraction_ratio) : m->refraction_ratio;
        float cos_t = dot(neg(ray->d), h->normal);
        float sin_t = sqrtf(1.0f - cos_t * cos_t);
        int refracted = ratio * sin_t <= 1.0f;
        if (refracted && (rand_next(g) >= fresnel_schlick(cos_t, ratio)))
            nr->d = refract_glsl(ray->d, h->normal, ratio);
        else
            nr->d = reflect_glsl(ray->d, h->normal);
        *att = mk(1, 1, 1);
    }
}

/* ray_trace, ray_tracer.comp:618-694 (path_reuse_count is 0 or 1: its division is exact) */
static v3 ray_trace_legacy(const scene_t *sc, const params_t *P, rng_t *g, ray_t ray, uint64_t *trav)
{
    v3 color = mk(0, 0, 0);
    v3 attenuation = mk(1, 1, 1);
    for (uint32_t left = P->max_bounces; left > 0;) {
        left -= 1;
        hit_t inter = scene_hit_legacy(sc, ray, trav);
        if (inter.time > ray.t_max) {                   /* miss: sample_infinite_light = 0 */
            color = add(color, mulv(attenuation, mk(0, 0, 0)));
            break;
        }
        const rvcp_material_t *m = &sc->mat[inter.material_id];
        if (m->ty == MATERIAL_LIGHT) { color = add(color, mulv(attenuation, ld3(m->albedo))); break; }
        v3 new_att;
        ray_t new_ray;
        material_scatter(m, &ray, &inter, g, P, &new_att, &new_ray);
        attenuation = mulv(attenuation, new_att);
        ray = new_ray;
        ray.o = add(ray.o, muls(ray.d, P->t_min));     /* :670 RAY_T_MIN */
        if (attenuation.x < P->eps && attenuation.y < P->eps && attenuation.z < P->eps) break;
        if (rand_next(g) >= P->rr) break;
        attenuation = divs(attenuation, P->rr);
    }
    return color;
}

/* Float -> UNORM8 conversion of the stored value x in [0, 1], two rules
 * (rvcp_config_t.unorm_rule):
 *   0 RVCP_UNORM_DRIVER  -- the reference driver's: q = floor(4096 x), u8 = (255 q + 2048) >> 12,
 *                           fitted to the reference's own render Notes/README/fractal.png
 *                           (tests/test_mandelbrot.py pins it on every pixel);
 *   1 RVCP_UNORM_NEAREST -- u8 = floor(255 x + 1/2).
 * Both are applied as a count of thresholds: u8 = #{k in 1..255 : x >= G[k]}, with
 * G[k] = ceil((4096 k - 2048) / 255) / 4096 (driver) or (k - 1/2) / 255 (nearest). */
static double unorm_G(int rule, int k)
{
    return rule == 1 ? (k - 0.5) / 255.0 : ceil((4096.0 * k - 2048.0) / 255.0) / 4096.0;
}
static float g_unorm_T[2][256];
static pthread_once_t g_unorm_once = PTHREAD_ONCE_INIT;
static void unorm_init(void)
{
    for (int r = 0; r < 2; r++) {
        g_unorm_T[r][0] = 0.0f;
        for (int k = 1; k < 256; k++) g_unorm_T[r][k] = (float)unorm_G(r, k);
    }
}
static int rule_index(int rule) { return rule == 1 ? 1 : 0; }
uint8_t rvcp_oracle_unorm_u8_rule(float c, int rule)
{
    pthread_once(&g_unorm_once, unorm_init);
    const float *T = g_unorm_T[rule_index(rule)];
    float x = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;
    int n = 0;
    for (int k = 1; k < 256; k++) n += (x >= T[k]);
    return (uint8_t)n;
}
uint8_t rvcp_oracle_unorm_u8(float c) { return rvcp_oracle_unorm_u8_rule(c, 0); }

/* ------------------------------------------------------------------------------------- */
/* Camera: sample_ray, :217-235                                                            */
/* ------------------------------------------------------------------------------------- */
typedef struct { v3 pos, fwd, up; float t_near, t_far, vfov; } cam_t;

static cam_t cam_of(const rvcp_push_constant_t *pc)
{
    cam_t c;
    c.pos = ld3(pc->camera.position);
    c.up = ld3(pc->camera.up);
    c.fwd = ld3(pc->camera.forward);
    c.t_near = pc->camera.t_near;
    c.t_far = pc->camera.t_far;
    c.vfov = pc->camera.vertical_fov;
    return c;
}

static ray_t sample_ray(const cam_t *c, float u_, float v_, float W, float H)
{
    float rad = c->vfov / 2.0f * PI_F / 180.0f;                 /* degree_to_radian :141 */
    float h = 2.0f * c->t_near * tanf(rad);
    float w = h * W / H;
    v3 u = muls(normalize(cross(c->fwd, c->up)), w);
    v3 v = muls(normalize(cross(c->fwd, u)), h);
    v3 pos = add(c->pos, muls(c->fwd, c->t_near));
    v3 uv_pos = add(add(pos, muls(u, u_ - 0.5f)), muls(v, v_ - 0.5f));
    float t_coef = length(sub(uv_pos, c->pos)) / length(sub(pos, c->pos));
    ray_t r = { c->pos, normalize(sub(uv_pos, c->pos)), c->t_near * t_coef, c->t_far * t_coef };
    return r;
}

/* ------------------------------------------------------------------------------------- */
/* Tone map: pow(clamp(c, 0, 1), 0.6) (:498) then UNORM8 store (:500).                     */
/* u8 = #{k in 1..255 : c >= T[k]}, T[k] = float(G[k]^(1/0.6)) (G above).   */
/* ------------------------------------------------------------------------------------- */
static float g_gamma_T[2][256];
static pthread_once_t g_gamma_once = PTHREAD_ONCE_INIT;
static void gamma_init(void)
{
    for (int r = 0; r < 2; r++) {
        g_gamma_T[r][0] = 0.0f;
        for (int k = 1; k < 256; k++) g_gamma_T[r][k] = (float)pow(unorm_G(r, k), 1.0 / 0.6);
    }
}
uint8_t rvcp_oracle_gamma_u8_rule(float c, int rule)
{
    pthread_once(&g_gamma_once, gamma_init);
    const float *T = g_gamma_T[rule_index(rule)];
    float x = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;     /* clamp, NaN -> 0 */
    int n = 0;
    for (int k = 1; k < 256; k++) n += (x >= T[k]);
    return (uint8_t)n;
}
uint8_t rvcp_oracle_gamma_u8(float c) { return rvcp_oracle_gamma_u8_rule(c, 0); }
float rvcp_oracle_gamma_threshold_rule(int k, int rule)
{
    pthread_once(&g_gamma_once, gamma_init);
    return (k >= 0 && k < 256) ? g_gamma_T[rule_index(rule)][k] : 0.0f;
}
float rvcp_oracle_gamma_threshold(int k) { return rvcp_oracle_gamma_threshold_rule(k, 0); }

/* ------------------------------------------------------------------------------------- */
/* main, :486-501, over a sub-rectangle of a W x H frame, multi-threaded by rows           */
/* ------------------------------------------------------------------------------------- */
typedef struct {
    const scene_t *sc; const params_t *P; cam_t cam; float time;
    uint32_t W, H, x0, y0, tw, th, tid, nthreads;
    float *lin; uint8_t *rgba; uint64_t trav;
} job_t;

static void render_pixel(job_t *J, uint32_t x, uint32_t y, uint32_t out_idx)
{
    const float Wf = (float)J->W, Hf = (float)J->H;
    float u_ = ((float)x + 0.5f) / Wf, v_ = ((float)y + 0.5f) / Hf;     /* :488 */
    rng_t g;
    srand_glsl(&g, J->time, u_, v_);                                    /* :489 */
    ray_t ray = sample_ray(&J->cam, u_, v_, Wf, Hf);                    /* :491 */
    v3 color = mk(0, 0, 0);
    const float sppf = (float)J->P->spp;
    if (J->P->integrator == 1) {                                       /* ray_tracer.comp:815-819 */
        for (uint32_t i = 0; i < J->P->spp; i++)
            color = add(color, ray_trace_legacy(J->sc, J->P, &g, ray, &J->trav));
        color = divs(color, sppf);
    } else {
        for (uint32_t i = 0; i < J->P->spp; i++)                       /* :494-496 */
            color = add(color, divs(ray_trace_games101(J->sc, J->P, &g, ray, &J->trav), sppf));
    }
    if (J->lin) {
        J->lin[3 * (size_t)out_idx + 0] = color.x;
        J->lin[3 * (size_t)out_idx + 1] = color.y;
        J->lin[3 * (size_t)out_idx + 2] = color.z;
    }
    if (J->rgba) {
        uint8_t (*q)(float, int) = J->P->integrator == 1 ? rvcp_oracle_unorm_u8_rule
                                                         : rvcp_oracle_gamma_u8_rule;
        const int rule = J->P->unorm_rule;
        J->rgba[4 * (size_t)out_idx + 0] = q(color.x, rule);
        J->rgba[4 * (size_t)out_idx + 1] = q(color.y, rule);
        J->rgba[4 * (size_t)out_idx + 2] = q(color.z, rule);
        J->rgba[4 * (size_t)out_idx + 3] = 255;
    }
}

/* Threads take 16-pixel chunks of the rectangle round-robin (balanced even for 1-row rects). */
static void *render_rows(void *arg)
{
    job_t *J = (job_t *)arg;
    const uint64_t n = (uint64_t)J->tw * J->th;
    for (uint64_t c = (uint64_t)J->tid * 16u; c < n; c += (uint64_t)J->nthreads * 16u)
        for (uint64_t i = c; i < c + 16u && i < n; i++) {
            const uint32_t ty = (uint32_t)(i / J->tw), tx = (uint32_t)(i % J->tw);
            render_pixel(J, J->x0 + tx, J->y0 + ty, (uint32_t)i);
        }
    return NULL;
}

/* Render the tw x th sub-rectangle at (x0, y0) of a W x H frame.  Output arrays are
 * tw*th*3 floats / tw*th*4 bytes (either may be NULL).  Returns 0 or a negative error. */
int rvcp_oracle_render(const rvcp_material_t *materials, uint32_t n_materials,
                       const rvcp_vertex_t *vertices, uint32_t n_vertices,
                       const rvcp_face_t *faces, uint32_t n_faces,
                       const rvcp_sphere_t *spheres, uint32_t n_spheres,
                       const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                       const rvcp_push_constant_t *push, const rvcp_config_t *cfg,
                       uint32_t W, uint32_t H, uint32_t x0, uint32_t y0, uint32_t tw,
                       uint32_t th, float *out_linear, uint8_t *out_rgba8,
                       uint64_t *out_traversals, int nthreads)
{
    if (!push || !cfg || !W || !H || x0 + tw > W || y0 + th > H) return RVCP_E_INVALID;
    if (n_materials == 0 || !materials) return RVCP_E_INVALID;
    for (uint32_t i = 0; i < n_faces; i++) {
        for (int k = 0; k < 3; k++) if (faces[i].vertices[k] >= n_vertices) return RVCP_E_INVALID;
        if (faces[i].material_id >= n_materials) return RVCP_E_INVALID;
    }
    for (uint32_t i = 0; i < n_lum_face_ids; i++)
        if (lum_face_ids[i] >= n_faces) return RVCP_E_INVALID;
    for (uint32_t i = 0; i < n_spheres; i++)
        if (spheres[i].material_id >= n_materials) return RVCP_E_INVALID;
    if (cfg->integrator != 0 && cfg->integrator != 1) return RVCP_E_UNSUPPORTED;
    pthread_once(&g_gamma_once, gamma_init);
    pthread_once(&g_unorm_once, unorm_init);

    scene_t sc = { materials, n_materials, vertices, n_vertices, faces, n_faces,
                   lum_face_ids, n_lum_face_ids, spheres, cfg->integrator == 1 ? n_spheres : 0 };
    params_t P = { cfg->spp, cfg->max_bounces, cfg->attenuation_stop_eps, cfg->ray_t_min,
                   cfg->ray_t_max, cfg->rr_probability, cfg->eps, cfg->lum_id_std140_quirk,
                   cfg->integrator, cfg->unorm_rule };
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th_ids = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th_ids) { free(jobs); free(th_ids); return RVCP_E_NOMEM; }
    cam_t cam = cam_of(push);
    for (int t = 0; t < nthreads; t++) {
        job_t j = { &sc, &P, cam, push->time, W, H, x0, y0, tw, th, (uint32_t)t,
                    (uint32_t)nthreads, out_linear, out_rgba8, 0 };
        jobs[t] = j;
    }
    int started = 0;
    for (int t = 1; t < nthreads; t++) {
        if (pthread_create(&th_ids[t], NULL, render_rows, &jobs[t]) != 0) break;
        started = t;
    }
    if (started < nthreads - 1) {        /* could not spawn: run the rest inline */
        for (int t = started + 1; t < nthreads; t++) render_rows(&jobs[t]);
    }
    render_rows(&jobs[0]);
    uint64_t trav = jobs[0].trav;
    for (int t = 1; t <= started; t++) pthread_join(th_ids[t], NULL);
    for (int t = 1; t < nthreads; t++) trav += jobs[t].trav;
    if (out_traversals) *out_traversals = trav;
    free(jobs);
    free(th_ids);
    return RVCP_OK;
}

/* ------------------------------------------------------------------------------------- */
/* The Mandelbrot operator, assets/shaders/mandelbrot.comp:12-33 (single-threaded).       */
/* out_rgba: W*H*4 grey UNORM8 of the escape time i; out_value (optional): i per pixel.    */
/* The iteration is evaluated as the reference's compiled shader evaluated it (DESIGN.md  */
/* §3.7): the two products of z.x' contracted into one fma, and z.y*z.x + z.x*z.y (which  */
/* is exactly 2*(z.x*z.y)) contracted with + c.y into fma(z.x + z.x, z.y, c.y); with the   */
/* driver's UNORM rule this reproduces Notes/README/fractal.png on every pixel; length is */
/* √dot with the fused 2-D dot of §3.1.                                                   */
/* ------------------------------------------------------------------------------------- */
int rvcp_oracle_mandelbrot(const rvcp_mandelbrot_push_t *push, uint32_t W, uint32_t H,
                           int unorm_rule, uint8_t *out_rgba, float *out_value)
{
    if (!push || !out_rgba || !W || !H) return RVCP_E_INVALID;
    for (uint32_t y = 0; y < H; y++) {
        for (uint32_t x = 0; x < W; x++) {
            float nx = ((float)x + 0.5f) / (float)W;                  /* :13 */
            float ny = ((float)y + 0.5f) / (float)H;
            float cx = (nx - 0.5f) * 2.0f, cy = (ny - 0.5f) * 2.0f;   /* :15 */
            cx = cx / push->scale + push->position[0];                /* :16 */
            cy = cy / push->scale + push->position[1];
            cx = cx - 1.0f;                                           /* :17 */
            cy = cy - 0.0f;
            float zx = 0.0f, zy = 0.0f, i;
            for (i = 0.0f; i < 1.0f; i += 0.005f) {                    /* :21 */
                float nzx = fmaf(zx, zx, -(zy * zy)) + cx;            /* :22-25 */
                float nzy = fmaf(zx + zx, zy, cy);
                zx = nzx;
                zy = nzy;
                if (sqrtf(fmaf(zy, zy, zx * zx)) > 4.0f) break;      /* length(z) > 4, §3.1 dot */
            }
            const size_t p = (size_t)y * W + x;
            const uint8_t u = rvcp_oracle_unorm_u8_rule(i, unorm_rule); /* vec4(vec3(i), 1) */
            out_rgba[4 * p + 0] = u;
            out_rgba[4 * p + 1] = u;
            out_rgba[4 * p + 2] = u;
            out_rgba[4 * p + 3] = 255;
            if (out_value) out_value[p] = i;
        }
    }
    return RVCP_OK;
}

/* ------------------------------------------------------------------------------------- */
/* Known-answer-test helpers (tests/test_oracle_kat.py)                                    */
/* ------------------------------------------------------------------------------------- */

/* out[0] = seed after srand(time, (u, v)); out[1..n] = the first n rand() values. */
void rvcp_oracle_rand_sequence(float time, float u, float v, int n, float *out)
{
    rng_t g;
    srand_glsl(&g, time, u, v);
    out[0] = g.seed;
    for (int i = 0; i < n; i++) out[1 + i] = rand_next(&g);
}

/* Single ray-triangle test (is_intersect_with_face).  ray = {ox,oy,oz,dx,dy,dz,tmin,tmax},
 * tri = 3 positions; out = {t, b1, b2} on hit.  Returns 1 on hit. */
int rvcp_oracle_intersect(const float *ray, const float *tri, float *out)
{
    rvcp_vertex_t v[3];
    memset(v, 0, sizeof v);
    for (int k = 0; k < 3; k++) {
        v[k].position[0] = tri[3 * k]; v[k].position[1] = tri[3 * k + 1];
        v[k].position[2] = tri[3 * k + 2]; v[k].normal[1] = 1.0f;
    }
    rvcp_face_t f = { {0, 1, 2}, 0 };
    scene_t sc = { NULL, 0, v, 3, &f, 1, NULL, 0, NULL, 0 };
    ray_t r = { mk(ray[0], ray[1], ray[2]), mk(ray[3], ray[4], ray[5]), ray[6], ray[7] };
    hit_t h;
    if (!is_intersect_with_face(&sc, &r, &f, &h)) return 0;
    /* recover b1, b2 exactly as the shader computed them */
    v3 e1 = sub(ld3(v[1].position), ld3(v[0].position));
    v3 e2 = sub(ld3(v[2].position), ld3(v[0].position));
    v3 s = sub(r.o, ld3(v[0].position));
    v3 s1 = cross(r.d, e2), s2 = cross(s, e1);
    float f_ = 1.0f / dot(s1, e1);
    out[0] = h.time;
    out[1] = f_ * dot(s1, s);
    out[2] = f_ * dot(s2, r.d);
    return 1;
}

/* Primary ray of pixel (x, y): out = {ox,oy,oz,dx,dy,dz,tmin,tmax}. */
void rvcp_oracle_sample_ray(const rvcp_push_constant_t *push, uint32_t W, uint32_t H,
                            uint32_t x, uint32_t y, float *out)
{
    cam_t cam = cam_of(push);
    float u_ = ((float)x + 0.5f) / (float)W, v_ = ((float)y + 0.5f) / (float)H;
    ray_t r = sample_ray(&cam, u_, v_, (float)W, (float)H);
    out[0] = r.o.x; out[1] = r.o.y; out[2] = r.o.z;
    out[3] = r.d.x; out[4] = r.d.y; out[5] = r.d.z;
    out[6] = r.t_min; out[7] = r.t_max;
}
