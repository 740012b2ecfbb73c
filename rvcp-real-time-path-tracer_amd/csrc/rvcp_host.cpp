// rvcp_host.cpp -- C-ABI host runtime of librvcp (include/rvcp.h).
//
// Replaces the Vulkano runtime of the reference (src/ray_tracer/vulkan.rs): pipeline
// creation (:576-603) -> rvcp_create, descriptor-set upload (:454-574) -> rvcp_upload_scene,
// push constants + dispatch (:406-452) -> rvcp_render / rvcp_render_shard_async.
//
// Compiled with hipcc -ffp-contract=off: the frame constants it derives (camera basis,
// light-area prefix sums, gamma thresholds) use the same float operations as the shader, so
// the kernel's results stay bit-identical to the CPU oracle.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/rvcp.h"
#include "rvcp_internal.h"

using namespace rvcp;

struct rvcp_ctx {
    rvcp_config_t cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, evm = nullptr, ev1 = nullptr;   // start, main kernel, end
    int grid_capacity[kMaxVariant + 1] = {};   // resident workgroups per kernel variant
    int legacy_capacity = 0;                   // ... of the RVCP_INTEGRATOR_LEGACY kernel
    int bvh_capacity = 0;                      // ... of the RVCP_ACCEL_BVH path kernel
    uint32_t n_simds = 1024;

    // scene (device)
    TriRecord *d_tri = nullptr;
    rvcp_face_t *d_faces = nullptr;
    rvcp_vertex_t *d_verts = nullptr;
    MatRecord *d_mats = nullptr;
    FaceShade *d_shade = nullptr;
    LightRecord *d_lights = nullptr;
    rvcp_material_t *d_rawmats = nullptr;     // RVCP_INTEGRATOR_LEGACY: fuzz / ior needed
    rvcp_sphere_t *d_spheres = nullptr;
    // opt-in BVH (RVCP_ACCEL_BVH): nodes, leaf-ordered triangles and their face ids
    Bvh4Node *d_bvh_nodes = nullptr;
    TriRecord *d_bvh_tris = nullptr;
    int32_t bvh_root = 0;
    int bvh_depth = 0;
    float *d_gamma = nullptr;
    float *d_unorm = nullptr;
    unsigned long long *d_counters = nullptr;
    uint32_t n_faces = 0, n_lights = 0, n_mats = 0, n_verts = 0, n_spheres = 0;
    float light_total = 0.0f, light_pdf = 0.0f;
    bool has_scene = false;

    // primary pre-pass output (variant 3): compact list of surface pixels
    SurfRecord *d_surf = nullptr;
    size_t cap_surf = 0;

    // staging for the synchronous host API
    uint32_t *d_rgba = nullptr;
    float *d_lin = nullptr;
    size_t cap_rgba = 0, cap_lin = 0;
    // n_gpus > 1: shard 0's packed stripes
    uint32_t *d_pack_rgba = nullptr;
    float *d_pack_lin = nullptr;
    size_t cap_surf_pack = 0;

    // RVCP_DEBUG_TIMELINE=<file>: per-wave timeline of the path kernel appended per render
    unsigned long long *d_timeline = nullptr;
    size_t cap_timeline = 0, last_timeline_waves = 0;

    // n_gpus > 1: contexts of the other GPUs (shards 1..N-1) and their packed shard buffers
    std::vector<rvcp_ctx *> subs;
    std::vector<uint32_t *> shard_rgba;
    std::vector<float *> shard_lin;
    std::vector<size_t> shard_cap;

    // last launch
    bool pending = false;
    bool last_trivial = false;
    uint64_t last_pixels = 0;
    uint32_t last_spp = 0;

    std::string err;
};

namespace {

thread_local std::string g_create_error;

int fail(rvcp_ctx *ctx, int code, const std::string &msg)
{
    if (ctx) ctx->err = msg;
    else g_create_error = msg;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                  \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((ctx), RVCP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- host-side vec3 with the shader's evaluation order ----
struct h3 { float x, y, z; };
inline h3 mk(float x, float y, float z) { return h3{x, y, z}; }
inline h3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }
inline h3 add(h3 a, h3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline h3 sub(h3 a, h3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline h3 muls(h3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
// the shader builtins, fused as in DESIGN.md §3.1 (these restate shader code, not glam)
inline float dot(h3 a, h3 b) { return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x)); }
inline h3 cross(h3 a, h3 b) {
    return mk(std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)),
              std::fma(a.x, b.y, -(a.y * b.x)));
}
inline float length(h3 a) { return std::sqrt(dot(a, a)); }
inline h3 normalize(h3 a) { return muls(a, 1.0f / std::sqrt(dot(a, a))); }
inline void st3(float *d, h3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

// get_face_area, ray_tracer_games101_branch.comp:302-307
float face_area(const rvcp_vertex_t *v, const rvcp_face_t &f)
{
    h3 v0 = ld3(v[f.vertices[0]].position), v1 = ld3(v[f.vertices[1]].position);
    h3 v2 = ld3(v[f.vertices[2]].position);
    return 0.5f * length(cross(sub(v1, v0), sub(v2, v0)));
}

// sample_ray's frame constants, :217-227
void camera_constants(const rvcp_push_constant_t &pc, uint32_t W, uint32_t H, FrameArgs &A)
{
    const float PI = 3.1415926f;
    h3 cpos = ld3(pc.camera.position), up = ld3(pc.camera.up), fwd = ld3(pc.camera.forward);
    const float rad = pc.camera.vertical_fov / 2.0f * PI / 180.0f;   // degree_to_radian :141
    const float h = 2.0f * pc.camera.t_near * std::tan(rad);
    const float w = h * (float)W / (float)H;
    h3 u = muls(normalize(cross(fwd, up)), w);
    h3 v = muls(normalize(cross(fwd, u)), h);
    h3 pos = add(cpos, muls(fwd, pc.camera.t_near));
    st3(A.cam_pos, cpos);
    st3(A.u, u);
    st3(A.v, v);
    st3(A.pos, pos);
    A.base_len = length(sub(pos, cpos));
    A.t_near = pc.camera.t_near;
    A.t_far = pc.camera.t_far;
    A.time = pc.time;
}

template <typename T>
int dev_upload(rvcp_ctx *ctx, T **dst, const void *src, size_t n)
{
    if (*dst) { (void)hipFree(*dst); *dst = nullptr; }
    const size_t bytes = n ? n * sizeof(T) : sizeof(T);
    HIP_TRY(ctx, hipMalloc((void **)dst, bytes));
    if (n) HIP_TRY(ctx, hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return RVCP_OK;
}

void free_scene(rvcp_ctx *ctx)
{
    (void)hipFree(ctx->d_tri); ctx->d_tri = nullptr;
    (void)hipFree(ctx->d_faces); ctx->d_faces = nullptr;
    (void)hipFree(ctx->d_verts); ctx->d_verts = nullptr;
    (void)hipFree(ctx->d_mats); ctx->d_mats = nullptr;
    (void)hipFree(ctx->d_shade); ctx->d_shade = nullptr;
    (void)hipFree(ctx->d_lights); ctx->d_lights = nullptr;
    (void)hipFree(ctx->d_rawmats); ctx->d_rawmats = nullptr;
    (void)hipFree(ctx->d_spheres); ctx->d_spheres = nullptr;
    (void)hipFree(ctx->d_bvh_nodes); ctx->d_bvh_nodes = nullptr;
    (void)hipFree(ctx->d_bvh_tris); ctx->d_bvh_tris = nullptr;
    ctx->has_scene = false;
}

}  // namespace

extern "C" {

const char *rvcp_version(void) { return "rvcp-mi355x 0.1.0 (gfx950)"; }

int rvcp_config_default_for(int32_t integrator, rvcp_config_t *cfg)
{
    if (!cfg) return RVCP_E_INVALID;
    if (integrator == RVCP_INTEGRATOR_GAMES101) return rvcp_config_default(cfg);
    if (integrator != RVCP_INTEGRATOR_LEGACY) return RVCP_E_UNSUPPORTED;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->integrator = RVCP_INTEGRATOR_LEGACY;
    cfg->spp = 5;                       // ray_tracer.comp:8
    cfg->max_bounces = 3;               // :9
    cfg->attenuation_stop_eps = 0.01f;  // :10 (unused by ray_trace)
    cfg->ray_t_min = 0.01f;             // :11
    cfg->ray_t_max = 1000.0f;           // :12
    cfg->rr_probability = 1.0f;         // :13
    cfg->eps = 0.001f;                  // :5
    cfg->lum_id_std140_quirk = 1;       // (unused by ray_trace)
    cfg->n_gpus = 1;
    return RVCP_OK;
}

int rvcp_config_default(rvcp_config_t *cfg)
{
    if (!cfg) return RVCP_E_INVALID;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->device = 0;
    cfg->integrator = RVCP_INTEGRATOR_GAMES101;
    cfg->spp = 20;                      // ray_tracer_games101_branch.comp:8
    cfg->max_bounces = 15;              // :9
    cfg->attenuation_stop_eps = 0.05f;  // :10
    cfg->ray_t_min = 0.01f;             // :11
    cfg->ray_t_max = 10000.0f;          // :12
    cfg->rr_probability = 0.8f;         // :13
    cfg->eps = 0.001f;                  // :5
    cfg->lum_id_std140_quirk = 1;
    cfg->n_gpus = 1;
    return RVCP_OK;
}

const char *rvcp_last_error(const rvcp_ctx_t *ctx)
{
    return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int rvcp_create(const rvcp_config_t *cfg, rvcp_ctx_t **out_ctx)
{
    if (!cfg || !out_ctx) return fail(nullptr, RVCP_E_INVALID, "null argument");
    *out_ctx = nullptr;
    if (cfg->integrator != RVCP_INTEGRATOR_GAMES101 && cfg->integrator != RVCP_INTEGRATOR_LEGACY)
        return fail(nullptr, RVCP_E_UNSUPPORTED, "unsupported integrator");
    if (cfg->spp == 0) return fail(nullptr, RVCP_E_INVALID, "spp must be > 0");
    if (cfg->kernel_variant < 0 || cfg->kernel_variant > kMaxVariant)
        return fail(nullptr, RVCP_E_INVALID, "unknown kernel_variant");
    if (cfg->n_gpus < 0 || cfg->n_gpus > 64)
        return fail(nullptr, RVCP_E_INVALID, "n_gpus must be in [0, 64]");
    if (cfg->accel != RVCP_ACCEL_NONE && cfg->accel != RVCP_ACCEL_BVH)
        return fail(nullptr, RVCP_E_INVALID, "unknown accel");
    if (cfg->accel == RVCP_ACCEL_BVH && cfg->integrator != RVCP_INTEGRATOR_GAMES101)
        return fail(nullptr, RVCP_E_UNSUPPORTED, "RVCP_ACCEL_BVH is implemented for the games101 integrator");
    if (!(cfg->ray_t_max < 16777216.0f))
        return fail(nullptr, RVCP_E_INVALID, "ray_t_max must be < 2^24 (miss test t_max + 1)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, RVCP_E_HIP, "no HIP device");
    if (cfg->device < 0 || cfg->device >= ndev)
        return fail(nullptr, RVCP_E_INVALID, "device ordinal out of range");

    rvcp_ctx *ctx = new (std::nothrow) rvcp_ctx();
    if (!ctx) return fail(nullptr, RVCP_E_NOMEM, "out of memory");
    ctx->cfg = *cfg;
    ctx->device = cfg->device;
    auto bail = [&](int rc) {
        g_create_error = ctx->err;
        rvcp_destroy(ctx);
        return rc;
    };
    int rc;
    if (hipSetDevice(ctx->device) != hipSuccess) return bail(fail(ctx, RVCP_E_HIP, "hipSetDevice"));
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->evm) != hipSuccess ||
        hipEventCreate(&ctx->ev1) != hipSuccess)
        return bail(fail(ctx, RVCP_E_HIP, "stream/event creation failed"));

    // Gamma thresholds T[k] = float(((k - 0.5) / 255)^(1/0.6)), DESIGN.md §3.3
    float T[257];
    T[0] = 0.0f;
    for (int k = 1; k < 256; k++) T[k] = (float)std::pow((k - 0.5) / 255.0, 1.0 / 0.6);
    T[256] = INFINITY;
    if ((rc = dev_upload<float>(ctx, &ctx->d_gamma, T, 257)) != RVCP_OK) return bail(rc);
    // UNORM8 thresholds U[k] = float((k - 0.5) / 255) for ray_tracer.comp's gamma-free store
    for (int k = 1; k < 256; k++) T[k] = (float)((k - 0.5) / 255.0);
    if ((rc = dev_upload<float>(ctx, &ctx->d_unorm, T, 257)) != RVCP_OK) return bail(rc);
    if (hipMalloc((void **)&ctx->d_counters, 4 * sizeof(unsigned long long)) != hipSuccess)
        return bail(fail(ctx, RVCP_E_HIP, "hipMalloc counters"));

    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
        cus = 256;
    // RVCP_DEBUG_BLOCKS_PER_CU caps the persistent grid (occupancy experiments only)
    const char *cap_env = std::getenv("RVCP_DEBUG_BLOCKS_PER_CU");
    const int cap = cap_env ? std::atoi(cap_env) : 0;
    ctx->n_simds = (uint32_t)cus * 4u;
    for (int v = 1; v <= kMaxVariant; v++) {
        int per_cu = 0;
        if (rvcp_games101_occupancy(v, &per_cu) != 0 || per_cu <= 0) per_cu = 1;
        if (cap > 0 && cap < per_cu) per_cu = cap;
        ctx->grid_capacity[v] = per_cu * cus;
    }
    {
        int per_cu = 0;
        if (rvcp_legacy_occupancy(&per_cu) != 0 || per_cu <= 0) per_cu = 1;
        if (cap > 0 && cap < per_cu) per_cu = cap;
        ctx->legacy_capacity = per_cu * cus;
        per_cu = 0;
        if (rvcp_games101_occupancy(kOccupancyBvh, &per_cu) != 0 || per_cu <= 0) per_cu = 1;
        if (cap > 0 && cap < per_cu) per_cu = cap;
        ctx->bvh_capacity = per_cu * cus;
    }
    if (cfg->n_gpus > 1) {   // one sub-context per further GPU (shards 1..N-1)
        for (int i = 1; i < cfg->n_gpus; i++) {
            rvcp_config_t sub_cfg = *cfg;
            sub_cfg.n_gpus = 1;
            sub_cfg.device = (cfg->device + i) % ndev;
            rvcp_ctx_t *sub = nullptr;
            if ((rc = rvcp_create(&sub_cfg, &sub)) != RVCP_OK) {
                ctx->err = "sub-context on device " + std::to_string(sub_cfg.device) + ": " + g_create_error;
                return bail(rc);
            }
            ctx->subs.push_back(sub);
            ctx->shard_rgba.push_back(nullptr);
            ctx->shard_lin.push_back(nullptr);
            ctx->shard_cap.push_back(0);
            if (sub_cfg.device != cfg->device) {   // direct xGMI copies into the frame's GPU
                int ok = 0;
                if (hipDeviceCanAccessPeer(&ok, cfg->device, sub_cfg.device) == hipSuccess && ok) {
                    (void)hipSetDevice(cfg->device);
                    const hipError_t pe = hipDeviceEnablePeerAccess(sub_cfg.device, 0);
                    if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                        return bail(fail(ctx, RVCP_E_HIP, "hipDeviceEnablePeerAccess failed"));
                    (void)hipGetLastError();
                }
            }
        }
        (void)hipSetDevice(cfg->device);
    }
    *out_ctx = ctx;
    return RVCP_OK;
}

int rvcp_destroy(rvcp_ctx_t *ctx)
{
    if (!ctx) return RVCP_OK;
    for (size_t i = 0; i < ctx->subs.size(); i++) {
        if (!ctx->subs[i]) continue;
        (void)hipSetDevice(ctx->subs[i]->device);
        (void)hipFree(ctx->shard_rgba[i]);
        (void)hipFree(ctx->shard_lin[i]);
        rvcp_destroy(ctx->subs[i]);
    }
    ctx->subs.clear();
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    free_scene(ctx);
    (void)hipFree(ctx->d_gamma);
    (void)hipFree(ctx->d_unorm);
    (void)hipFree(ctx->d_counters);
    (void)hipFree(ctx->d_rgba);
    (void)hipFree(ctx->d_lin);
    (void)hipFree(ctx->d_surf);
    (void)hipFree(ctx->d_timeline);
    (void)hipFree(ctx->d_pack_rgba);
    (void)hipFree(ctx->d_pack_lin);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->evm) (void)hipEventDestroy(ctx->evm);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return RVCP_OK;
}

static int upload_one(rvcp_ctx_t *ctx, const rvcp_material_t *materials, uint32_t n_materials,
                      const rvcp_vertex_t *vertices, uint32_t n_vertices,
                      const rvcp_face_t *faces, uint32_t n_faces,
                      const rvcp_sphere_t *spheres, uint32_t n_spheres,
                      const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                      const uint32_t *lum_sphere_ids, uint32_t n_lum_sphere_ids);

int rvcp_upload_scene(rvcp_ctx_t *ctx, const rvcp_material_t *materials, uint32_t n_materials,
                      const rvcp_vertex_t *vertices, uint32_t n_vertices,
                      const rvcp_face_t *faces, uint32_t n_faces,
                      const rvcp_sphere_t *spheres, uint32_t n_spheres,
                      const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                      const uint32_t *lum_sphere_ids, uint32_t n_lum_sphere_ids)
{
    if (!ctx) return RVCP_E_INVALID;
    int rc = upload_one(ctx, materials, n_materials, vertices, n_vertices, faces, n_faces,
                        spheres, n_spheres, lum_face_ids, n_lum_face_ids, lum_sphere_ids,
                        n_lum_sphere_ids);
    for (rvcp_ctx *sub : ctx->subs) {
        if (rc != RVCP_OK) break;
        rc = upload_one(sub, materials, n_materials, vertices, n_vertices, faces, n_faces,
                        spheres, n_spheres, lum_face_ids, n_lum_face_ids, lum_sphere_ids,
                        n_lum_sphere_ids);
        if (rc != RVCP_OK) ctx->err = "sub-context upload: " + sub->err;
    }
    (void)hipSetDevice(ctx->device);
    return rc;
}

static int upload_one(rvcp_ctx_t *ctx, const rvcp_material_t *materials, uint32_t n_materials,
                      const rvcp_vertex_t *vertices, uint32_t n_vertices,
                      const rvcp_face_t *faces, uint32_t n_faces,
                      const rvcp_sphere_t *spheres, uint32_t n_spheres,
                      const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                      const uint32_t *lum_sphere_ids, uint32_t n_lum_sphere_ids)
{
    (void)lum_sphere_ids; (void)n_lum_sphere_ids;
    if (!ctx) return RVCP_E_INVALID;
    if (!materials || n_materials == 0) return fail(ctx, RVCP_E_INVALID, "need >= 1 material");
    if ((n_vertices && !vertices) || (n_faces && !faces) || (n_lum_face_ids && !lum_face_ids) ||
        (n_spheres && !spheres))
        return fail(ctx, RVCP_E_INVALID, "null array with nonzero length");
    for (uint32_t i = 0; i < n_spheres; i++)
        if (spheres[i].material_id >= n_materials)
            return fail(ctx, RVCP_E_INVALID, "sphere " + std::to_string(i) + " material out of range");
    for (uint32_t i = 0; i < n_faces; i++) {
        for (int k = 0; k < 3; k++)
            if (faces[i].vertices[k] >= n_vertices)
                return fail(ctx, RVCP_E_INVALID, "face " + std::to_string(i) + " vertex index out of range");
        if (faces[i].material_id >= n_materials)
            return fail(ctx, RVCP_E_INVALID, "face " + std::to_string(i) + " material out of range");
    }
    for (uint32_t i = 0; i < n_lum_face_ids; i++)
        if (lum_face_ids[i] >= n_faces)
            return fail(ctx, RVCP_E_INVALID, "luminous face id out of range");
    HIP_TRY(ctx, hipSetDevice(ctx->device));

    // triangles: v0, e1 = v1 - v0, e2 = v2 - v0 (:243-248)
    std::vector<TriRecord> tri(n_faces);
    for (uint32_t i = 0; i < n_faces; i++) {
        h3 v0 = ld3(vertices[faces[i].vertices[0]].position);
        h3 v1 = ld3(vertices[faces[i].vertices[1]].position);
        h3 v2 = ld3(vertices[faces[i].vertices[2]].position);
        std::memset(&tri[i], 0, sizeof(TriRecord));
        st3(tri[i].v0, v0);
        st3(tri[i].e1, sub(v1, v0));
        st3(tri[i].e2, sub(v2, v0));
    }
    std::vector<MatRecord> mats(n_materials);
    for (uint32_t i = 0; i < n_materials; i++) {
        std::memcpy(mats[i].albedo, materials[i].albedo, sizeof(float) * 3);
        mats[i].ty = materials[i].ty;
        for (int c = 0; c < 3; c++) mats[i].alb_pi[c] = materials[i].albedo[c] / 3.1415926f;
        mats[i].pad = 0;
    }
    std::vector<FaceShade> shade(n_faces);
    for (uint32_t i = 0; i < n_faces; i++) {
        FaceShade &fs = shade[i];
        std::memset(&fs, 0, sizeof(fs));
        std::memcpy(fs.n0, vertices[faces[i].vertices[0]].normal, 12);
        std::memcpy(fs.n1, vertices[faces[i].vertices[1]].normal, 12);
        std::memcpy(fs.n2, vertices[faces[i].vertices[2]].normal, 12);
        fs.mat = faces[i].material_id;
        fs.ty = mats[fs.mat].ty;
        std::memcpy(fs.alb_pi, mats[fs.mat].alb_pi, 12);
    }
    // light table (sample_light_games101, :384-404) with the std140 id quirk (:109-111)
    const bool quirk = ctx->cfg.lum_id_std140_quirk != 0;
    std::vector<LightRecord> lights(n_lum_face_ids ? n_lum_face_ids : 1);
    float total = 0.0f;
    for (uint32_t i = 0; i < n_lum_face_ids; i++) {
        const uint32_t id = quirk ? ((4u * i < n_lum_face_ids) ? lum_face_ids[4u * i] : 0u)
                                  : lum_face_ids[i];
        total += face_area(vertices, faces[id]);
    }
    float run = 0.0f;
    for (uint32_t i = 0; i < n_lum_face_ids; i++) {
        const uint32_t id = quirk ? ((4u * i < n_lum_face_ids) ? lum_face_ids[4u * i] : 0u)
                                  : lum_face_ids[i];
        const rvcp_face_t &f = faces[id];
        run += face_area(vertices, f);
        LightRecord &L = lights[i];
        std::memset(&L, 0, sizeof(L));
        L.cum = run;
        L.face = id;
        std::memcpy(L.v0, vertices[f.vertices[0]].position, 12);
        std::memcpy(L.v1, vertices[f.vertices[1]].position, 12);
        std::memcpy(L.v2, vertices[f.vertices[2]].position, 12);
        st3(L.n, normalize(ld3(vertices[f.vertices[0]].normal)));
        std::memcpy(L.le, materials[f.material_id].albedo, 12);
    }

    free_scene(ctx);
    int rc;
    if ((rc = dev_upload<TriRecord>(ctx, &ctx->d_tri, tri.data(), n_faces)) ||
        (rc = dev_upload<rvcp_face_t>(ctx, &ctx->d_faces, faces, n_faces)) ||
        (rc = dev_upload<rvcp_vertex_t>(ctx, &ctx->d_verts, vertices, n_vertices)) ||
        (rc = dev_upload<MatRecord>(ctx, &ctx->d_mats, mats.data(), n_materials)) ||
        (rc = dev_upload<FaceShade>(ctx, &ctx->d_shade, shade.data(), n_faces)) ||
        (rc = dev_upload<LightRecord>(ctx, &ctx->d_lights, lights.data(), n_lum_face_ids)) ||
        (rc = dev_upload<rvcp_material_t>(ctx, &ctx->d_rawmats, materials, n_materials)) ||
        (rc = dev_upload<rvcp_sphere_t>(ctx, &ctx->d_spheres, spheres, n_spheres)))
        return rc;
    ctx->n_spheres = n_spheres;
    if (ctx->cfg.accel == RVCP_ACCEL_BVH && n_faces > 0) {
        std::vector<float> pos((size_t)n_faces * 9);
        for (uint32_t i = 0; i < n_faces; i++)
            for (int v = 0; v < 3; v++)
                std::memcpy(&pos[(size_t)i * 9 + 3 * v], vertices[faces[i].vertices[v]].position, 12);
        std::vector<BvhNode> nodes;
        std::vector<uint32_t> order;
        int32_t root = 0;
        const int depth = bvh_build(reinterpret_cast<const float (*)[3][3]>(pos.data()), n_faces,
                                    nodes, order, root);
        if (depth >= kBvhStack) return fail(ctx, RVCP_E_UNSUPPORTED, "BVH deeper than the traversal stack");
        std::vector<TriRecord> btri(order.size());
        for (size_t j = 0; j < order.size(); j++) {       // leaf order, face id in pad[0]
            btri[j] = tri[order[j]];
            std::memcpy(&btri[j].pad[0], &order[j], 4);
        }
        std::vector<Bvh4Node> nodes4;
        int32_t root4 = 0;
        if (bvh4_collapse(nodes, root, nodes4, root4) > kBvhStack)
            return fail(ctx, RVCP_E_UNSUPPORTED, "BVH traversal stack bound exceeded");
        if ((rc = dev_upload<Bvh4Node>(ctx, &ctx->d_bvh_nodes, nodes4.data(), nodes4.size())) ||
            (rc = dev_upload<TriRecord>(ctx, &ctx->d_bvh_tris, btri.data(), btri.size())))
            return rc;
        ctx->bvh_root = root4;
        ctx->bvh_depth = depth;
    }
    ctx->n_faces = n_faces;
    ctx->n_verts = n_vertices;
    ctx->n_mats = n_materials;
    ctx->n_lights = n_lum_face_ids;
    ctx->light_total = total;
    ctx->light_pdf = 1.0f / total;
    ctx->has_scene = true;
    return RVCP_OK;
}

int rvcp_upload_scene_file(rvcp_ctx_t *ctx, const char *path, rvcp_camera_t *out_camera)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!path) return fail(ctx, RVCP_E_INVALID, "null path");
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(ctx, RVCP_E_INVALID, std::string("cannot open scene file ") + path);
    std::vector<unsigned char> data;
    unsigned char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) data.insert(data.end(), buf, buf + got);
    const bool read_error = std::ferror(f) != 0;
    std::fclose(f);
    if (read_error) return fail(ctx, RVCP_E_INVALID, "error reading scene file");
    constexpr size_t kHeader = 128;
    if (data.size() < kHeader || std::memcmp(data.data(), "RVCPSCN1", 8) != 0)
        return fail(ctx, RVCP_E_INVALID, "not an RVCPSCN1 scene file");
    uint32_t version, header_bytes;
    rvcp_lengths_t L;
    std::memcpy(&version, data.data() + 8, 4);
    std::memcpy(&header_bytes, data.data() + 12, 4);
    std::memcpy(&L, data.data() + 16, sizeof(L));
    if (version != 1 || header_bytes != kHeader)
        return fail(ctx, RVCP_E_INVALID, "unsupported scene file version");
    const uint64_t need = kHeader + 32ull * L.materials_len + 32ull * L.spheres_len +
                          32ull * L.vertices_len + 16ull * L.faces_len +
                          4ull * L.luminous_sphere_id_len + 4ull * L.luminous_face_id_len;
    if (need != data.size())
        return fail(ctx, RVCP_E_INVALID, "scene file size does not match its lengths");
    // copy each array into storage of its own type (the byte buffer has no alignment promise)
    size_t off = kHeader;
    auto take = [&](auto &vec, uint32_t n) {
        vec.resize(n);
        if (n) std::memcpy(vec.data(), data.data() + off, n * sizeof(vec[0]));
        off += (size_t)n * sizeof(vec[0]);
    };
    std::vector<rvcp_material_t> mats;
    std::vector<rvcp_sphere_t> sph;
    std::vector<rvcp_vertex_t> verts;
    std::vector<rvcp_face_t> faces;
    std::vector<uint32_t> lsph, lface;
    take(mats, L.materials_len);
    take(sph, L.spheres_len);
    take(verts, L.vertices_len);
    take(faces, L.faces_len);
    take(lsph, L.luminous_sphere_id_len);
    take(lface, L.luminous_face_id_len);
    const int rc = rvcp_upload_scene(ctx, mats.data(), L.materials_len, verts.data(),
                                     L.vertices_len, faces.data(), L.faces_len, sph.data(),
                                     L.spheres_len, lface.data(), L.luminous_face_id_len,
                                     lsph.data(), L.luminous_sphere_id_len);
    if (rc == RVCP_OK && out_camera) std::memcpy(out_camera, data.data() + 40, sizeof(*out_camera));
    return rc;
}

uint32_t rvcp_shard_rows(uint32_t height, uint32_t shard_index, uint32_t shard_count)
{
    if (shard_count == 0 || shard_index >= shard_count) return 0;
    const uint32_t stripes = (height + 7) / 8;
    uint32_t rows = 0;
    for (uint32_t s = shard_index; s < stripes; s += shard_count)
        rows += (s + 1) * 8 <= height ? 8 : height - s * 8;
    return rows;
}

int rvcp_render_shard_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                            uint32_t height, uint32_t shard_index, uint32_t shard_count,
                            void *d_rgba8, void *d_linear_rgb, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!push || !d_rgba8 || width == 0 || height == 0 || shard_count == 0 ||
        shard_index >= shard_count)
        return fail(ctx, RVCP_E_INVALID, "invalid render arguments");
    if ((uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "frame too large (W*H must be < 2^31)");
    if (!ctx->has_scene) return fail(ctx, RVCP_E_NO_SCENE, "render before rvcp_upload_scene");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;

    const uint32_t rows = rvcp_shard_rows(height, shard_index, shard_count);
    FrameArgs A;
    std::memset(&A, 0, sizeof(A));
    camera_constants(*push, width, height, A);
    A.width = width;
    A.height = height;
    A.shard_index = shard_index;
    A.shard_count = shard_count;
    A.n_pixels = rows * width;
    A.spp = ctx->cfg.spp;
    A.max_bounces = ctx->cfg.max_bounces;
    A.att_stop = ctx->cfg.attenuation_stop_eps;
    A.t_min = ctx->cfg.ray_t_min;
    A.t_max = ctx->cfg.ray_t_max;
    A.rr = ctx->cfg.rr_probability;
    A.eps = ctx->cfg.eps;
    A.n_faces = ctx->n_faces;
    A.n_lights = ctx->n_lights;
    A.light_total = ctx->light_total;
    A.light_pdf = ctx->light_pdf;
    A.want_linear = d_linear_rgb ? 1u : 0u;
    A.variant = ctx->cfg.kernel_variant != 0 ? ctx->cfg.kernel_variant
              : ctx->n_faces >= kTiledMinFaces ? 5
              : (uint64_t)A.n_pixels * A.spp >= kWideMinSamples ? 6 : kDefaultVariant;
    A.accel = (ctx->cfg.accel == RVCP_ACCEL_BVH && ctx->n_faces > 0) ? RVCP_ACCEL_BVH : RVCP_ACCEL_NONE;
    if (A.accel == RVCP_ACCEL_BVH) A.variant = 3;    // the BVH traversal lives in the v3 kernels
    A.bvh_root = ctx->bvh_root;
    const bool legacy = ctx->cfg.integrator == RVCP_INTEGRATOR_LEGACY;
    A.n_spheres = legacy ? ctx->n_spheres : 0u;

    // With MAX_BOUNCES == 0 or ATTENUATION_STOP_EPS > 1 every sample returns 0 before its
    // first traversal (:413-419): the frame is black.  ray_tracer.comp has no attenuation
    // test before its first traversal (:629-634).
    const bool trivial = A.max_bounces == 0 || (!legacy && 1.0f < A.att_stop);
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, 4 * sizeof(unsigned long long), s));
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, s));
    if (A.n_pixels > 0) {
        int rc;
        if (trivial) {
            HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
            rc = rvcp_launch_fill((uint32_t *)d_rgba8, (float *)d_linear_rgb, A.n_pixels,
                                  0xFF000000u, s);
        } else {
            const uint32_t cap = (uint32_t)(legacy ? ctx->legacy_capacity
                                           : A.accel ? ctx->bvh_capacity
                                                     : ctx->grid_capacity[A.variant]);
            A.n_simds = ctx->n_simds;
            uint32_t waves = 0, chunk = 0;
            rvcp_static_split(A.n_pixels, cap * (kBlock / kWave), A.n_simds, &waves, &chunk);
            uint32_t blocks = (waves + (kBlock / kWave) - 1) / (kBlock / kWave);
            if (blocks > cap) blocks = cap;
            if (blocks == 0) blocks = 1;
            A.static_chunk = chunk;
            A.static_chunks = waves * chunk;
            A.dyn_chunk = kDynChunk;
            A.chunk_min = kMinChunk;
            A.chunk_window = kChunkWindow;
            if (const char *c = std::getenv("RVCP_DEBUG_CHUNK")) {   // fixed grab (experiments)
                const int v = std::atoi(c);
                if (v >= 1 && v <= 4096) A.dyn_chunk = A.chunk_min = (uint32_t)v;
            }
            if (const char *c = std::getenv("RVCP_DEBUG_CHUNK_WINDOW")) {
                const int v = std::atoi(c);
                if (v >= 1) A.chunk_window = (uint32_t)v;
            }
            ctx->last_timeline_waves = 0;
            if (std::getenv("RVCP_DEBUG_TIMELINE") && !legacy && A.variant >= 3) {
                const size_t waves = (size_t)blocks * (kBlock / kWave);
                if (ctx->cap_timeline < waves) {
                    (void)hipFree(ctx->d_timeline);
                    ctx->d_timeline = nullptr;
                    ctx->cap_timeline = 0;
                    HIP_TRY(ctx, hipMalloc((void **)&ctx->d_timeline, waves * 32));
                    ctx->cap_timeline = waves;
                }
                A.timeline = ctx->d_timeline;
                ctx->last_timeline_waves = waves;
            }
            if (legacy) {
                HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
                rc = rvcp_launch_legacy(&A, ctx->d_tri, ctx->d_shade, ctx->d_spheres,
                                        ctx->d_rawmats, ctx->d_unorm, (uint32_t *)d_rgba8,
                                        (float *)d_linear_rgb, ctx->d_counters, blocks, s);
            } else if (A.variant >= 3) {
                if (ctx->cap_surf < A.n_pixels) {
                    (void)hipFree(ctx->d_surf);
                    ctx->d_surf = nullptr;
                    ctx->cap_surf = 0;
                    HIP_TRY(ctx, hipMalloc((void **)&ctx->d_surf, (size_t)A.n_pixels * sizeof(SurfRecord)));
                    ctx->cap_surf = A.n_pixels;
                }
                rc = rvcp_launch_games101_v3(&A, ctx->d_tri, ctx->d_faces, ctx->d_verts,
                                             ctx->d_mats, ctx->d_lights, ctx->d_gamma,
                                             (uint32_t *)d_rgba8, (float *)d_linear_rgb,
                                             ctx->d_counters, ctx->d_surf, ctx->d_shade,
                                             ctx->d_bvh_nodes, ctx->d_bvh_tris,
                                             blocks, s, ctx->evm);
            } else {
                HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
                rc = rvcp_launch_games101(&A, ctx->d_tri, ctx->d_faces, ctx->d_verts, ctx->d_mats,
                                          ctx->d_lights, ctx->d_gamma, (uint32_t *)d_rgba8,
                                          (float *)d_linear_rgb, ctx->d_counters, blocks, s);
            }
        }
        if (rc != 0) return fail(ctx, RVCP_E_HIP, std::string("kernel launch failed: ") +
                                                      hipGetErrorString(hipGetLastError()));
    } else {
        HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, s));
    ctx->pending = true;
    ctx->last_trivial = trivial;
    ctx->last_pixels = A.n_pixels;
    ctx->last_spp = A.spp;
    return RVCP_OK;
}

int rvcp_render_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                      uint32_t height, void *d_rgba8, void *d_linear_rgb, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->subs.empty())
        return fail(ctx, RVCP_E_UNSUPPORTED, "rvcp_render_async drives one GPU; use rvcp_render for n_gpus > 1");
    return rvcp_render_shard_async(ctx, push, width, height, 0, 1, d_rgba8, d_linear_rgb, stream);
}

int rvcp_wait(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    return rvcp_sync_stats(ctx, stats);
}

int rvcp_sync_stats(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->pending) return fail(ctx, RVCP_E_INVALID, "no render in flight");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev1));
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        unsigned long long c[4] = {0, 0, 0, 0};
        HIP_TRY(ctx, hipMemcpy(c, ctx->d_counters, sizeof(c), hipMemcpyDeviceToHost));
        stats->kernel_ms = ms;
        float ms_main = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms_main, ctx->evm, ctx->ev1));
        stats->main_kernel_ms = ms_main;
        stats->traversals_executed = c[0];
        // the reference re-traces the (RNG-independent) primary ray in every sample
        stats->traversals = ctx->last_trivial ? 0 : c[0] + ctx->last_pixels * (ctx->last_spp - 1);
        stats->samples = ctx->last_pixels * ctx->last_spp;
        stats->faces = ctx->n_faces;
        stats->wave_iterations = c[2];
    }
    if (ctx->last_timeline_waves) {
        std::vector<unsigned long long> t(4 * ctx->last_timeline_waves);
        HIP_TRY(ctx, hipMemcpy(t.data(), ctx->d_timeline, t.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = std::fopen(std::getenv("RVCP_DEBUG_TIMELINE"), "ab")) {
            std::fwrite(t.data(), 8, t.size(), f);
            std::fclose(f);
        }
        ctx->last_timeline_waves = 0;
    }
    ctx->pending = false;           // a render is waited for once
    return RVCP_OK;
}

// n_gpus > 1: every GPU renders its stripes packed (shard k of N on GPU k), then each shard
// is copied into the frame on ctx->device with one strided copy (stripe j of shard k ->
// frame rows 8(jN + k) .. +8), over xGMI when the GPUs differ.  Stats are summed over shards;
// kernel_ms is the slowest shard's.
static int render_multi(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t W,
                        uint32_t H, bool want_lin, rvcp_stats_t *stats)
{
    const uint32_t N = (uint32_t)ctx->subs.size() + 1;
    int rc;
    // 1. launch every shard (shard 0 renders on ctx itself, into a packed buffer of its own)
    for (uint32_t k = 0; k < N; k++) {
        rvcp_ctx *c = k == 0 ? ctx : ctx->subs[k - 1];
        const size_t rows = rvcp_shard_rows(H, k, N), px = rows * W;
        if (k > 0 && (ctx->shard_cap[k - 1] < px || (want_lin && !ctx->shard_lin[k - 1]))) {
            HIP_TRY(ctx, hipSetDevice(c->device));
            (void)hipFree(ctx->shard_rgba[k - 1]);
            (void)hipFree(ctx->shard_lin[k - 1]);
            ctx->shard_rgba[k - 1] = nullptr;
            ctx->shard_lin[k - 1] = nullptr;
            ctx->shard_cap[k - 1] = 0;
            HIP_TRY(ctx, hipMalloc((void **)&ctx->shard_rgba[k - 1], px * 4 + 4));
            HIP_TRY(ctx, hipMalloc((void **)&ctx->shard_lin[k - 1], px * 12 + 12));
            ctx->shard_cap[k - 1] = px;
        }
    }
    // shard 0 needs its own packed buffer too: reuse the staging's tail is not possible, so
    // keep it in shard_rgba[-1] semantics via a dedicated allocation on ctx
    const size_t px0 = (size_t)rvcp_shard_rows(H, 0, N) * W;
    if (ctx->cap_surf_pack < px0 || (want_lin && !ctx->d_pack_lin)) {
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        (void)hipFree(ctx->d_pack_rgba);
        (void)hipFree(ctx->d_pack_lin);
        ctx->d_pack_rgba = nullptr;
        ctx->d_pack_lin = nullptr;
        ctx->cap_surf_pack = 0;
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_pack_rgba, px0 * 4 + 4));
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_pack_lin, px0 * 12 + 12));
        ctx->cap_surf_pack = px0;
    }
    for (uint32_t k = 0; k < N; k++) {
        rvcp_ctx *c = k == 0 ? ctx : ctx->subs[k - 1];
        uint32_t *d_rgba = k == 0 ? ctx->d_pack_rgba : ctx->shard_rgba[k - 1];
        float *d_lin = want_lin ? (k == 0 ? ctx->d_pack_lin : ctx->shard_lin[k - 1]) : nullptr;
        if ((rc = rvcp_render_shard_async(c, push, W, H, k, N, d_rgba, d_lin, c->stream)) != RVCP_OK) {
            if (k > 0) ctx->err = "shard " + std::to_string(k) + ": " + c->err;
            (void)hipSetDevice(ctx->device);
            return rc;
        }
    }
    // 2. wait for each shard and copy its stripes into the frame on ctx->device
    rvcp_stats_t total;
    std::memset(&total, 0, sizeof(total));
    for (uint32_t k = 0; k < N; k++) {
        rvcp_ctx *c = k == 0 ? ctx : ctx->subs[k - 1];
        rvcp_stats_t st;
        if ((rc = rvcp_sync_stats(c, &st)) != RVCP_OK) {
            if (k > 0) ctx->err = "shard " + std::to_string(k) + ": " + c->err;
            (void)hipSetDevice(ctx->device);
            return rc;
        }
        total.kernel_ms = st.kernel_ms > total.kernel_ms ? st.kernel_ms : total.kernel_ms;
        total.main_kernel_ms = st.main_kernel_ms > total.main_kernel_ms ? st.main_kernel_ms : total.main_kernel_ms;
        total.traversals += st.traversals;
        total.traversals_executed += st.traversals_executed;
        total.samples += st.samples;
        total.wave_iterations += st.wave_iterations;
        total.faces = st.faces;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        const uint32_t stripes = (H + 7) / 8;
        const uint32_t full = H / 8;                       // stripes with 8 rows
        uint32_t n_full = 0;                               // full stripes of shard k
        for (uint32_t s = k; s < full; s += N) n_full++;
        const uint8_t *src = (const uint8_t *)(k == 0 ? ctx->d_pack_rgba : ctx->shard_rgba[k - 1]);
        const float *srcl = k == 0 ? ctx->d_pack_lin : ctx->shard_lin[k - 1];
        for (int pass = 0; pass < (want_lin ? 2 : 1); pass++) {
            const size_t bpp = pass == 0 ? 4 : 12;
            const uint8_t *sp = pass == 0 ? src : (const uint8_t *)srcl;
            uint8_t *dp = pass == 0 ? (uint8_t *)ctx->d_rgba : (uint8_t *)ctx->d_lin;
            if (n_full)
                HIP_TRY(ctx, hipMemcpy2DAsync(dp + (size_t)8 * k * W * bpp, (size_t)8 * N * W * bpp,
                                              sp, (size_t)8 * W * bpp, (size_t)8 * W * bpp, n_full,
                                              hipMemcpyDefault, ctx->stream));
            // a last, partial stripe (H % 8 rows), if it is shard k's
            if (full < stripes && (full % N) == k) {
                const size_t rows = H - 8 * full;
                HIP_TRY(ctx, hipMemcpyAsync(dp + (size_t)8 * full * W * bpp,
                                            sp + (size_t)8 * n_full * W * bpp, rows * W * bpp,
                                            hipMemcpyDefault, ctx->stream));
            }
        }
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (stats) *stats = total;
    return RVCP_OK;
}

int rvcp_render(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                uint32_t height, uint8_t *out_rgba8, float *out_linear_rgb, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!out_rgba8) return fail(ctx, RVCP_E_INVALID, "out_rgba8 is required");
    if (width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "invalid frame size");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t npx = (size_t)width * height;
    if (ctx->cap_rgba < npx) {
        (void)hipFree(ctx->d_rgba);
        ctx->d_rgba = nullptr;
        ctx->cap_rgba = 0;
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_rgba, npx * 4));
        ctx->cap_rgba = npx;
    }
    if (out_linear_rgb && ctx->cap_lin < npx) {
        (void)hipFree(ctx->d_lin);
        ctx->d_lin = nullptr;
        ctx->cap_lin = 0;
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_lin, npx * 12));
        ctx->cap_lin = npx;
    }
    int rc;
    if (ctx->subs.empty()) {
        rc = rvcp_render_shard_async(ctx, push, width, height, 0, 1, ctx->d_rgba,
                                     out_linear_rgb ? ctx->d_lin : nullptr, ctx->stream);
        if (rc != RVCP_OK) return rc;
        if ((rc = rvcp_sync_stats(ctx, stats)) != RVCP_OK) return rc;
    } else if ((rc = render_multi(ctx, push, width, height, out_linear_rgb != nullptr, stats)) != RVCP_OK) {
        return rc;
    }
    HIP_TRY(ctx, hipMemcpy(out_rgba8, ctx->d_rgba, npx * 4, hipMemcpyDeviceToHost));
    if (out_linear_rgb) HIP_TRY(ctx, hipMemcpy(out_linear_rgb, ctx->d_lin, npx * 12, hipMemcpyDeviceToHost));
    return RVCP_OK;
}

int rvcp_mandelbrot(rvcp_ctx_t *ctx, const rvcp_mandelbrot_push_t *push, uint32_t width,
                    uint32_t height, uint8_t *out_rgba8, float *out_value, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!push || !out_rgba8 || width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "invalid mandelbrot arguments");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t npx = (size_t)width * height;
    if (ctx->cap_rgba < npx) {
        (void)hipFree(ctx->d_rgba);
        ctx->d_rgba = nullptr;
        ctx->cap_rgba = 0;
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_rgba, npx * 4));
        ctx->cap_rgba = npx;
    }
    // the float escape values reuse the linear-RGB staging buffer (npx floats <= 3 npx)
    if (out_value && ctx->cap_lin < npx) {
        (void)hipFree(ctx->d_lin);
        ctx->d_lin = nullptr;
        ctx->cap_lin = 0;
        HIP_TRY(ctx, hipMalloc((void **)&ctx->d_lin, npx * 12));
        ctx->cap_lin = npx;
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    if (rvcp_launch_mandelbrot(push->position[0], push->position[1], push->scale, width, height,
                               ctx->d_unorm, ctx->d_rgba, out_value ? ctx->d_lin : nullptr,
                               ctx->stream) != 0)
        return fail(ctx, RVCP_E_HIP, "mandelbrot launch failed");
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev1));
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        stats->kernel_ms = ms;
        stats->main_kernel_ms = ms;
    }
    HIP_TRY(ctx, hipMemcpy(out_rgba8, ctx->d_rgba, npx * 4, hipMemcpyDeviceToHost));
    if (out_value) HIP_TRY(ctx, hipMemcpy(out_value, ctx->d_lin, npx * 4, hipMemcpyDeviceToHost));
    return RVCP_OK;
}

int rvcp_assemble_frame_async(rvcp_ctx_t *ctx, const void *d_gathered, uint32_t slot_rows,
                              uint32_t width, uint32_t height, uint32_t shard_count,
                              void *d_frame, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!d_gathered || !d_frame || width == 0 || height == 0 || shard_count == 0)
        return fail(ctx, RVCP_E_INVALID, "invalid assemble arguments");
    for (uint32_t k = 0; k < shard_count; k++)
        if (rvcp_shard_rows(height, k, shard_count) > slot_rows)
            return fail(ctx, RVCP_E_INVALID, "slot_rows smaller than a shard");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    if (rvcp_launch_assemble((const uint32_t *)d_gathered, slot_rows, width, height, shard_count,
                             (uint32_t *)d_frame, s) != 0)
        return fail(ctx, RVCP_E_HIP, "assemble launch failed");
    return RVCP_OK;
}

}  // extern "C"
