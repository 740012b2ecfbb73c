// rvcp_host.cpp -- C-ABI host runtime of librvcp (include/rvcp.h).
//
// Replaces the Vulkano runtime of the reference (src/ray_tracer/vulkan.rs): pipeline
// creation (:576-603) -> rvcp_create, descriptor-set upload (:454-574) -> rvcp_upload_scene,
// push constants + dispatch (:406-452) -> rvcp_render / rvcp_render_shard_async.
//
// Compiled with hipcc -ffp-contract=off: the frame constants it derives (camera basis,
// light-area prefix sums, gamma thresholds) use the same float operations as the shader, so
// the kernel's results stay bit-identical to the CPU oracle.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <exception>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rvcp.h"
#include "rvcp_internal.h"
#include "rvcp_jit.h"
#include "rvcp_scene_prep.h"
#include "build/rvcp_build_id.h"     // kRvcpSourceHash (Makefile)

using namespace rvcp;

// Experiment knobs (grid caps, fixed queue grabs, small-frame spreading, per-wave timelines,
// generic-scan forcing) are read from the environment only in the debug build of the library
// (make debug -> build/librvcp_debug.so, -DRVCP_DEBUG_KNOBS, used by tools/).  The product
// library's behaviour depends on rvcp_config_t alone: here the names are not even compiled in.
#ifdef RVCP_DEBUG_KNOBS
#define RVCP_KNOB(name) std::getenv(name)
#else
#define RVCP_KNOB(name) ((const char *)nullptr)
#endif

// The specialised pre-pass (rvcp_spec_primary_kernel) with the specialised path kernels; the
// debug build's RVCP_DEBUG_GENERIC_PREPASS=1 keeps the built-in one (A/B)
static bool jit_spec_prepass()
{
    const char *e = RVCP_KNOB("RVCP_DEBUG_GENERIC_PREPASS");
    return !(e && *e == '1');
}

// rvcp_rccl_init / rvcp_gather_wait give up after this long unless rvcp_rccl_set_timeout says
// otherwise: far above a frame (C5 brute force, the slowest workload, 6.5 s) and far below
// "forever", which is what a blocking ncclCommInitRank or an unbounded event wait gives when a
// peer never arrives
constexpr uint32_t kDefaultCommTimeoutMs = 60000;


struct rvcp_ctx {
    rvcp_config_t cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, evm = nullptr, ev1 = nullptr;   // start, main kernel, end
    hipEvent_t evg0 = nullptr, evg1 = nullptr;                // gather start / end
    // rvcp_gather_frame_async without a caller stream runs on gstream (high priority), joined
    // to the render stream by events: evr (render done) before the gather, evg1 (gather done)
    // before the next render on this context overwrites the shard buffer the gather reads
    hipStream_t gstream = nullptr;
    hipStream_t render_stream = nullptr;     // the stream of the last render (the caller's or ours)
    hipEvent_t evr = nullptr;
    bool gather_on_gstream = false;
    bool gather_pending = false;
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
    uint32_t bvh_n4 = 0;
    uint32_t bvh_slots = 0;
    int bvh_depth = 0;
    uint32_t bvh_prefix = 0;    // faces [0, bvh_prefix) left out of the BVH (FrameArgs::bvh_prefix)
    float *d_gamma = nullptr;
    float *d_unorm = nullptr;
    unsigned long long *d_counters = nullptr;
    uint32_t n_faces = 0, n_lights = 0, n_mats = 0, n_verts = 0, n_spheres = 0;
    bool lights_same = false;      // every light record samples the same face
    bool rcp_fast = false;         // scan_rcp_fast_scene (FrameArgs::rcp_fast)
    bool has_metal = false;        // a material of type 1 (FrameArgs::has_metal)
    // scene-specialised path kernels (rvcp_jit.cpp), or null: generic kernels
    std::shared_ptr<JitKernels> jit;
    std::string jit_err;
    float light_total = 0.0f, light_pdf = 0.0f;
    bool has_scene = false;

    // primary pre-pass output (variant 3): compact list of surface pixels
    SurfRecord *d_surf = nullptr;
    size_t cap_surf = 0;
    float *d_acc = nullptr;         // linear colours for tonemap_kernel when the caller wants none
    size_t cap_acc = 0;
    // mode-2 batches: the frames' FrameCam records (16 floats each), staged through pinned
    // host memory (one render in flight per context, so the staging is free again at the next)
    float *d_cams = nullptr, *h_cams = nullptr;
    uint32_t cap_cams = 0;

    // staging for the synchronous host API
    uint32_t *d_rgba = nullptr;
    float *d_lin = nullptr;
    size_t cap_rgba = 0, cap_lin = 0;
    // n_gpus > 1: shard 0's packed stripes
    uint32_t *d_pack_rgba = nullptr;
    float *d_pack_lin = nullptr;
    size_t cap_surf_pack = 0;

    // debug build: per-wave timeline of the path kernel appended per render
    unsigned long long *d_timeline = nullptr;
    size_t cap_timeline = 0, last_timeline_waves = 0;

    // n_gpus > 1: contexts of the other GPUs (shards 1..N-1) and their packed shard buffers
    std::vector<rvcp_ctx *> subs;
    std::vector<uint32_t *> shard_rgba;
    std::vector<float *> shard_lin;
    std::vector<size_t> shard_cap;

    // one process per GPU: the RCCL communicator of rvcp_gather_frame_async (rank `comm_rank`
    // of `comm_world`; created by rvcp_rccl_init, or the caller's by rvcp_rccl_attach)
    ncclComm_t comm = nullptr;
    bool comm_owned = false;
    uint32_t comm_world = 0, comm_rank = 0;
    // deadline of rvcp_rccl_init and rvcp_gather_wait (rvcp_rccl_set_timeout; 0 = none)
    uint32_t comm_timeout_ms = kDefaultCommTimeoutMs;
    // the last communicator was given up after a deadline: gathers return RVCP_E_TIMEOUT (not
    // "no communicator") until rvcp_rccl_init / rvcp_rccl_attach provides a new one
    bool comm_timed_out = false;
    // the creation worker of an rvcp_rccl_init that timed out, while it is still blocked inside
    // RCCL: a further rvcp_rccl_init on this context is refused (RVCP_E_BUSY) until it returns,
    // so retries cannot pile up blocked threads and half-made communicators
    std::shared_ptr<struct CommJob> init_job;
    // detached ncclCommAbort calls of this context's communicators (abort_comm): rvcp_destroy
    // waits for them (bounded) before it frees the buffers and streams their kernels used
    std::vector<std::shared_ptr<std::atomic<bool>>> aborts;
    // end events of gathers that timed out and whose stream did not drain (a collective on an
    // attached communicator, which only its owner can abort): renders no longer wait for them,
    // the gather stream they sit on is retired, and rvcp_destroy checks them before freeing
    // device memory (HIP's hipFree synchronises the whole device)
    std::vector<hipEvent_t> stuck_gathers;
    std::vector<hipStream_t> retired_gstreams;

    // last launch
    bool pending = false;
    bool last_trivial = false;
    bool last_spec = false;
    int32_t last_variant = 0;
    uint64_t last_pixels = 0;
    uint32_t last_spp = 0;
    uint32_t last_shard_index = 0, last_shard_count = 0;   // of the last rvcp_render_shard_async
    uint32_t last_width = 0, last_height = 0;

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

// RCCL, resolved at run time: dlopen("librccl.so.1") returns the copy the process already
// holds (PyTorch-ROCm's, soname librccl.so.1, or the host's own) and otherwise the system one,
// so librvcp needs no RCCL to load and shares one RCCL with its host.
struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    // non-blocking creation, abort and the communicator's asynchronous state: what makes a
    // missing or failed peer a timeout instead of a hang (rccl.h: ncclCommInitRankConfig,
    // ncclCommAbort, ncclCommGetAsyncError; present in every RCCL >= 2.14)
    ncclResult_t (*comm_init_rank_config)(ncclComm_t *, int, ncclUniqueId, int, ncclConfig_t *) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
    std::string why;
};

const RcclApi &rccl_api()
{
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char *e = dlerror();
            api.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
        api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
        api.comm_init_rank_config = (decltype(api.comm_init_rank_config))dlsym(h, "ncclCommInitRankConfig");
        api.comm_abort = (decltype(api.comm_abort))dlsym(h, "ncclCommAbort");
        api.get_async_error = (decltype(api.get_async_error))dlsym(h, "ncclCommGetAsyncError");
        api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
        api.gather = (decltype(api.gather))dlsym(h, "ncclGather");
        api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
        api.ok = api.get_unique_id && api.comm_init_rank && api.comm_init_rank_config &&
                 api.comm_abort && api.get_async_error && api.comm_destroy && api.gather &&
                 api.error_string;
        if (!api.ok)
            api.why = "librccl.so.1 lacks ncclGather / ncclCommInitRankConfig / ncclCommAbort / "
                      "ncclCommGetAsyncError";
    });
    return api;
}

// Report an error without allocating on the failure path that may itself be out of memory.
int fail_noexcept(rvcp_ctx *ctx, int code, const char *msg) noexcept
{
    try {
        if (ctx) ctx->err = msg;
        else g_create_error = msg;
    } catch (...) {
    }
    return code;
}

template <typename F>
int barrier(rvcp_ctx *ctx, F &&f) noexcept
{
    try {
        return f();
    } catch (const std::bad_alloc &) {
        return fail_noexcept(ctx, RVCP_E_NOMEM, "out of host memory");
    } catch (const std::exception &e) {
        return fail_noexcept(ctx, RVCP_E_INTERNAL, e.what());
    } catch (...) {
        return fail_noexcept(ctx, RVCP_E_INTERNAL, "unknown C++ exception");
    }
}

#define HIP_TRY(ctx, expr)                                                                  \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((ctx), RVCP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// sample_ray's frame constants, :217-227
void camera_constants(const rvcp_push_constant_t &pc, uint32_t W, uint32_t H, FrameArgs &A)
{
    const float PI = 3.1415926f;
    h3 cpos = ld3h(pc.camera.position), up = ld3h(pc.camera.up), fwd = ld3h(pc.camera.forward);
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

// The primary ray's range is [t_near, t_far] x t_coef (sample_ray, :226-233), and a miss is
// written as t_max + 1 (:287) and detected as t > t_max (:424): once t_max reaches 2^24 the +1
// is lost and the shader takes a miss for a hit on uninitialised data.  The kernels detect a
// miss by the absent face instead, so such a frame would differ from the reference's; it is
// refused, as rvcp_config_t.ray_t_max >= 2^24 is for the secondary rays.  t_coef is at most
// |corner of the image plane - eye| / t_near = sqrt(1 + tan^2(fov / 2) (1 + (W / H)^2))
// (u, v, forward orthogonal); a 1e-3 margin covers the float rounding of the shader's t_coef.
bool primary_t_range_ok(const rvcp_push_constant_t &pc, uint32_t W, uint32_t H)
{
    const double tf = pc.camera.t_far;
    const double t = std::tan((double)pc.camera.vertical_fov / 2.0 * 3.1415926 / 180.0);
    const double a = (double)W / (double)H;
    const double tc = std::sqrt(1.0 + t * t * (1.0 + a * a));
    return std::fabs(tf) * tc * (1.0 + 1e-3) < 16777216.0;
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
    ctx->jit.reset();
    ctx->has_scene = false;
}

}  // namespace

using Clock = std::chrono::steady_clock;
static void abort_comm(rvcp_ctx_t *ctx);
static int wait_gather_done(rvcp_ctx_t *ctx);

extern "C" {

// 0.2.0: ABI revision 2 (rvcp.h RVCP_ABI_VERSION: rvcp_stats_t is 64 B)
const char *rvcp_version(void) { return "rvcp-mi355x 0.2.0 (gfx950, ABI 2)"; }

uint32_t rvcp_abi_version(void) { return RVCP_ABI_VERSION; }

// Self-test / measurement hooks (not part of rvcp.h): the library's source identity (SHA-256
// prefix of every source it is built from, "+debug" for the knob build) and the key of the
// scene-specialised module ctx's last upload built (0: none) -- bench.py binds the committed
// PMC summaries to both.
const char *rvcp_internal_build_id(void)
{
#ifdef RVCP_DEBUG_KNOBS
    static const std::string id = std::string(kRvcpSourceHash) + "+debug";
    return id.c_str();
#else
    return kRvcpSourceHash;
#endif
}

uint64_t rvcp_internal_module_key(const rvcp_ctx_t *ctx)
{
    return (ctx && ctx->jit) ? ctx->jit->key_hash : 0;
}

static int impl_config_default_for(int32_t integrator, rvcp_config_t *cfg)
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

static int impl_config_default(rvcp_config_t *cfg)
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

static int impl_create(const rvcp_config_t *cfg, rvcp_ctx_t **out_ctx)
{
    if (!cfg || !out_ctx) return fail(nullptr, RVCP_E_INVALID, "null argument");
    *out_ctx = nullptr;
    if (cfg->integrator != RVCP_INTEGRATOR_GAMES101 && cfg->integrator != RVCP_INTEGRATOR_LEGACY)
        return fail(nullptr, RVCP_E_UNSUPPORTED, "unsupported integrator");
    if (cfg->spp == 0) return fail(nullptr, RVCP_E_INVALID, "spp must be > 0");
    if (cfg->kernel_variant < 0 || cfg->kernel_variant > kMaxVariant || cfg->kernel_variant == 7 ||
        cfg->kernel_variant == 8 || cfg->kernel_variant == 9)
        return fail(nullptr, RVCP_E_INVALID, "unknown kernel_variant");
    if (cfg->n_gpus < 0 || cfg->n_gpus > 64)
        return fail(nullptr, RVCP_E_INVALID, "n_gpus must be in [0, 64]");
    if (cfg->specialize != RVCP_SPECIALIZE_AUTO && cfg->specialize != RVCP_SPECIALIZE_OFF)
        return fail(nullptr, RVCP_E_INVALID, "unknown specialize");
    if (cfg->unorm_rule != RVCP_UNORM_DRIVER && cfg->unorm_rule != RVCP_UNORM_NEAREST)
        return fail(nullptr, RVCP_E_INVALID, "unknown unorm_rule");
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
    try {
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
        hipEventCreate(&ctx->ev1) != hipSuccess || hipEventCreate(&ctx->evg0) != hipSuccess ||
        hipEventCreate(&ctx->evg1) != hipSuccess ||
        hipEventCreateWithFlags(&ctx->evr, hipEventDisableTiming) != hipSuccess)
        return bail(fail(ctx, RVCP_E_HIP, "stream/event creation failed"));
    // (the frame gather's own stream is created by the first gather that needs it: a context
    // that never gathers holds one stream, so the hardware queues -- GPU_MAX_HW_QUEUES, 4 by
    // default -- stay free for other contexts' render streams; frames in flight on contexts
    // whose streams shared a queue would run one after another)

    // UNORM8 thresholds on the stored value g: u8 >= k  <=>  g >= G[k].
    // RVCP_UNORM_DRIVER: u8 = (floor(4096 g) * 255 + 2048) >> 12, so G[k] = m_k / 4096 with
    // m_k = ceil((4096 k - 2048) / 255) (exact in float); RVCP_UNORM_NEAREST: G[k] = (k - 1/2) / 255.
    // Gamma thresholds on the linear colour: T[k] = float(G[k]^(1/0.6)) (pow(c, 0.6), :498).
    double G[256];
    for (int k = 1; k < 256; k++)
        G[k] = cfg->unorm_rule == RVCP_UNORM_NEAREST ? (k - 0.5) / 255.0
                                                     : std::ceil((4096.0 * k - 2048.0) / 255.0) / 4096.0;
    float T[257];
    T[0] = 0.0f;
    for (int k = 1; k < 256; k++) T[k] = (float)std::pow(G[k], 1.0 / 0.6);
    T[256] = INFINITY;
    if ((rc = dev_upload<float>(ctx, &ctx->d_gamma, T, 257)) != RVCP_OK) return bail(rc);
    // the gamma-free store of ray_tracer.comp:820-822 and mandelbrot.comp:32-33
    for (int k = 1; k < 256; k++) T[k] = (float)G[k];
    if ((rc = dev_upload<float>(ctx, &ctx->d_unorm, T, 257)) != RVCP_OK) return bail(rc);
    if (hipMalloc((void **)&ctx->d_counters, kCounterWords * sizeof(unsigned long long)) != hipSuccess)
        return bail(fail(ctx, RVCP_E_HIP, "hipMalloc counters"));

    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
        cus = 256;
    // debug build: cap on the persistent grid (occupancy experiments only)
    const char *cap_env = RVCP_KNOB("RVCP_DEBUG_BLOCKS_PER_CU");
    const int cap = cap_env ? std::atoi(cap_env) : 0;
    ctx->n_simds = (uint32_t)cus * 4u;
    for (int v = 1; v <= kMaxVariant; v++) {
        if (v == 7 || v == 8 || v == 9) continue;
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
    } catch (...) {     // the exception barrier reports it; free what was built
        rvcp_destroy(ctx);
        throw;
    }
    *out_ctx = ctx;
    return RVCP_OK;
}

static int impl_destroy(rvcp_ctx_t *ctx)
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
    // a frame still in flight (possibly on the caller's stream) reads the buffers freed below
    if (ctx->pending && ctx->ev1) (void)hipEventSynchronize(ctx->ev1);
    // (a gather still pending is waited for with the deadline: a peer that never came must not
    // hang the destroy; on expiry the communicator is aborted)
    if (ctx->gather_pending && ctx->evg1 && wait_gather_done(ctx) == RVCP_OK)
        ctx->gather_pending = false;
    if (ctx->gather_pending) abort_comm(ctx);
    // the detached aborts must have returned before their communicators' buffers and streams
    // go; and a gather that never drained still reads this context's buffers, while any hipFree
    // would wait for it (HIP synchronises the device): both bounded by the deadline
    const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(
        ctx->comm_timeout_ms ? std::min<uint32_t>(ctx->comm_timeout_ms, 10000u) : 10000u);
    bool stuck = false;
    for (;;) {
        stuck = false;
        for (const auto &a : ctx->aborts) stuck |= !a->load();
        for (hipEvent_t e : ctx->stuck_gathers) stuck |= hipEventQuery(e) == hipErrorNotReady;
        if (!stuck || Clock::now() >= deadline) break;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (stuck) {
        // leak the device side rather than hang: the streams, events, buffers and modules stay
        // allocated for the life of the process (the owner of the attached communicator can
        // still abort it); the host side is freed
        g_create_error = "rvcp_destroy: a gather (or its communicator's abort) is still stuck "
                         "after the deadline; the context's device memory and streams are leaked";
        new std::shared_ptr<JitKernels>(std::move(ctx->jit));   // never unloaded
        delete ctx;
        return RVCP_E_TIMEOUT;
    }
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm && ctx->comm_owned) (void)rccl_api().comm_destroy(ctx->comm);
    ctx->comm = nullptr;
    for (hipEvent_t e : ctx->stuck_gathers) (void)hipEventDestroy(e);
    for (hipStream_t s : ctx->retired_gstreams) (void)hipStreamDestroy(s);
    free_scene(ctx);
    (void)hipFree(ctx->d_gamma);
    (void)hipFree(ctx->d_unorm);
    (void)hipFree(ctx->d_counters);
    (void)hipFree(ctx->d_rgba);
    (void)hipFree(ctx->d_lin);
    (void)hipFree(ctx->d_surf);
    (void)hipFree(ctx->d_acc);
    (void)hipFree(ctx->d_cams);
    (void)hipHostFree(ctx->h_cams);
    (void)hipFree(ctx->d_timeline);
    (void)hipFree(ctx->d_pack_rgba);
    (void)hipFree(ctx->d_pack_lin);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->evm) (void)hipEventDestroy(ctx->evm);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->evg0) (void)hipEventDestroy(ctx->evg0);
    if (ctx->evg1) (void)hipEventDestroy(ctx->evg1);
    if (ctx->evr) (void)hipEventDestroy(ctx->evr);
    if (ctx->gstream) (void)hipStreamDestroy(ctx->gstream);
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

static int impl_upload_scene(rvcp_ctx_t *ctx, const rvcp_material_t *materials, uint32_t n_materials,
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
    if (ctx->pending)
        return fail(ctx, RVCP_E_INVALID, "a frame is in flight on this context (rvcp_wait first)");
    SceneInput in;
    in.materials = materials; in.n_materials = n_materials;
    in.vertices = vertices; in.n_vertices = n_vertices;
    in.faces = faces; in.n_faces = n_faces;
    in.spheres = spheres; in.n_spheres = n_spheres;
    in.lum_face_ids = lum_face_ids; in.n_lum_face_ids = n_lum_face_ids;
    SceneTables tab;
    std::string err;
    if (prepare_scene(in, ctx->cfg.lum_id_std140_quirk != 0, tab, err) != RVCP_OK)
        return fail(ctx, RVCP_E_INVALID, err);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const std::vector<TriRecord> &tri = tab.tri;
    const float total = tab.light_total;

    free_scene(ctx);
    int rc;
    if ((rc = dev_upload<TriRecord>(ctx, &ctx->d_tri, tri.data(), n_faces)) ||
        (rc = dev_upload<rvcp_face_t>(ctx, &ctx->d_faces, faces, n_faces)) ||
        (rc = dev_upload<rvcp_vertex_t>(ctx, &ctx->d_verts, vertices, n_vertices)) ||
        (rc = dev_upload<MatRecord>(ctx, &ctx->d_mats, tab.mats.data(), n_materials)) ||
        (rc = dev_upload<FaceShade>(ctx, &ctx->d_shade, tab.shade.data(), n_faces)) ||
        (rc = dev_upload<LightRecord>(ctx, &ctx->d_lights, tab.lights.data(), n_lum_face_ids)) ||
        (rc = dev_upload<rvcp_material_t>(ctx, &ctx->d_rawmats, materials, n_materials)) ||
        (rc = dev_upload<rvcp_sphere_t>(ctx, &ctx->d_spheres, spheres, n_spheres)))
        return rc;
    ctx->n_spheres = n_spheres;
    ctx->bvh_prefix = 0;
    std::shared_ptr<JitKernels> bvh_jit;
    if (ctx->cfg.accel == RVCP_ACCEL_BVH && n_faces > 0) {
        std::vector<float> pos((size_t)n_faces * 9);
        for (uint32_t i = 0; i < n_faces; i++)
            for (int v = 0; v < 3; v++)
                std::memcpy(&pos[(size_t)i * 9 + 3 * v], vertices[faces[i].vertices[v]].position, 12);
        const auto *P = reinterpret_cast<const float (*)[3][3]>(pos.data());
        // The hybrid: when the scene starts with a run of big faces (C5: the
        // Cornell room before 100 000 small triangles), those are tested by the specialised scan
        // -- at full lane utilisation, no dependent loads -- and the BVH holds only the rest, so
        // its boxes are tight and every ray enters it with the room's nearest hit as its bound.
        // Only with a specialised module for them (games101, specialize AUTO, the JIT's range);
        // the kernels without one test the prefix with the generic test.
        uint32_t K = 0;
        if (ctx->cfg.specialize == RVCP_SPECIALIZE_AUTO && ctx->cfg.integrator != RVCP_INTEGRATOR_LEGACY &&
            !RVCP_KNOB("RVCP_NO_BVH_PREFIX")) {
            K = bvh_big_prefix(P, n_faces, kJitMaxFaces);
            if (K < 8 || n_faces - K < 64 || !jit_scene_in_range(tri.data(), K)) K = 0;
            if (K) {
                std::string jerr;
                bvh_jit = jit_path_kernels(ctx->device, tri.data(), K, jerr, false, n_spheres == 0,
                                           false, true);
                HIP_TRY(ctx, hipSetDevice(ctx->device));
                if (!bvh_jit || !bvh_jit->bvh_path || !bvh_jit->bvh_primary) {
                    K = 0;
                    bvh_jit.reset();
                }
            }
        }
        std::vector<BvhNode> nodes;
        std::vector<uint32_t> order;
        int32_t root = 0;
        const int depth = bvh_build(P + K, n_faces - K, nodes, order, root);
        for (uint32_t &id : order)                       // the BVH's ids are faces K ...
            if (id != kBvhPadId) id += K;
        ctx->bvh_prefix = K;
        if (depth >= kBvhStack) return fail(ctx, RVCP_E_UNSUPPORTED, "BVH deeper than the traversal stack");
        // the leaf-ordered triangles packed as 10 floats per slot (v0, e1, e2, face id bits),
        // what the traversal reads (bvh_leaf); leaves start at even slots, so 16-B aligned.
        // A leaf reference is ~((start << 5) | (count - 1)) in an int32: start < 2^26.
        const size_t S = order.size();
        if (S >= (size_t(1) << 26))
            return fail(ctx, RVCP_E_UNSUPPORTED, "BVH leaf slots exceed 2^26 (mesh too large for the leaf encoding)");
        std::vector<TriRecord> btri((10 * S * 4 + sizeof(TriRecord) - 1) / sizeof(TriRecord) + 1);
        float *packed = reinterpret_cast<float *>(btri.data());
        for (size_t j = 0; j < S; j++) {
            if (order[j] == kBvhPadId) continue;        // padding slot: never referenced
            std::memcpy(packed + 10 * j, &tri[order[j]], 9 * sizeof(float));
            std::memcpy(packed + 10 * j + 9, &order[j], 4);
        }
        ctx->bvh_slots = 0;     // the packed records start the buffer
        std::vector<Bvh4Node> nodes4;
        int32_t root4 = 0;
        if (bvh4_collapse(nodes, root, nodes4, root4) > kBvhStack)
            return fail(ctx, RVCP_E_UNSUPPORTED, "BVH traversal stack bound exceeded");
        // only the byte-quantised copy (Bvh4QNode, 64 B) is traversed: it is uploaded alone,
        // at the start of the node buffer (FrameArgs::bvh_n4 = 0)
        std::vector<Bvh4QNode> q4;
        bvh4_quantize(nodes4, q4);
        std::vector<Bvh4Node> qbuf((q4.size() * sizeof(Bvh4QNode) + sizeof(Bvh4Node) - 1) / sizeof(Bvh4Node));
        if (!q4.empty()) std::memcpy(static_cast<void *>(qbuf.data()), q4.data(), q4.size() * sizeof(Bvh4QNode));
        ctx->bvh_n4 = 0;
        if ((rc = dev_upload<Bvh4Node>(ctx, &ctx->d_bvh_nodes, qbuf.data(), qbuf.size())) ||
            (rc = dev_upload<TriRecord>(ctx, &ctx->d_bvh_tris, btri.data(), btri.size())))
            return rc;
        ctx->bvh_root = root4;
        ctx->bvh_depth = depth;
    }
    // scene-specialised scan: compiled here, once per scene and process
    ctx->jit.reset();
    ctx->jit_err.clear();
    if (bvh_jit) ctx->jit = bvh_jit;          // the BVH hybrid's module (above)
    if (ctx->cfg.specialize == RVCP_SPECIALIZE_AUTO && ctx->cfg.accel == RVCP_ACCEL_NONE &&
        n_faces >= 1 && n_faces <= kJitMaxFaces && jit_scene_in_range(tri.data(), n_faces) &&
        !RVCP_KNOB("RVCP_NO_SPECIALIZE")) {
        ctx->jit = jit_path_kernels(ctx->device, tri.data(), n_faces, ctx->jit_err,
                                    ctx->cfg.integrator == RVCP_INTEGRATOR_LEGACY,
                                    n_spheres == 0, n_spheres <= 64 && n_materials <= 64, false,
                                    spheres, n_spheres, n_materials);
        HIP_TRY(ctx, hipSetDevice(ctx->device));
    }
    ctx->rcp_fast = scan_rcp_fast_scene(tri.data(), n_faces);
    ctx->n_faces = n_faces;
    ctx->n_verts = n_vertices;
    ctx->n_mats = n_materials;
    ctx->has_metal = false;
    for (uint32_t i = 0; i < n_materials; i++)
        if (materials[i].ty == 1u) ctx->has_metal = true;
    ctx->n_lights = n_lum_face_ids;
    ctx->lights_same = n_lum_face_ids >= 1;
    for (uint32_t i = 1; i < n_lum_face_ids; i++)
        if (tab.lights[i].face != tab.lights[0].face) ctx->lights_same = false;
    ctx->light_total = total;
    ctx->light_pdf = 1.0f / total;
    ctx->has_scene = true;
    return RVCP_OK;
}

static int impl_upload_scene_file(rvcp_ctx_t *ctx, const char *path, rvcp_camera_t *out_camera)
{
    if (!ctx) return RVCP_E_INVALID;
    SceneFile sf;
    std::string err;
    if (read_scene_file(path, sf, err) != RVCP_OK) return fail(ctx, RVCP_E_INVALID, err);
    const rvcp_lengths_t &L = sf.lengths;
    const int rc = rvcp_upload_scene(ctx, sf.materials.data(), L.materials_len, sf.vertices.data(),
                                     L.vertices_len, sf.faces.data(), L.faces_len, sf.spheres.data(),
                                     L.spheres_len, sf.lum_face_ids.data(), L.luminous_face_id_len,
                                     sf.lum_sphere_ids.data(), L.luminous_sphere_id_len);
    if (rc == RVCP_OK && out_camera) *out_camera = sf.camera;
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

// n_frames consecutive frames of one shard (pushes[k] for frame k) into outputs laid out frame
// after frame, `slot` = the largest shard's rows apart (rvcp_render_frames_async); n_frames = 1
// is rvcp_render_shard_async.
static int render_frames(rvcp_ctx_t *ctx, const rvcp_push_constant_t *pushes, uint32_t n_frames,
                         uint32_t width, uint32_t height, uint32_t shard_index,
                         uint32_t shard_count, void *d_rgba8, void *d_linear_rgb, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    const rvcp_push_constant_t *push = pushes;
    if (!push || n_frames == 0 || !d_rgba8 || width == 0 || height == 0 || shard_count == 0 ||
        shard_index >= shard_count)
        return fail(ctx, RVCP_E_INVALID, "invalid render arguments");
    if ((uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "frame too large (W*H must be < 2^31)");
    // frame k of a batch starts `stride` pixels after frame k-1 (the largest shard's pixels)
    const uint32_t stride = rvcp_shard_rows(height, 0, shard_count) * width;
    if ((uint64_t)n_frames * stride >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "batch too large (n_frames x shard pixels must be < 2^31)");
    if (n_frames > 1 && !ctx->subs.empty())
        return fail(ctx, RVCP_E_UNSUPPORTED, "frame batches drive one GPU (n_gpus = 1)");
    if (!ctx->has_scene) return fail(ctx, RVCP_E_NO_SCENE, "render before rvcp_upload_scene");
    for (uint32_t k = 0; k < n_frames; k++)
        if (!primary_t_range_ok(pushes[k], width, height))
            return fail(ctx, RVCP_E_INVALID, "camera t_far x t_coef must stay below 2^24 (the "
                        "shader's miss test t_max + 1, :287, :424)");
    // one frame in flight per context: its surface list, counters and events are the frame's
    if (ctx->pending)
        return fail(ctx, RVCP_E_INVALID, "a frame is in flight on this context (rvcp_wait first)");
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
    A.lights_same = ctx->lights_same ? 1u : 0u;
    A.rcp_fast = ctx->rcp_fast ? 1u : 0u;
    A.has_metal = ctx->has_metal ? 1u : 0u;
    A.light_total = ctx->light_total;
    A.light_pdf = ctx->light_pdf;
    {   // :465-471: denom = max(0.1, pdf) * rr, pdf = 0.5 / 3.1415926 (cos > 0) or 0; IEEE 1/denom
        const float pdf1 = 0.5f / 3.1415926f;
        A.brdf_den[1] = std::fmax(0.1f, pdf1) * A.rr;
        A.brdf_den[0] = std::fmax(0.1f, 0.0f) * A.rr;
        A.brdf_rcp[1] = 1.0f / A.brdf_den[1];
        A.brdf_rcp[0] = 1.0f / A.brdf_den[0];
    }
    A.want_linear = d_linear_rgb ? 1u : 0u;
    // automatic schedule: 10 / 5 (LDS tiles; the workgroup's rays pooled into full passes on
    // large frames, one ray per lane on small ones) for large meshes, 10 also for mid-size
    // meshes on large frames, else 3, or 6 (6 waves/SIMD) for
    // large frames -- with the scene-specialised scan only for very large frames
    // (kSpecWideMinSamples: its 6-wave build is slower below)
    const bool jit_ok = ctx->jit && ctx->cfg.ray_t_min > 0.0f;
    const bool big_frame = (uint64_t)A.n_pixels * A.spp >= kTiledDualMinSamples;
    A.variant = ctx->cfg.kernel_variant != 0 ? ctx->cfg.kernel_variant
              : ctx->n_faces >= kTiledMinFaces ? (big_frame ? kTiledPoolVariant : 5)
              : (!jit_ok && ctx->n_faces > kTiledWideMinFaces && big_frame) ? kTiledPoolVariant
              : ((uint64_t)A.n_pixels * A.spp >= (jit_ok ? kSpecWideMinSamples : kWideMinSamples)) ? 6
              : kDefaultVariant;
    A.accel = (ctx->cfg.accel == RVCP_ACCEL_BVH && ctx->n_faces > 0) ? RVCP_ACCEL_BVH : RVCP_ACCEL_NONE;
    if (A.accel == RVCP_ACCEL_BVH) A.variant = 3;    // the BVH traversal lives in the v3 kernels
    A.bvh_root = ctx->bvh_root;
    A.bvh_n4 = ctx->bvh_n4;
    A.bvh_slots = ctx->bvh_slots;
    A.bvh_prefix = A.accel == RVCP_ACCEL_BVH ? ctx->bvh_prefix : 0u;
    const bool legacy = ctx->cfg.integrator == RVCP_INTEGRATOR_LEGACY;
    A.n_spheres = legacy ? ctx->n_spheres : 0u;
    A.n_mats = ctx->n_mats;

    // With MAX_BOUNCES == 0 or ATTENUATION_STOP_EPS > 1 every sample returns 0 before its
    // first traversal (:413-419): the frame is black.  ray_tracer.comp has no attenuation
    // test before its first traversal (:629-634).
    const bool trivial = A.max_bounces == 0 || (!legacy && 1.0f < A.att_stop);
    // a batch shares one surface list and one path kernel: the pre-pass schedules (3-6, 10 and
    // the persistent BVH path kernel) only
    if (n_frames > 1 && !trivial && !legacy && A.variant < 3)
        return fail(ctx, RVCP_E_UNSUPPORTED, "frame batches need a pre-pass schedule of the games101 "
                    "integrator (schedules 3-6, 10, or the BVH path kernel) or mode 2");
    std::vector<FrameArgs> FA;          // per frame of the batch (camera, time, pixel base)
    const uint32_t frame_px = A.n_pixels;
    const uint32_t split_px = frame_px * n_frames;          // the queue of the whole batch
    // a batch's cameras and times in device memory: mode 2's one kernel and the pre-pass
    // schedules' one pre-pass launch read them per frame
    const bool cams = n_frames > 1 && !trivial && frame_px > 0 && (legacy || A.variant >= 3);
    if (cams) {
        if (ctx->cap_cams < n_frames) {
            (void)hipFree(ctx->d_cams);
            (void)hipHostFree(ctx->h_cams);
            ctx->d_cams = ctx->h_cams = nullptr;
            ctx->cap_cams = 0;
            HIP_TRY(ctx, hipMalloc((void **)&ctx->d_cams, (size_t)n_frames * 64));
            HIP_TRY(ctx, hipHostMalloc((void **)&ctx->h_cams, (size_t)n_frames * 64));
            ctx->cap_cams = n_frames;
        }
        for (uint32_t k = 0; k < n_frames; ++k) {
            FrameArgs C;
            std::memset(&C, 0, sizeof(C));
            camera_constants(pushes[k], width, height, C);
            float *c = ctx->h_cams + 16 * (size_t)k;
            std::memcpy(c, C.cam_pos, 12);
            std::memcpy(c + 3, C.u, 12);
            std::memcpy(c + 6, C.v, 12);
            std::memcpy(c + 9, C.pos, 12);
            c[12] = C.base_len;
            c[13] = C.t_near;
            c[14] = C.t_far;
            c[15] = C.time;
        }
        HIP_TRY(ctx, hipMemcpyAsync(ctx->d_cams, ctx->h_cams, (size_t)n_frames * 64,
                                    hipMemcpyHostToDevice, s));
    }
    if (cams && legacy) {
        // mode 2 has no pre-pass: its one kernel queues the batch's pixels frame after frame
        // and reads each frame's camera and time from d_cams (FrameArgs::batch_cams)
        A.batch_cams = ctx->d_cams;
        A.frame_pixels = frame_px;
        A.frame_stride = stride;
        A.n_pixels = split_px;
    }
    ctx->last_spec = false;
    // a gather of this context's previous frame may still read the caller's shard buffer
    if (ctx->gather_on_gstream) HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->evg1, 0));
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, kCounterWords * sizeof(unsigned long long), s));
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, s));
    if (A.n_pixels > 0) {
        int rc;
        if (trivial) {
            HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
            rc = rvcp_launch_fill((uint32_t *)d_rgba8, (float *)d_linear_rgb,
                                  n_frames > 1 ? n_frames * stride : A.n_pixels, 0xFF000000u, s);
        } else {
            // the scene-specialised path kernel (§4.7) replaces schedules 3 and 6 when the
            // upload compiled one; its exactness argument needs t_min > 0
            const JitKernels *jk = ctx->jit.get();
            const int jit_per_cu = !jk ? 0 : A.variant == 6 ? jk->blocks_per_cu6
                                 : A.variant == 3 ? jk->blocks_per_cu5 : 0;
            const bool spec = !legacy && !A.accel && jit_per_cu > 0 && A.t_min > 0.0f;
            // mode 2 with the specialised triangle scan (its kernel also checks per wave
            // that every ray is finite and has t_min > 0)
            const bool spec_legacy = legacy && jk && jk->legacy && jk->blocks_per_cu_legacy > 0;
            // the BVH hybrid's kernels (the prefix faces by the specialised scan); without them
            // (t_min <= 0) the built-in BVH kernels test the prefix with the generic test
            const bool spec_bvh = !legacy && A.accel && A.bvh_prefix > 0 && jk && jk->bvh_path &&
                                  jk->bvh_primary && jk->blocks_per_cu_bvh > 0 && A.t_min > 0.0f;
            uint32_t cap = (uint32_t)(legacy ? ctx->legacy_capacity
                                     : A.accel ? ctx->bvh_capacity
                                               : ctx->grid_capacity[A.variant]);
            if (spec) cap = (uint32_t)jit_per_cu * (ctx->n_simds / 4u);
            if (spec_bvh) cap = (uint32_t)jk->blocks_per_cu_bvh * (ctx->n_simds / 4u);
            if (spec_legacy) cap = (uint32_t)jk->blocks_per_cu_legacy * (ctx->n_simds / 4u);
            A.n_simds = ctx->n_simds;
            uint32_t waves = 0, chunk = 0;
            const uint32_t wpb = (uint32_t)((legacy || A.accel ? kBlock : variant_block(A.variant)) / kWave);
            if (ctx->cfg.grid_waves_per_simd > 0) {     // the caller's grid per frame (rvcp.h)
                const uint64_t lim = (uint64_t)ctx->cfg.grid_waves_per_simd * ctx->n_simds / wpb;
                if (lim < cap) cap = lim > 0 ? (uint32_t)lim : 1u;
            }
            rvcp_static_split(split_px, cap * wpb, A.n_simds, &waves, &chunk);
            uint32_t blocks = (waves + wpb - 1) / wpb;
            if (blocks > cap) blocks = cap;
            if (blocks == 0) blocks = 1;
            A.static_chunk = chunk;
            A.static_chunks = waves * chunk;
            A.dyn_chunk = kDynChunk;
            A.chunk_min = kMinChunk;
            A.chunk_window = kChunkWindow;
            if (const char *c = RVCP_KNOB("RVCP_DEBUG_CHUNK")) {   // fixed grab (experiments)
                const int v = std::atoi(c);
                if (v >= 1 && v <= (int)kDynChunk) A.dyn_chunk = A.chunk_min = (uint32_t)v;   // <= 64: mode 2 prefills a grab into 64 LDS slots
            }
            if (const char *c = RVCP_KNOB("RVCP_DEBUG_CHUNK_WINDOW")) {
                const int v = std::atoi(c);
                if (v >= 1) A.chunk_window = (uint32_t)v;
            }
            A.spread_min = 0;
            A.early_tail = 0;
            if (const char *c = RVCP_KNOB("RVCP_DEBUG_SPREAD")) A.spread_min = (uint32_t)std::atoi(c);
            if (const char *c = RVCP_KNOB("RVCP_DEBUG_EARLY_TAIL")) A.early_tail = (uint32_t)std::atoi(c);
            // schedules 3/6 spreading a small surface list run the full resident grid
            if (A.spread_min && !legacy && !A.accel && (A.variant == 3 || A.variant == 6)) blocks = cap;
            ctx->last_timeline_waves = 0;
            if (RVCP_KNOB("RVCP_DEBUG_TIMELINE") && (legacy || A.variant >= 3)) {
                const size_t waves = (size_t)blocks * wpb;
                if (ctx->cap_timeline < waves) {
                    (void)hipFree(ctx->d_timeline);
                    ctx->d_timeline = nullptr;
                    ctx->cap_timeline = 0;
                    HIP_TRY(ctx, hipMalloc((void **)&ctx->d_timeline, waves * 64));
                    ctx->cap_timeline = waves;
                }
                A.timeline = ctx->d_timeline;
                ctx->last_timeline_waves = waves;
            }
            // the mode-2 and v3-family kernels leave linear colours and tonemap_kernel stores
            // the bytes: into the caller's linear buffer, else the context's scratch
            float *lin = (float *)d_linear_rgb;
            const uint32_t n_lin = n_frames > 1 ? n_frames * stride : A.n_pixels;
            if (!lin && (legacy || A.variant >= 3)) {
                if (ctx->cap_acc < n_lin) {
                    (void)hipFree(ctx->d_acc);
                    ctx->d_acc = nullptr;
                    ctx->cap_acc = 0;
                    HIP_TRY(ctx, hipMalloc((void **)&ctx->d_acc, (size_t)n_lin * 12));
                    ctx->cap_acc = n_lin;
                }
                lin = ctx->d_acc;
            }
            if (legacy) {
                HIP_TRY(ctx, hipEventRecord(ctx->evm, s));
                rc = rvcp_launch_legacy(&A, ctx->d_tri, ctx->d_shade, ctx->d_spheres,
                                        ctx->d_rawmats, ctx->d_unorm, (uint32_t *)d_rgba8,
                                        lin, ctx->d_counters, blocks, s,
                                        spec_legacy ? (void *)jk->legacy : nullptr);
                if (spec_legacy) ctx->last_spec = true;
            } else if (A.variant >= 3) {
                const uint32_t n_surf = split_px;
                if (ctx->cap_surf < n_surf) {
                    (void)hipFree(ctx->d_surf);
                    ctx->d_surf = nullptr;
                    ctx->cap_surf = 0;
                    HIP_TRY(ctx, hipMalloc((void **)&ctx->d_surf, (size_t)n_surf * sizeof(SurfRecord)));
                    ctx->cap_surf = n_surf;
                }
                {
                    FA.assign(n_frames, A);
                    for (uint32_t k = 1; k < n_frames; ++k) {
                        camera_constants(pushes[k], width, height, FA[k]);
                        FA[k].pix_base = k * stride;
                    }
                    rc = rvcp_launch_games101_v3(FA.data(), n_frames, stride, ctx->d_tri,
                                                 ctx->d_faces, ctx->d_verts,
                                                 ctx->d_mats, ctx->d_lights, ctx->d_gamma,
                                                 (uint32_t *)d_rgba8, lin,
                                                 ctx->d_counters, ctx->d_surf, ctx->d_shade,
                                                 ctx->d_bvh_nodes, ctx->d_bvh_tris,
                                                 blocks, s, ctx->evm,
                                                 spec ? (void *)(A.variant == 6 ? jk->path6 : jk->path5)
                                                      : spec_bvh ? (void *)jk->bvh_path : nullptr,
                                                 cams && frame_px <= kPrepassBatchMaxPixels
                                                     ? ctx->d_cams : nullptr,
                                                 spec && jit_spec_prepass() ? (void *)jk->primary
                                                 : spec_bvh ? (void *)jk->bvh_primary : nullptr);
                }
                if (spec || spec_bvh) ctx->last_spec = true;
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
    ctx->render_stream = s;
    ctx->last_trivial = trivial;
    ctx->last_variant = (trivial || A.n_pixels == 0) ? 0 : legacy ? 8
                      : A.accel ? 7 : A.variant;
    if (ctx->last_spec && ctx->last_variant != 0) ctx->last_variant |= RVCP_VARIANT_SPECIALIZED;
    ctx->last_pixels = (uint64_t)frame_px * n_frames;       // stats cover the whole batch
    ctx->last_spp = A.spp;
    ctx->last_shard_index = shard_index;
    ctx->last_shard_count = shard_count;
    ctx->last_width = width;
    ctx->last_height = height;
    return RVCP_OK;
}

static int impl_render_shard_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                                   uint32_t height, uint32_t shard_index, uint32_t shard_count,
                                   void *d_rgba8, void *d_linear_rgb, void *stream)
{
    return render_frames(ctx, push, 1, width, height, shard_index, shard_count, d_rgba8,
                         d_linear_rgb, stream);
}

static int impl_render_frames_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *pushes,
                                    uint32_t n_frames, uint32_t width, uint32_t height,
                                    uint32_t shard_index, uint32_t shard_count, void *d_rgba8,
                                    void *d_linear_rgb, void *stream)
{
    return render_frames(ctx, pushes, n_frames, width, height, shard_index, shard_count, d_rgba8,
                         d_linear_rgb, stream);
}

static int impl_render_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                      uint32_t height, void *d_rgba8, void *d_linear_rgb, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->subs.empty())
        return fail(ctx, RVCP_E_UNSUPPORTED, "rvcp_render_async drives one GPU; use rvcp_render for n_gpus > 1");
    return rvcp_render_shard_async(ctx, push, width, height, 0, 1, d_rgba8, d_linear_rgb, stream);
}

static int impl_wait(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    return rvcp_sync_stats(ctx, stats);
}

static int impl_sync_stats(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->pending) return fail(ctx, RVCP_E_INVALID, "no render in flight");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipEventSynchronize(ctx->ev1));
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        unsigned long long c[kCounterWords] = {};
        HIP_TRY(ctx, hipMemcpy(c, ctx->d_counters, sizeof(c), hipMemcpyDeviceToHost));
        // the path kernel's per-wave clock stamps (clock_stamp): shader-clock ticks over
        // 100-MHz ticks, summed over its waves
        stats->shader_clock_ghz = c[kClockWord + 1]
            ? 0.1 * (double)c[kClockWord] / (double)c[kClockWord + 1] : 0.0;
        stats->kernel_ms = ms;
        float ms_main = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms_main, ctx->evm, ctx->ev1));
        stats->main_kernel_ms = ms_main;
        stats->traversals_executed = c[0];
        // the reference re-traces the (RNG-independent) primary ray in every sample
        stats->traversals = ctx->last_trivial ? 0 : c[0] + ctx->last_pixels * (ctx->last_spp - 1);
        stats->samples = ctx->last_pixels * ctx->last_spp;
        stats->faces = ctx->n_faces;
        stats->kernel_variant = ctx->last_variant;
        stats->wave_iterations = c[2];
    }
    if (ctx->last_timeline_waves) {
        std::vector<unsigned long long> t(8 * ctx->last_timeline_waves);
        HIP_TRY(ctx, hipMemcpy(t.data(), ctx->d_timeline, t.size() * 8, hipMemcpyDeviceToHost));
        const char *path = RVCP_KNOB("RVCP_DEBUG_TIMELINE");
        if (FILE *f = path ? std::fopen(path, "ab") : nullptr) {
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
        total.kernel_variant = st.kernel_variant;
        if (k == 0) total.shader_clock_ghz = st.shader_clock_ghz;
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

static int impl_render(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                uint32_t height, uint8_t *out_rgba8, float *out_linear_rgb, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!out_rgba8) return fail(ctx, RVCP_E_INVALID, "out_rgba8 is required");
    if (ctx->pending)
        return fail(ctx, RVCP_E_INVALID, "a frame is in flight on this context (rvcp_wait first)");
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

static int impl_mandelbrot(rvcp_ctx_t *ctx, const rvcp_mandelbrot_push_t *push, uint32_t width,
                    uint32_t height, uint8_t *out_rgba8, float *out_value, rvcp_stats_t *stats)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!push || !out_rgba8 || width == 0 || height == 0 || (uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "invalid mandelbrot arguments");
    if (ctx->pending)
        return fail(ctx, RVCP_E_INVALID, "a frame is in flight on this context (rvcp_wait first)");
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

static int impl_assemble_frame_async(rvcp_ctx_t *ctx, const void *d_gathered, uint32_t slot_rows,
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


// ---- one process per GPU: the frame gather over RCCL ----
static int impl_rccl_unique_id(uint8_t *out_id)
{
    if (!out_id) return fail(nullptr, RVCP_E_INVALID, "null id buffer");
    const RcclApi &R = rccl_api();
    if (!R.ok) return fail(nullptr, RVCP_E_UNSUPPORTED, R.why);
    static_assert(sizeof(ncclUniqueId) == RVCP_RCCL_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    const ncclResult_t r = R.get_unique_id(&id);
    if (r != ncclSuccess) return fail(nullptr, RVCP_E_HIP, std::string("ncclGetUniqueId: ") + R.error_string(r));
    std::memcpy(out_id, &id, sizeof(id));
    return RVCP_OK;
}

// debug build only (tools/rccl_timeout_diag.py): stage stamps of the communicator paths on stderr
static void rccl_trace(const char *what, long v = 0)
{
    static const bool on = RVCP_KNOB("RVCP_DEBUG_RCCL_TRACE") != nullptr;
    if (on) std::fprintf(stderr, "rvcp rccl: %s %ld\n", what, v);
}

static Clock::time_point comm_deadline(const rvcp_ctx_t *ctx)
{
    return ctx->comm_timeout_ms ? Clock::now() + std::chrono::milliseconds(ctx->comm_timeout_ms)
                                : Clock::time_point::max();
}

// Abort ctx's communicator (ours) after a deadline or an asynchronous error: ncclCommAbort
// raises RCCL's abort flag, which its kernels poll in every wait loop, so a gather stuck on a
// peer that never comes finishes and the streams drain; the context stays usable for
// single-GPU renders.  The abort itself runs on a detached thread: it also joins RCCL's own
// threads, and a wait for a peer that never comes must not become a wait inside the abort.  A
// caller's communicator (rvcp_rccl_attach) is the caller's to abort.
static void abort_comm(rvcp_ctx_t *ctx)
{
    if (ctx->comm && ctx->comm_owned) {
        const ncclComm_t c = ctx->comm;
        rccl_trace("abort: detached ncclCommAbort");
        auto done = std::make_shared<std::atomic<bool>>(false);
        ctx->aborts.push_back(done);          // rvcp_destroy waits for it (bounded)
        std::thread([c, done] {
            (void)rccl_api().comm_abort(c);
            done->store(true);
        }).detach();
    }
    if (ctx->comm_owned) ctx->comm = nullptr;
}

// A gather that timed out and whose stream did not drain (an attached communicator, which this
// library cannot abort, or an abort that has not taken effect): the context forgets the
// communicator (the caller's stays the caller's to abort), later renders stop waiting for the
// gather (a wait on its end event would never return), the gather stream it sits on is retired
// (a new gather gets a fresh one), and its end event is kept for rvcp_destroy.
static int retire_stuck_gather(rvcp_ctx_t *ctx)
{
    ctx->stuck_gathers.push_back(ctx->evg1);
    ctx->evg1 = nullptr;
    if (ctx->gather_on_gstream && ctx->gstream) {
        ctx->retired_gstreams.push_back(ctx->gstream);
        ctx->gstream = nullptr;
    }
    ctx->gather_on_gstream = false;
    ctx->gather_pending = false;
    ctx->comm = nullptr;
    HIP_TRY(ctx, hipEventCreate(&ctx->evg1));
    return RVCP_OK;
}

// Wait until a non-blocking communicator has finished its last call (ncclInProgress ->
// ncclSuccess), bounded by `deadline`.  RVCP_E_TIMEOUT on expiry, RVCP_E_HIP on an RCCL error.
static int wait_comm_ready(rvcp_ctx_t *ctx, ncclComm_t comm, Clock::time_point deadline,
                           const char *what)
{
    const RcclApi &R = rccl_api();
    for (unsigned spin = 0;; spin++) {
        ncclResult_t st = ncclInProgress;
        const ncclResult_t r = R.get_async_error(comm, &st);
        if (r != ncclSuccess)
            return fail(ctx, RVCP_E_HIP, std::string(what) + ": ncclCommGetAsyncError: " + R.error_string(r));
        if (st == ncclSuccess) return RVCP_OK;
        if (st != ncclInProgress)
            return fail(ctx, RVCP_E_HIP, std::string(what) + ": " + R.error_string(st));
        if (Clock::now() >= deadline)
            return fail(ctx, RVCP_E_TIMEOUT, std::string(what) + ": no progress within " +
                        std::to_string(ctx->comm_timeout_ms) + " ms (a peer rank missing or failed)");
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 100 ? 20 : 1000));
    }
}

// The communicator's creation runs on a worker thread: ncclCommInitRankConfig (blocking = 0)
// and the poll of ncclCommGetAsyncError until the rendezvous completes.  The caller waits for
// the worker with the deadline, so rvcp_rccl_init returns in time whatever RCCL does inside
// (on this image's RCCL 2.27.7 the "non-blocking" ncclCommInitRankConfig itself does not return
// while a peer is absent: profiles/history/r05g_rccl_diag.log, tools/rccl_timeout_diag.py); a worker left
// behind aborts its half-made communicator if it ever gets control back (detached: the process
// never waits for it, and exits cleanly, tests/test_gpu_rccl_timeout.py).
struct CommJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t result = ncclSuccess;
    ncclComm_t comm = nullptr;
};

// Creation workers abandoned at their deadline and still blocked inside RCCL, process-wide
// (reported in the messages: each holds a thread and a half-made communicator until RCCL
// returns, which on RCCL 2.27.7 is never while the peer stays absent)
static std::atomic<int> g_blocked_init_workers{0};

static int impl_rccl_init(rvcp_ctx_t *ctx, const uint8_t *id, uint32_t world, uint32_t rank)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!id || world == 0 || rank >= world || world > 4096)
        return fail(ctx, RVCP_E_INVALID, "invalid RCCL rank / world");
    if (ctx->comm) return fail(ctx, RVCP_E_INVALID, "context already has a communicator");
    if (ctx->init_job) {
        // the worker of this context's last timed-out creation: refuse a new one while it is
        // still blocked inside RCCL (retries must not leak a thread each)
        std::lock_guard<std::mutex> g(ctx->init_job->m);
        if (!ctx->init_job->done)
            return fail(ctx, RVCP_E_BUSY, "rvcp_rccl_init: this context's previous creation timed "
                        "out and its worker is still blocked inside RCCL (" +
                        std::to_string(g_blocked_init_workers.load()) + " such worker(s) in the "
                        "process); use another context, or retry once RCCL has returned");
    }
    ctx->init_job.reset();
    const RcclApi &R = rccl_api();
    if (!R.ok) return fail(ctx, RVCP_E_UNSUPPORTED, R.why);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const Clock::time_point deadline = comm_deadline(ctx);
    auto job = std::make_shared<CommJob>();
    const int dev = ctx->device;
    std::thread([job, uid, world, rank, dev]() mutable {
        const RcclApi &R = rccl_api();
        (void)hipSetDevice(dev);
        // non-blocking: a library older than this header reads only the fields it knows (`size`
        // tells it how many there are)
        ncclConfig_t conf = NCCL_CONFIG_INITIALIZER;
        conf.blocking = 0;
        ncclComm_t comm = nullptr;
        rccl_trace("init worker: calling ncclCommInitRankConfig, world", (long)world);
        ncclResult_t r = R.comm_init_rank_config(&comm, (int)world, uid, (int)rank, &conf);
        rccl_trace("init worker: returned", (long)r);
        for (unsigned spin = 0; r == ncclSuccess || r == ncclInProgress; spin++) {
            ncclResult_t st = ncclInProgress;
            if (!comm || R.get_async_error(comm, &st) != ncclSuccess) { r = ncclInternalError; break; }
            if (st != ncclInProgress) { r = st; break; }
            {
                std::lock_guard<std::mutex> g(job->m);
                if (job->abandoned) break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(spin < 100 ? 20 : 1000));
        }
        bool keep;
        {
            std::lock_guard<std::mutex> g(job->m);
            keep = !job->abandoned && r == ncclSuccess;
            job->result = r;
            if (keep) job->comm = comm;
            job->done = true;
            if (job->abandoned) g_blocked_init_workers--;
        }
        job->cv.notify_all();
        if (!keep && comm) {
            rccl_trace("init worker: ncclCommAbort");
            (void)R.comm_abort(comm);
            rccl_trace("init worker: ncclCommAbort returned");
        }
    }).detach();
    std::unique_lock<std::mutex> lk(job->m);
    bool finished;
    if (ctx->comm_timeout_ms == 0) {
        job->cv.wait(lk, [&] { return job->done; });
        finished = true;
    } else {
        finished = job->cv.wait_until(lk, deadline, [&] { return job->done; });
    }
    if (!finished) {
        job->abandoned = true;
        const int blocked = ++g_blocked_init_workers;
        ctx->init_job = job;
        ctx->comm_timed_out = true;
        rccl_trace("init: deadline, worker abandoned");
        return fail(ctx, RVCP_E_TIMEOUT, "ncclCommInitRankConfig: no rendezvous within " +
                    std::to_string(ctx->comm_timeout_ms) + " ms (a peer rank missing or failed); "
                    "the half-made communicator is aborted once RCCL returns; its creation worker "
                    "is left blocked inside RCCL (" + std::to_string(blocked) + " in the process) "
                    "and this context refuses another rvcp_rccl_init until it returns");
    }
    if (job->result != ncclSuccess)
        return fail(ctx, RVCP_E_HIP, std::string("ncclCommInitRankConfig: ") + R.error_string(job->result));
    ctx->comm = job->comm;
    ctx->comm_owned = true;
    ctx->comm_timed_out = false;
    ctx->comm_world = world;
    ctx->comm_rank = rank;
    return RVCP_OK;
}

static int impl_rccl_set_timeout(rvcp_ctx_t *ctx, uint32_t timeout_ms)
{
    if (!ctx) return RVCP_E_INVALID;
    ctx->comm_timeout_ms = timeout_ms;
    return RVCP_OK;
}

static int impl_rccl_attach(rvcp_ctx_t *ctx, void *nccl_comm, uint32_t world, uint32_t rank)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!nccl_comm || world == 0 || rank >= world)
        return fail(ctx, RVCP_E_INVALID, "invalid communicator / rank / world");
    if (ctx->comm) return fail(ctx, RVCP_E_INVALID, "context already has a communicator");
    if (!rccl_api().ok) return fail(ctx, RVCP_E_UNSUPPORTED, rccl_api().why);
    ctx->comm = (ncclComm_t)nccl_comm;
    ctx->comm_owned = false;
    ctx->comm_timed_out = false;
    ctx->comm_world = world;
    ctx->comm_rank = rank;
    return RVCP_OK;
}

static int impl_gather_frame_async(rvcp_ctx_t *ctx, const void *d_shard_rgba8, uint32_t width,
                                   uint32_t height, void *d_gathered, void *d_frame, void *stream)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->comm && ctx->comm_timed_out)
        return fail(ctx, RVCP_E_TIMEOUT, "the communicator was given up after a gather or creation "
                    "deadline; rvcp_rccl_init / rvcp_rccl_attach a new one first");
    if (!ctx->comm) return fail(ctx, RVCP_E_INVALID, "no communicator (rvcp_rccl_init first)");
    const bool root = ctx->comm_rank == 0;
    if (!d_shard_rgba8 || width == 0 || height == 0 || (root && (!d_gathered || !d_frame)))
        return fail(ctx, RVCP_E_INVALID, "invalid gather arguments");
    if ((uint64_t)width * height >= (1ull << 31))
        return fail(ctx, RVCP_E_INVALID, "frame too large (W*H must be < 2^31)");
    // the gather assumes this rank rendered shard comm_rank of comm_world of this frame size;
    // anything else would assemble a scrambled frame on rank 0
    if (ctx->last_shard_count != ctx->comm_world || ctx->last_shard_index != ctx->comm_rank ||
        ctx->last_width != width || ctx->last_height != height)
        return fail(ctx, RVCP_E_INVALID, "gather after a render of another shard / frame size "
                    "(rvcp_render_shard_async must use shard_index = rank, shard_count = world)");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // the caller's stream, or the context's gather stream behind the render (evr): the
    // gather and rank 0's assembly then leave the render stream free for the next frame
    if (!stream && !ctx->gstream) {
        // the frame gather's own stream, at the device's highest priority: its RCCL and
        // assembly kernels are dispatched ahead of other streams' queued work
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
            hipStreamCreateWithPriority(&ctx->gstream, hipStreamNonBlocking, greatest) != hipSuccess) {
            ctx->gstream = nullptr;
            return fail(ctx, RVCP_E_HIP, "gather stream creation failed");
        }
    }
    hipStream_t s = stream ? (hipStream_t)stream : ctx->gstream;
    if (!stream) {
        HIP_TRY(ctx, hipEventRecord(ctx->evr, ctx->render_stream ? ctx->render_stream : ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->evr, 0));
    }
    const uint32_t N = ctx->comm_world;
    const uint32_t slot = rvcp_shard_rows(height, 0, N);      // shard 0 has the most rows
    HIP_TRY(ctx, hipEventRecord(ctx->evg0, s));
    const ncclResult_t r = rccl_api().gather(d_shard_rgba8, root ? d_gathered : nullptr,
                                             (size_t)slot * width, ncclUint32, 0, ctx->comm, s);
    if (r != ncclSuccess && r != ncclInProgress)
        return fail(ctx, RVCP_E_HIP, std::string("ncclGather: ") + rccl_api().error_string(r));
    if (r == ncclInProgress) {
        // a non-blocking communicator -- ours, or an attached one created with blocking = 0
        // (torch's non-blocking communicators) -- may still be connecting to its peers (first
        // gather): the collective is on stream s only once it has, so the assembly and evg1
        // must not be queued before that; bounded by the deadline
        const int rc = wait_comm_ready(ctx, ctx->comm, comm_deadline(ctx), "ncclGather");
        if (rc != RVCP_OK) {
            // ours is aborted; an attached one only its owner may abort: dropped either way
            abort_comm(ctx);
            ctx->comm = nullptr;
            ctx->comm_timed_out = rc == RVCP_E_TIMEOUT;
            return rc;
        }
    }
    if (root && rvcp_launch_assemble((const uint32_t *)d_gathered, slot, width, height, N,
                                     (uint32_t *)d_frame, s) != 0)
        return fail(ctx, RVCP_E_HIP, "assemble launch failed");
    HIP_TRY(ctx, hipEventRecord(ctx->evg1, s));
    ctx->gather_pending = true;
    ctx->gather_on_gstream = !stream;
    return RVCP_OK;
}

// Poll the gather's end event against the deadline (a hipEventSynchronize would block forever
// when a peer never enters the collective); on expiry, or when RCCL reports an asynchronous
// error, abort the communicator so that the stuck kernel exits and the streams drain.
static int wait_gather_done(rvcp_ctx_t *ctx)
{
    const Clock::time_point deadline = comm_deadline(ctx);
    const RcclApi &R = rccl_api();
    for (unsigned spin = 0;; spin++) {
        const hipError_t q = hipEventQuery(ctx->evg1);
        if (q == hipSuccess) return RVCP_OK;
        if (q != hipErrorNotReady)
            return fail(ctx, RVCP_E_HIP, std::string("gather: ") + hipGetErrorString(q));
        if (ctx->comm && (spin & 63) == 63) {
            ncclResult_t st = ncclSuccess;
            if (R.get_async_error(ctx->comm, &st) == ncclSuccess && st != ncclSuccess &&
                st != ncclInProgress) {
                const std::string msg = std::string("ncclGather: ") + R.error_string(st);
                abort_comm(ctx);
                return fail(ctx, RVCP_E_HIP, msg);
            }
        }
        if (Clock::now() >= deadline) {
            const bool owned = ctx->comm_owned;
            abort_comm(ctx);
            // the aborted kernels exit; give the stream a bounded moment to drain so that the
            // context's buffers are no longer read when the caller frees or reuses them
            const Clock::time_point drain = Clock::now() + std::chrono::seconds(owned ? 5 : 0);
            while (hipEventQuery(ctx->evg1) == hipErrorNotReady && Clock::now() < drain)
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
            const bool drained = hipEventQuery(ctx->evg1) == hipSuccess;
            ctx->comm_timed_out = true;
            if (drained) {
                ctx->gather_pending = false;
                ctx->gather_on_gstream = false;
                ctx->comm = nullptr;
            } else {
                const int rc = retire_stuck_gather(ctx);
                if (rc != RVCP_OK) return rc;
            }
            return fail(ctx, RVCP_E_TIMEOUT, "gather not complete within " +
                        std::to_string(ctx->comm_timeout_ms) +
                        " ms (a peer rank missing or failed); " +
                        (owned ? "communicator aborted" : "the attached communicator is dropped "
                                 "(abort it: only its owner can)") +
                        (drained ? "" : "; its stream has not drained: later renders do not wait "
                                        "for it, and a new gather needs a new communicator"));
        }
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 2000 ? 5 : 200));
    }
}

static int impl_gather_wait(rvcp_ctx_t *ctx, float *gather_ms, float *frame_ms)
{
    if (!ctx) return RVCP_E_INVALID;
    if (!ctx->gather_pending) return fail(ctx, RVCP_E_INVALID, "no gather in flight");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const int rc = wait_gather_done(ctx);
    if (rc != RVCP_OK) return rc;
    ctx->gather_pending = false;
    float ms = 0.0f;
    if (gather_ms) {
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->evg0, ctx->evg1));
        *gather_ms = ms;
    }
    if (frame_ms) {
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->evg1));
        *frame_ms = ms;
    }
    return RVCP_OK;
}

// ---------------------------------------------------------------------------------------
// Exception barrier: every int-returning entry point runs its implementation inside
// `barrier`, so no C++ exception (std::bad_alloc from a host vector or string, anything a
// runtime library throws) crosses the C-ABI (rvcp.h conventions).
// ---------------------------------------------------------------------------------------

int rvcp_config_default_for(int32_t integrator, rvcp_config_t *cfg)
{
    return barrier(nullptr, [&] { return impl_config_default_for(integrator, cfg); });
}

int rvcp_config_default(rvcp_config_t *cfg)
{
    return barrier(nullptr, [&] { return impl_config_default(cfg); });
}

int rvcp_create(const rvcp_config_t *cfg, rvcp_ctx_t **out_ctx)
{
    return barrier(nullptr, [&] { return impl_create(cfg, out_ctx); });
}

int rvcp_destroy(rvcp_ctx_t *ctx)
{
    return barrier(nullptr, [&] { return impl_destroy(ctx); });
}

int rvcp_upload_scene(rvcp_ctx_t *ctx, const rvcp_material_t *materials, uint32_t n_materials,
                      const rvcp_vertex_t *vertices, uint32_t n_vertices,
                      const rvcp_face_t *faces, uint32_t n_faces,
                      const rvcp_sphere_t *spheres, uint32_t n_spheres,
                      const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                      const uint32_t *lum_sphere_ids, uint32_t n_lum_sphere_ids)
{
    return barrier(ctx, [&] { return impl_upload_scene(ctx, materials, n_materials, vertices,
        n_vertices, faces, n_faces, spheres, n_spheres, lum_face_ids, n_lum_face_ids,
        lum_sphere_ids, n_lum_sphere_ids); });
}

int rvcp_upload_scene_file(rvcp_ctx_t *ctx, const char *path, rvcp_camera_t *out_camera)
{
    return barrier(ctx, [&] { return impl_upload_scene_file(ctx, path, out_camera); });
}

int rvcp_render_shard_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                            uint32_t height, uint32_t shard_index, uint32_t shard_count,
                            void *d_rgba8, void *d_linear_rgb, void *stream)
{
    return barrier(ctx, [&] { return impl_render_shard_async(ctx, push, width, height,
        shard_index, shard_count, d_rgba8, d_linear_rgb, stream); });
}

int rvcp_render_frames_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *pushes, uint32_t n_frames,
                             uint32_t width, uint32_t height, uint32_t shard_index,
                             uint32_t shard_count, void *d_rgba8, void *d_linear_rgb, void *stream)
{
    return barrier(ctx, [&] {
        return impl_render_frames_async(ctx, pushes, n_frames, width, height, shard_index,
                                        shard_count, d_rgba8, d_linear_rgb, stream);
    });
}

int rvcp_render_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                      uint32_t height, void *d_rgba8, void *d_linear_rgb, void *stream)
{
    return barrier(ctx, [&] { return impl_render_async(ctx, push, width, height, d_rgba8,
        d_linear_rgb, stream); });
}

int rvcp_wait(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    return barrier(ctx, [&] { return impl_wait(ctx, stats); });
}

int rvcp_sync_stats(rvcp_ctx_t *ctx, rvcp_stats_t *stats)
{
    return barrier(ctx, [&] { return impl_sync_stats(ctx, stats); });
}

int rvcp_render(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push, uint32_t width,
                uint32_t height, uint8_t *out_rgba8, float *out_linear_rgb, rvcp_stats_t *stats)
{
    return barrier(ctx, [&] { return impl_render(ctx, push, width, height, out_rgba8,
        out_linear_rgb, stats); });
}

int rvcp_mandelbrot(rvcp_ctx_t *ctx, const rvcp_mandelbrot_push_t *push, uint32_t width,
                    uint32_t height, uint8_t *out_rgba8, float *out_value, rvcp_stats_t *stats)
{
    return barrier(ctx, [&] { return impl_mandelbrot(ctx, push, width, height, out_rgba8,
        out_value, stats); });
}

int rvcp_assemble_frame_async(rvcp_ctx_t *ctx, const void *d_gathered, uint32_t slot_rows,
                              uint32_t width, uint32_t height, uint32_t shard_count,
                              void *d_frame, void *stream)
{
    return barrier(ctx, [&] { return impl_assemble_frame_async(ctx, d_gathered, slot_rows,
        width, height, shard_count, d_frame, stream); });
}

int rvcp_rccl_unique_id(uint8_t *out_id)
{
    return barrier(nullptr, [&] { return impl_rccl_unique_id(out_id); });
}

int rvcp_rccl_init(rvcp_ctx_t *ctx, const uint8_t *id, uint32_t world, uint32_t rank)
{
    return barrier(ctx, [&] { return impl_rccl_init(ctx, id, world, rank); });
}

int rvcp_rccl_set_timeout(rvcp_ctx_t *ctx, uint32_t timeout_ms)
{
    return barrier(ctx, [&] { return impl_rccl_set_timeout(ctx, timeout_ms); });
}

int rvcp_rccl_attach(rvcp_ctx_t *ctx, void *nccl_comm, uint32_t world, uint32_t rank)
{
    return barrier(ctx, [&] { return impl_rccl_attach(ctx, nccl_comm, world, rank); });
}

int rvcp_gather_frame_async(rvcp_ctx_t *ctx, const void *d_shard_rgba8, uint32_t width,
                            uint32_t height, void *d_gathered, void *d_frame, void *stream)
{
    return barrier(ctx, [&] { return impl_gather_frame_async(ctx, d_shard_rgba8, width, height,
        d_gathered, d_frame, stream); });
}

int rvcp_gather_wait(rvcp_ctx_t *ctx, float *gather_ms, float *frame_ms)
{
    return barrier(ctx, [&] { return impl_gather_wait(ctx, gather_ms, frame_ms); });
}

}  // extern "C"
