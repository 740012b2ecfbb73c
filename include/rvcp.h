/*
 * rvcp.h -- C-ABI of librvcp, the MI355X (gfx950) replacement for the Vulkano compute
 * pipeline of YXHXianYu/RVCP-Real-Time-Path-Tracer (`src/ray_tracer/vulkan.rs`).
 *
 * The hot path behind this ABI is the per-pixel path-tracing kernel that `src/ray_tracer`
 * dispatches: `assets/shaders/ray_tracer_games101_branch.comp` (selected by
 * `src/ray_tracer/shader.rs:12`).  Every struct below is byte-identical to the reference's
 * Rust-side upload struct (`#[repr(C)]`, `BufferContents`), so a Rust caller can hand the
 * same `Vec<Aligned*>` it used to give `Buffer::from_iter` straight to this library.
 *
 * Conventions
 *   - All functions return 0 (RVCP_OK) on success and a negative RVCP_E_* code on failure.
 *     Nothing aborts or throws across the ABI; `rvcp_last_error(ctx)` returns a message.
 *   - A context is not thread-safe: use one context per host thread.
 *   - One frame in flight per context: a render, upload or Mandelbrot call while an async
 *     frame is pending (rvcp_render_async / rvcp_render_shard_async not yet waited for with
 *     rvcp_wait / rvcp_sync_stats) fails with RVCP_E_INVALID.  Use one context per frame in
 *     flight.
 *   - Host pointers stay owned by the caller; the library copies what it needs.
 *   - Pointers named `d_*` are HIP device pointers; `stream` is a `hipStream_t` (NULL = the
 *     context's own stream, created by rvcp_create).
 */
#ifndef RVCP_H
#define RVCP_H

#ifndef __HIPCC_RTC__               /* hipRTC (the scene-specialised kernels) has these built in */
#include <stddef.h>
#include <stdint.h>
#else
using __hip_internal::int32_t;
using __hip_internal::uint8_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#ifndef offsetof
#define offsetof(t, m) __builtin_offsetof(t, m)
#endif
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------
 * Upload structs (byte-identical to the reference; RVCP_STATIC_ASSERTs below)
 * ------------------------------------------------------------------------------------- */

/* == AlignedCamera, src/ray_tracer/scene/camera.rs:27-37 (64 B).
 *    Shader view: struct Camera, ray_tracer_games101_branch.comp:37-44 (std430 push block). */
typedef struct rvcp_camera {
    float position[4];      /* xyz + pad (utils.rs:5-7 vec3_to_f32_4) */
    float up[4];            /* xyz + pad */
    float forward[3];
    float t_near;
    float t_far;
    float vertical_fov;     /* degrees */
    uint32_t _padding[2];
} rvcp_camera_t;

/* == PushConstant { camera: AlignedCamera, time: f32 }, src/ray_tracer/vulkan.rs:113-118
 *    (68 B).  `time` is the RNG seed input (vulkan.rs:418-421 stamps unix_secs % 1000). */
typedef struct rvcp_push_constant {
    rvcp_camera_t camera;
    float time;
} rvcp_push_constant_t;

/* == AlignedMaterial, src/ray_tracer/scene/material.rs:20-28 (32 B, std140 array stride).
 *    ty: 0 Lambertian, 1 Metal, 2 Dielectric, 3 Light (material.rs:4-10). */
typedef struct rvcp_material {
    float albedo[3];        /* Le for lights */
    uint32_t ty;
    float fuzz;
    float refraction_ratio;
    uint32_t _padding[2];
} rvcp_material_t;

/* == AlignedVertex, src/ray_tracer/scene/mesh.rs:13-18 (32 B). */
typedef struct rvcp_vertex {
    float position[4];
    float normal[4];
} rvcp_vertex_t;

/* == AlignedFace, src/ray_tracer/scene/mesh.rs:37-42 (16 B). */
typedef struct rvcp_face {
    uint32_t vertices[3];
    uint32_t material_id;
} rvcp_face_t;

/* == AlignedSphere, src/ray_tracer/scene/sphere.rs:10-17 (32 B).  Traced by integrator
 *    RVCP_INTEGRATOR_LEGACY (ray_tracer.comp:300-321); the games101 shader never reads
 *    spheres. */
typedef struct rvcp_sphere {
    float center[3];
    float radius;
    uint32_t material_id;
    uint32_t _padding[3];
} rvcp_sphere_t;

/* == CameraData push constant of the Mandelbrot operator, src/mandelbrot/shader.rs:9-12 /
 *    assets/shaders/mandelbrot.comp:5-8 (vec2 position @0, float scale @8; 12 B). */
typedef struct rvcp_mandelbrot_push {
    float position[2];
    float scale;
} rvcp_mandelbrot_push_t;

/* == the 6 x u32 LengthBuffer, vulkan.rs:481-500 / ray_tracer_games101_branch.comp:58-65. */
typedef struct rvcp_lengths {
    uint32_t materials_len;
    uint32_t spheres_len;
    uint32_t vertices_len;
    uint32_t faces_len;
    uint32_t luminous_sphere_id_len;
    uint32_t luminous_face_id_len;
} rvcp_lengths_t;

/* ---------------------------------------------------------------------------------------
 * Configuration: the shader's compile-time #defines become runtime parameters with the
 * same defaults (ray_tracer_games101_branch.comp:5-13).
 * ------------------------------------------------------------------------------------- */
enum {
    /* ray_trace_games101 of ray_tracer_games101_branch.comp: the shader src/ray_tracer
     * dispatches (shader.rs:12).  Triangles only; area-light NEE; gamma 0.6 on store. */
    RVCP_INTEGRATOR_GAMES101 = 0,
    /* ray_trace of ray_tracer.comp (compiled by src/ray_tracer_deprecated/shader.rs:12):
     * spheres then triangles, Lambertian / metal / dielectric scattering, no NEE, no gamma
     * (ray_tracer.comp:618-694, :802-822).  Its #define defaults (ray_tracer.comp:5-13) come
     * from rvcp_config_default_for(RVCP_INTEGRATOR_LEGACY, ...); attenuation_stop_eps and
     * lum_id_std140_quirk are unused (the black-path test uses eps, :672). */
    RVCP_INTEGRATOR_LEGACY = 1,
};

enum {
    RVCP_ACCEL_NONE = 0,              /* brute-force scan, as the shader (parity) */
    RVCP_ACCEL_BVH = 1,               /* opt-in BVH (README.md:28-32 TODO "BVH") */
};

enum {
    RVCP_SPECIALIZE_AUTO = 0,
    RVCP_SPECIALIZE_OFF = 1,
};

enum {
    RVCP_UNORM_DRIVER = 0,            /* the reference driver's 12-bit fixed-point conversion */
    RVCP_UNORM_NEAREST = 1,           /* round-to-nearest */
};

typedef struct rvcp_config {
    int32_t device;                   /* HIP device ordinal */
    int32_t integrator;               /* RVCP_INTEGRATOR_* */
    uint32_t spp;                     /* SPP (:8) = 20 */
    uint32_t max_bounces;             /* MAX_BOUNCES (:9) = 15 */
    float attenuation_stop_eps;       /* ATTENUATION_STOP_EPS (:10) = 0.05 */
    float ray_t_min;                  /* RAY_T_MIN (:11) = 0.01 */
    float ray_t_max;                  /* RAY_T_MAX (:12) = 10000 */
    float rr_probability;             /* RR_PROBABILITY (:13) = 0.8 */
    float eps;                        /* EPS (:5) = 0.001 */
    /* 1 (default) reproduces what the reference GPU reads from the std140 `uint v[100]`
     * LuminousFaceIdBuffer that the host fills with tightly packed u32s
     * (ray_tracer_games101_branch.comp:109-111 vs vulkan.rs:473-478): element i is
     * ids[4*i] when 4*i < n_ids, else 0.  0 = the intended packed semantics. */
    int32_t lum_id_std140_quirk;
    /* Kernel schedule, for A/B measurement only: 0 = automatic (3; 6 for large frames with the
     * generic scan; 10 for meshes of 256+ faces on frames of 512 Ki samples or more, 5 on
     * smaller ones), 1 = one ray per lane per iteration, 2 = shadow + continuation ray per
     * lane per iteration, 3 = primary pre-pass + 2 over surface pixels (scalar-cache scan),
     * 4 = 3 with the scan staged through LDS tiles shared by the workgroup, 5 = 4 with one ray
     * per lane per iteration (shadow ray, then path ray: no empty ray slots), 6 = 3 compiled
     * for 6 waves per SIMD, 10 = 4 with the workgroup's rays pooled in LDS and scanned in
     * 64-ray passes (7, 8 and 9 are not schedules: the BVH wavefront form that held 9 was
     * measured 2.8x slower than the BVH path kernel and removed in round 4).  Every schedule
     * produces bit-identical frames. */
    int32_t kernel_variant;
    /* Acceleration structure: RVCP_ACCEL_NONE (default) scans every triangle like the
     * shader (bit-exact, the parity path).  RVCP_ACCEL_BVH (opt-in, games101 only) builds a
     * bounding-volume hierarchy at upload and tests only the triangles whose (slightly
     * enlarged) boxes the ray reaches, with the same exact triangle test and nearest-hit
     * rule; frames match the brute-force ones except where a ray runs almost parallel to a
     * triangle's plane.  With specialize = AUTO, a mesh whose leading faces
     * (at most 64) are all large -- a room around many small triangles, as C5 -- keeps those
     * faces out of the BVH and tests them first with the scene-specialised scan (the BVH
     * hybrid; stats report RVCP_VARIANT_SPECIALIZED). */
    int32_t accel;
    /* GPUs one context drives (0 or 1 = one).  With n_gpus = N > 1, rvcp_create opens devices
     * device, device+1, ... (mod the device count), rvcp_upload_scene uploads to all of them,
     * and rvcp_render deals the frame's 8-row stripes round-robin over them (stripe s -> GPU
     * s mod N), renders all shards concurrently and copies each shard's stripes into the frame
     * on `device` with one strided peer copy per shard (xGMI); the frame is bit-identical to
     * a 1-GPU render.  The single-process form of SURVEY.md §8(e); one process per GPU with
     * rvcp_render_shard_async + an RCCL gather (bench.py) is the other. */
    int32_t n_gpus;
    /* Float -> UNORM8 conversion of the stored colour (imageStore to the R8G8B8A8/B8G8R8A8
     * UNORM image, ray_tracer_games101_branch.comp:500, ray_tracer.comp:822,
     * mandelbrot.comp:33).  RVCP_UNORM_DRIVER (0, default): the conversion the reference's
     * driver performed, measured on its own render Notes/README/fractal.png (every one of its
     * 1,048,576 pixels reproduced): u8 = (floor(4096 x) * 255 + 2048) >> 12.
     * RVCP_UNORM_NEAREST (1): round-to-nearest, u8 = floor(255 x + 1/2). */
    int32_t unorm_rule;
    /* Scene-specialised scan: RVCP_SPECIALIZE_AUTO (0, default) compiles, at
     * rvcp_upload_scene, path kernels whose triangle scan is written out for the uploaded
     * scene (games101 integrator, brute force, at most 64 faces; hipRTC, ~1 s once per scene
     * and process) and uses them for schedules 3 and 6 when ray_t_min > 0 (and, with accel =
     * BVH, for the BVH hybrid's leading faces).  Frames are
     * bit-identical to the generic kernels; without hipRTC the generic kernels run.
     * RVCP_SPECIALIZE_OFF (1): always the generic kernels. */
    int32_t specialize;
    /* Persistent grid of one frame's path kernel, in waves per SIMD: 0 (default) = every
     * resident slot the kernel's occupancy allows; N > 0 caps it at N waves per SIMD (never
     * above the occupancy).  A pixel is a serial chain of SPP samples, so a frame ends with a
     * tail in which lanes whose pixels are done wait for the last chains; a caller that keeps
     * F > 1 frames in flight on F contexts can leave room for the next frame's waves so that
     * they start in that tail.  No effect on the frame's bits. */
    uint32_t grid_waves_per_simd;
} rvcp_config_t;

/* Per-render statistics (all optional). */
typedef struct rvcp_stats {
    double kernel_ms;                 /* device time of the render kernel(s), HIP events */
    uint64_t traversals;              /* scene traversals the reference algorithm performs
                                         (get_intersection_with_scene calls) */
    uint64_t traversals_executed;     /* traversals this kernel actually ran (primary hits
                                         are reused across a pixel's samples) */
    uint64_t samples;                 /* pixels * spp */
    uint32_t faces;                   /* F, triangles tested per traversal */
    int32_t kernel_variant;           /* the kernel schedule that ran (rvcp_config_t::
                                         kernel_variant resolved; 7 = BVH path kernel,
                                         8 = RVCP_INTEGRATOR_LEGACY kernel, 0 = none), plus
                                         RVCP_VARIANT_SPECIALIZED when the scene-specialised
                                         path kernel ran */
    uint64_t wave_iterations;         /* wave-level trace iterations; lane utilisation of the
                                         scan = traversals_executed / (64 * wave_iterations) */
    double main_kernel_ms;            /* device time of the dominant (path-tracing) kernel
                                         alone, HIP events on the launch stream; kernel_ms
                                         also covers the primary pre-pass and counter reset */
    double shader_clock_ghz;          /* the shader clock that kernel ran at: its waves'
                                         s_memtime ticks over their s_memrealtime (100 MHz)
                                         ticks, start to end, summed; 0 when not measured
                                         (schedules 1 / 2, trivial frames) */
} rvcp_stats_t;

#define RVCP_VARIANT_SPECIALIZED 16

/* Layout checks: sizes/offsets the reference's Rust structs and std140/std430 blocks imply. */
#ifdef __cplusplus
#define RVCP_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define RVCP_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif
RVCP_STATIC_ASSERT(sizeof(rvcp_camera_t) == 64, "AlignedCamera is 64 B");
RVCP_STATIC_ASSERT(offsetof(rvcp_camera_t, forward) == 32, "Camera.forward @32");
RVCP_STATIC_ASSERT(offsetof(rvcp_camera_t, t_near) == 44, "Camera.t_near @44");
RVCP_STATIC_ASSERT(offsetof(rvcp_camera_t, vertical_fov) == 52, "Camera.vertical_fov @52");
RVCP_STATIC_ASSERT(sizeof(rvcp_push_constant_t) == 68, "PushConstant is 68 B");
RVCP_STATIC_ASSERT(offsetof(rvcp_push_constant_t, time) == 64, "PushConstant.time @64");
RVCP_STATIC_ASSERT(sizeof(rvcp_material_t) == 32, "AlignedMaterial is 32 B");
RVCP_STATIC_ASSERT(offsetof(rvcp_material_t, ty) == 12, "Material.ty @12");
RVCP_STATIC_ASSERT(offsetof(rvcp_material_t, refraction_ratio) == 20, "Material.ior @20");
RVCP_STATIC_ASSERT(sizeof(rvcp_vertex_t) == 32, "AlignedVertex is 32 B");
RVCP_STATIC_ASSERT(offsetof(rvcp_vertex_t, normal) == 16, "Vertex.normal @16");
RVCP_STATIC_ASSERT(sizeof(rvcp_face_t) == 16, "AlignedFace is 16 B");
RVCP_STATIC_ASSERT(sizeof(rvcp_sphere_t) == 32, "AlignedSphere is 32 B");
RVCP_STATIC_ASSERT(sizeof(rvcp_lengths_t) == 24, "LengthBuffer is 24 B");
RVCP_STATIC_ASSERT(sizeof(rvcp_mandelbrot_push_t) == 12, "Mandelbrot CameraData is 12 B");

typedef struct rvcp_ctx rvcp_ctx_t;

/* Error codes */
#define RVCP_OK               0
#define RVCP_E_INVALID      (-1)   /* bad argument */
#define RVCP_E_HIP          (-2)   /* HIP runtime error */
#define RVCP_E_NO_SCENE     (-3)   /* render before upload */
#define RVCP_E_UNSUPPORTED  (-4)
#define RVCP_E_NOMEM        (-5)   /* host or device allocation failed */
#define RVCP_E_INTERNAL     (-6)   /* unexpected internal error (caught at the ABI boundary) */
#define RVCP_E_TIMEOUT      (-7)   /* a collective did not complete within the deadline
                                    * (rvcp_rccl_set_timeout): a peer rank is missing or failed;
                                    * the context's own communicator has been aborted */
#define RVCP_E_BUSY         (-8)   /* rvcp_rccl_init refused: the context's previous creation
                                    * timed out and its worker is still blocked inside RCCL */

/* ABI revision of this header, returned by rvcp_abi_version().  2 (round 6): rvcp_stats_t grew
 * from 56 to 64 bytes (shader_clock_ghz), RVCP_E_TIMEOUT / RVCP_E_BUSY, rvcp_abi_version and the
 * code-cache entry points.  A caller compiled against another revision must not pass its
 * rvcp_stats_t ("ABI revisions"). */
#define RVCP_ABI_VERSION 2

/* ---------------------------------------------------------------------------------------
 * Entry points
 * ------------------------------------------------------------------------------------- */

/* Library version string. */
const char *rvcp_version(void);

/* RVCP_ABI_VERSION of the header the library was built with: a caller checks it against its
 * own before passing structs (rvcp_stats_t changed size between revisions 1 and 2). */
uint32_t rvcp_abi_version(void);

/* On-disk cache of the scene-specialised code objects: rvcp_upload_scene
 * compiles a module per scene with hipRTC (~0.7 s); with a cache directory the code object is
 * stored under a key that covers the generated source, the kernel source, the compile options
 * and the hipRTC version, and a later process that uploads the same scene loads it instead.
 * An entry is checked (header, key, length, checksum) before it is loaded; a damaged or
 * foreign entry is recompiled and rewritten, never trusted.  The checksum detects damage, not
 * tampering: the directory is trusted like the user's own files (as any JIT cache is), so it
 * must not be writable by others (the library creates it 0700).  The reference has no counterpart
 * (its SPIR-V is compiled into the binary, src/ray_tracer/shader.rs:9-14).
 * dir: the directory (created if missing); NULL or "" disables the cache.  Default:
 * $XDG_CACHE_HOME/rvcp-mi355x, else $HOME/.cache/rvcp-mi355x (the only environment the product
 * library reads).  Process-wide. */
int rvcp_set_code_cache_dir(const char *dir);

/* Counters of the on-disk cache since the process started: out[0] modules loaded from disk,
 * out[1] modules compiled (and stored), out[2] entries rejected (damaged / foreign / unloadable)
 * and recompiled. */
int rvcp_code_cache_counts(uint64_t out[3]);

/* Fill `cfg` with the reference's #define defaults.  Replaces nothing (the reference bakes
 * them into the SPIR-V at `vulkano_shaders::shader!`, src/ray_tracer/shader.rs:9-14). */
int rvcp_config_default(rvcp_config_t *cfg);

/* Same, for integrator `integrator` (RVCP_INTEGRATOR_*): the #defines of the shader that
 * integrator restates (ray_tracer_games101_branch.comp:5-13 or ray_tracer.comp:5-13).
 * RVCP_E_UNSUPPORTED for an unknown integrator. */
int rvcp_config_default_for(int32_t integrator, rvcp_config_t *cfg);

/* Create a context on cfg->device.  Replaces pipeline creation:
 * `Vk::create_compute_pipeline(device, ray_tracer_shader::load(device))`,
 * src/ray_tracer/vulkan.rs:576-603 (called at :239-242). */
int rvcp_create(const rvcp_config_t *cfg, rvcp_ctx_t **out_ctx);

/* Free the context and all device memory it owns. */
int rvcp_destroy(rvcp_ctx_t *ctx);

/* Last error message for `ctx` ("" if none).  ctx may be NULL (global create errors). */
const char *rvcp_last_error(const rvcp_ctx_t *ctx);

/* Upload a scene.  Replaces `Vk::create_descriptor_set_0s`, src/ray_tracer/vulkan.rs:454-574
 * (bindings 1 LengthBuffer, 2 MaterialBuffer, 4 VertexBuffer, 5 FaceBuffer,
 * 7 LuminousFaceIdBuffer).  `lum_face_ids` are the packed u32 ids the host computes at
 * vulkan.rs:473-478; the std140 quirk is applied inside.  Spheres (binding 3) are traced by
 * RVCP_INTEGRATOR_LEGACY and ignored by games101; luminous sphere ids (binding 6) are read
 * by neither integrator's dispatched path and may be NULL/0.  Face vertex indices and
 * material ids are validated (the reference does not bound-check; out-of-range ids are an
 * error). */
int rvcp_upload_scene(rvcp_ctx_t *ctx,
                      const rvcp_material_t *materials, uint32_t n_materials,
                      const rvcp_vertex_t *vertices, uint32_t n_vertices,
                      const rvcp_face_t *faces, uint32_t n_faces,
                      const rvcp_sphere_t *spheres, uint32_t n_spheres,
                      const uint32_t *lum_face_ids, uint32_t n_lum_face_ids,
                      const uint32_t *lum_sphere_ids, uint32_t n_lum_sphere_ids);

/* Load a binary scene file (.rvcpscn: "RVCPSCN1" header, rvcp_lengths_t, rvcp_camera_t,
 * then the upload arrays in the layouts above; format in scene_io.py) and upload it as
 * rvcp_upload_scene would.  The camera stored in the file is copied to *out_camera when
 * non-NULL.  Replaces the reference's compiled-in scene (`Scene::default`,
 * src/ray_tracer/scene/mod.rs:21) as the way to feed large meshes.
 * RVCP_E_INVALID for an unreadable, truncated or malformed file. */
int rvcp_upload_scene_file(rvcp_ctx_t *ctx, const char *path, rvcp_camera_t *out_camera);

/* Render one full frame synchronously into host memory.  Replaces the per-frame
 * `push_constants(...)` + `dispatch([W/8, H/8, 1])` + present of vulkan.rs:406-452 and
 * :298-404.  out_rgba8: W*H*4 bytes, row-major, logical RGBA (the reference's swapchain was
 * B8G8R8A8_UNORM, records/swapchain_image.txt:8), alpha 255.  out_linear_rgb (optional):
 * W*H*3 floats, the pre-clamp, pre-gamma `color` of ray_tracer_games101_branch.comp:497
 * (ray_tracer.comp:819 for RVCP_INTEGRATOR_LEGACY, whose RGBA8 store has no gamma).
 * Unlike the reference, W and H need not be multiples of 8 (every pixel is rendered). */
int rvcp_render(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push,
                uint32_t width, uint32_t height,
                uint8_t *out_rgba8, float *out_linear_rgb, rvcp_stats_t *stats);

/* The reference's second compute operator, assets/shaders/mandelbrot.comp (dispatched by
 * src/mandelbrot/vulkan.rs:380-400 with CameraData {position, scale}; defaults [0, 0] and 1.0,
 * src/mandelbrot/config.rs:11-12).  Writes the W x H grey RGBA8 frame (escape time i,
 * UNORM8, alpha 255) and optionally the float i per pixel.  Synchronous, like rvcp_render;
 * needs no scene.  stats (optional) gets kernel_ms only. */
int rvcp_mandelbrot(rvcp_ctx_t *ctx, const rvcp_mandelbrot_push_t *push,
                    uint32_t width, uint32_t height,
                    uint8_t *out_rgba8, float *out_value, rvcp_stats_t *stats);

/* Asynchronous shard render into device memory, for multi-GPU frame assembly.
 * The frame is cut into 8-row stripes (the reference's 8x8 workgroup rows); stripe s is
 * rendered by shard (s % shard_count).  This call renders the stripes of `shard_index`
 * and packs them contiguously, in increasing stripe order, into d_rgba8
 * (rvcp_shard_rows(H, idx, count) * W * 4 bytes) and optionally d_linear_rgb (rows*W*3
 * floats).  Pixel values are bit-identical to a single-GPU render of the whole frame.
 * Enqueued on `stream`; stats->kernel_ms/traversals are filled by rvcp_sync_stats(). */
int rvcp_render_shard_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push,
                            uint32_t width, uint32_t height,
                            uint32_t shard_index, uint32_t shard_count,
                            void *d_rgba8, void *d_linear_rgb, void *stream);

/* A batch of n_frames consecutive frames of one shard (frame k rendered with pushes[k]: its
 * camera and its time seed), enqueued as one unit on `stream`.  The swapchain loop of
 * vulkan.rs:367-369, 392-401 keeps one frame per swapchain image in flight; here the frames
 * of a batch share one surface list and one persistent path kernel, so lanes whose pixels of
 * frame k are done take pixels of frame k+1 while the last sample chains of frame k finish
 *  -- frames in flight at lane granularity instead of wave granularity.
 * Layout: frame k's packed shard rows start at pixel k * S of d_rgba8 (and of d_linear_rgb,
 * 3 floats per pixel, optional), S = rvcp_shard_rows(height, 0, shard_count) * width, the
 * largest shard's pixels (for a smaller shard the rows after its own are padding and hold
 * unspecified values); with shard_count = 1, S = W*H and the frames are simply consecutive.
 * Every frame is bit-identical to rvcp_render_shard_async with the same push.  One pending
 * batch per context; rvcp_sync_stats covers the whole batch (samples = n_frames x shard
 * pixels x spp).  Integrator mode 2 (RVCP_INTEGRATOR_LEGACY) has no pre-pass: its one kernel
 * queues the batch's pixels frame after frame, reading each frame's camera and time from a
 * table the call uploads.  Needs a one-GPU context and, for games101, a pre-pass schedule (the
 * automatic ones: 3-6, 10, the BVH path kernel); schedules 1 and 2 return
 * RVCP_E_UNSUPPORTED unless n_frames = 1. */
int rvcp_render_frames_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *pushes,
                             uint32_t n_frames, uint32_t width, uint32_t height,
                             uint32_t shard_index, uint32_t shard_count,
                             void *d_rgba8, void *d_linear_rgb, void *stream);

/* Wait for the last async render of ctx and fetch its statistics.  It waits for the render
 * only: a gather enqueued behind it (rvcp_gather_frame_async) needs rvcp_gather_wait before
 * rank 0's assembled frame may be read. */
int rvcp_sync_stats(rvcp_ctx_t *ctx, rvcp_stats_t *stats);

/* The asynchronous pair of SURVEY.md §8(b) (the reference's per-image fences,
 * vulkan.rs:367-369, 392-401): enqueue one full frame into DEVICE memory on `stream` (NULL:
 * the context's own stream) and return; rvcp_wait blocks until it is done and fills stats.
 * d_rgba8: W*H*4 bytes, d_linear_rgb (optional): W*H*3 floats, as rvcp_render.  Equivalent to
 * rvcp_render_shard_async(..., 0, 1, ...) / rvcp_sync_stats.  One GPU: a context with
 * n_gpus > 1 returns RVCP_E_UNSUPPORTED (use rvcp_render). */
int rvcp_render_async(rvcp_ctx_t *ctx, const rvcp_push_constant_t *push,
                      uint32_t width, uint32_t height,
                      void *d_rgba8, void *d_linear_rgb, void *stream);
int rvcp_wait(rvcp_ctx_t *ctx, rvcp_stats_t *stats);

/* Rows of an H-row frame owned by shard `shard_index` of `shard_count`. */
uint32_t rvcp_shard_rows(uint32_t height, uint32_t shard_index, uint32_t shard_count);

/* Assemble a frame on the device from gathered shard buffers.  d_gathered holds
 * shard_count slots of `slot_rows` rows (slot_rows >= max shard rows) each, shard k's
 * packed stripes at slot k.  Writes the W x H RGBA8 frame to d_frame.  Enqueued on stream. */
int rvcp_assemble_frame_async(rvcp_ctx_t *ctx, const void *d_gathered, uint32_t slot_rows,
                              uint32_t width, uint32_t height, uint32_t shard_count,
                              void *d_frame, void *stream);

/* ---------------------------------------------------------------------------------------
 * One process per GPU: every rank renders its stripes with
 * rvcp_render_shard_async(ctx, ..., rank, world, d_shard, ...) into a shard buffer of
 * rvcp_shard_rows(H, 0, world) rows (shard 0 has the most rows; shorter shards send padding),
 * then rvcp_gather_frame_async gathers the shards to rank 0 with one RCCL ncclGather over
 * xGMI and assembles the frame there on the device.  The reference is single-device
 * (src/ray_tracer/vulkan.rs:145-193 picks one physical device); this replaces nothing in it
 * and adds the multi-GPU form north_star asks for.  RCCL is loaded at run time
 * (librccl.so.1: the copy the process already holds, e.g. PyTorch-ROCm's, else the system
 * one); without it these return RVCP_E_UNSUPPORTED.
 * ------------------------------------------------------------------------------------- */
#define RVCP_RCCL_ID_BYTES 128     /* sizeof(ncclUniqueId) */

/* Rank 0: create the communicator id (ncclGetUniqueId) to hand to every rank by any
 * out-of-band channel (MPI, a TCP store, torch.distributed's broadcast). */
int rvcp_rccl_unique_id(uint8_t out_id[RVCP_RCCL_ID_BYTES]);

/* Every rank, collectively: create ctx's communicator (non-blocking ncclCommInitRankConfig on
 * ctx's device, polled with ncclCommGetAsyncError).  Returns once all `world` ranks have
 * joined, or RVCP_E_TIMEOUT when they have not within the context's deadline.  The creation
 * runs on a worker thread, because RCCL's "non-blocking" creation call itself does not return
 * while a peer is absent: on a timeout the worker is left behind (it aborts the half-made
 * communicator if RCCL ever returns), the message counts such workers in the process, and the
 * context refuses a further rvcp_rccl_init with RVCP_E_BUSY while its worker is still blocked --
 * at most one blocked worker per context; the context stays usable for single-GPU renders (and
 * rvcp_rccl_attach).  Destroyed with the context.  The reference has no counterpart (single device); its own
 * recover-not-hang path is the swapchain's OutOfDate -> recreate (src/ray_tracer/vulkan.rs:
 * 355-364). */
int rvcp_rccl_init(rvcp_ctx_t *ctx, const uint8_t id[RVCP_RCCL_ID_BYTES], uint32_t world,
                   uint32_t rank);

/* Deadline of rvcp_rccl_init and rvcp_gather_wait (and of the wait for a pending gather in
 * rvcp_destroy), in milliseconds; 0 = wait forever.  Default 60000.  It must exceed the
 * render time of the frames a gather waits behind. */
int rvcp_rccl_set_timeout(rvcp_ctx_t *ctx, uint32_t timeout_ms);

/* Use the caller's existing communicator (an ncclComm_t over ctx's device, rank `rank` of
 * `world`) instead; the caller keeps ownership (and is the one to abort it).  A non-blocking
 * communicator (ncclConfig_t.blocking = 0) is supported: a gather that returns ncclInProgress
 * is polled until it is on the stream, bounded by the deadline. */
int rvcp_rccl_attach(rvcp_ctx_t *ctx, void *nccl_comm, uint32_t world, uint32_t rank);

/* Every rank, collectively, after its rvcp_render_shard_async on the same stream: gather the
 * shards to rank 0 (ncclGather, root 0, shard k at slot k of d_gathered) and, on rank 0,
 * assemble the W x H RGBA8 frame into d_frame.  d_shard_rgba8: rvcp_shard_rows(H, 0, world)
 * * W * 4 bytes on every rank; d_gathered (world times that) and d_frame (W*H*4 bytes) are
 * needed on rank 0 only (NULL elsewhere).  Enqueued on `stream`, behind the caller's own
 * ordering; with stream = NULL on ctx's gather stream (highest priority), after the
 * preceding render by an event, and the next render on ctx waits for the gather by an event,
 * so the render stream is free for the next frame meanwhile.  The frame is bit-identical to
 * a single-GPU render.  The preceding render on ctx must have been
 * shard_index = rank, shard_count = world of the same W x H frame (else RVCP_E_INVALID). */
int rvcp_gather_frame_async(rvcp_ctx_t *ctx, const void *d_shard_rgba8, uint32_t width,
                            uint32_t height, void *d_gathered, void *d_frame, void *stream);

/* Wait for ctx's last rvcp_gather_frame_async and report its device time (ncclGather plus, on
 * rank 0, the assembly) in *gather_ms and, if frame_ms is not NULL, the time from the start of
 * the preceding render to the end of the gather in *frame_ms (HIP events on the gather's
 * stream).  RVCP_E_INVALID when no gather was enqueued since the last call.  The wait polls
 * against the context's deadline (rvcp_rccl_set_timeout): when the gather has not finished by
 * then -- a peer rank never entered it -- or RCCL reports an asynchronous error, the
 * context's communicator is aborted (ncclCommAbort; its kernels exit) and RVCP_E_TIMEOUT
 * (resp. RVCP_E_HIP) is returned; rvcp_rccl_init may then build a new one.  An attached
 * communicator is not aborted (it is the caller's) but dropped.  When the gather's stream has
 * not drained (always the case for an attached communicator whose peer never comes), later
 * renders on ctx no longer wait for that gather, later gathers return RVCP_E_TIMEOUT until a
 * new communicator is initialised or attached (they then run on a fresh gather stream), and
 * rvcp_destroy waits for the stuck gather at most min(deadline, 10 s): past that it frees the
 * host side, leaks the context's device memory and streams (a hipFree would wait for the stuck
 * collective: HIP synchronises the device) and returns RVCP_E_TIMEOUT, with the message in
 * rvcp_last_error(NULL).
 * rvcp_sync_stats / rvcp_wait wait for the render only: rank 0's assembled frame (d_frame)
 * is complete after this call, not after theirs. */
int rvcp_gather_wait(rvcp_ctx_t *ctx, float *gather_ms, float *frame_ms);

#ifdef __cplusplus
}
#endif

#endif /* RVCP_H */
