// rvcp_internal.h -- device-side data layout shared by the host runtime (rvcp_host.cpp) and
// the gfx950 kernels (rvcp_kernels.hip).  Not part of the C-ABI.
#pragma once

#ifndef __HIPCC_RTC__             // hipRTC (rvcp_jit.cpp) provides the fixed-width types
#include <stdint.h>

#include <vector>
#else
using __hip_internal::int32_t;
using __hip_internal::uint8_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

namespace rvcp {

// Wave width on CDNA4.
constexpr int kWave = 64;
// Threads per workgroup of the path-tracing kernel (4 independent waves).
constexpr int kBlock = 256;
// schedule 10 (LDS-tiled scan with the workgroup ray pool): waves per workgroup
#ifndef RVCP_TILED_POOL_WAVES
#define RVCP_TILED_POOL_WAVES 8
#endif
constexpr int kTiledPoolWaves = RVCP_TILED_POOL_WAVES;
// LDS state columns of the path kernels (path_body LDS_STATE): a_p 0-2, nee_C 3-5, nee_dist 6,
// acc 7-9, att 10-12, col 13-15
constexpr int kStateCols = 16;
// Pixels a wave takes from the frame queue per atomic.
constexpr uint32_t kChunk = 64;
// Small frames: the grid is sized so that a wave starts with at least kMinStatic pixels, and
// the pixels are spread over all those waves (more waves per SIMD to hide latency).
constexpr uint32_t kMinStatic = 8;
// Frame-queue grabs after a wave's static chunk: what the wave consumes in kChunkWindow
// s_memrealtime ticks (100 MHz), between kMinChunk and kDynChunk pixels (queue_take,
// DESIGN.md §4.1).
constexpr uint32_t kDynChunk = 64;
constexpr uint32_t kMinChunk = 2;
constexpr uint32_t kChunkWindow = 10000;    // 100 us
// Kernel schedules (rvcp_config_t::kernel_variant): 1 = one ray per lane per iteration,
// 2 = shadow + continuation ray per lane per iteration, 3 = primary pre-pass kernel + the
// variant-2 loop over surface pixels only.
// 4 = variant 3 with the triangle scan staged through LDS tiles shared by the workgroup
// (the automatic choice for meshes of kTiledMinFaces faces or more on frames of
// kTiledDualMinSamples pixel-samples or more).
// 5 = variant 4 with one ray per lane per iteration (the shadow ray, then the path ray), so no
// ray slot is empty; the automatic choice for large meshes on smaller frames, whose rays do not
// fill the chip twice over.
// 6 = variant 3 compiled for 6 waves per SIMD instead of 5 (80 VGPRs, a few spills): faster
// once the frame is large enough that latency hiding beats the spills (automatic from
// kWideMinSamples pixel-samples per frame).
// 10 = variant 4 with the workgroup ray pool: the rays of a workgroup of kTiledPoolWaves waves
// are scanned against each LDS tile in 64-ray passes shared out over its waves (the automatic
// choice wherever 4 was).  (7 and 8 are the stats codes of the BVH and mode-2 kernels, 9 is
// unused: a non-tiled pool measured slower)
constexpr int kDefaultVariant = 3;
constexpr int kMaxVariant = 10;
// d_counters (u64 words): executed traversals, queue head, wave iterations, surface-list
// length, and at kClockWord (a cache line of its own) the path kernel's clock stamps
// (shader-clock ticks, 100-MHz ticks; clock_stamp in rvcp_kernels.hip)
constexpr int kCounterWords = 32;
constexpr int kClockWord = 16;
constexpr int kTiledPoolVariant = 10;
constexpr int variant_block(int v) { return v == kTiledPoolVariant ? kTiledPoolWaves * kWave : kBlock; }
constexpr uint64_t kWideMinSamples = 8ull << 20;   // auto: variant 6 from 8 Msamples per frame
// auto, scene-specialised scan: its 6-wave build (variant 6) from 256 Msamples per frame -- C4's
// 2048^2 SPP=64 frame 23.39 -> 23.00 ms, while C3 (31 M) is 0.3 % and C2 6 % slower at 6 waves
// (profiles/history/r04z_ab_waves6.log)
// A batch's pre-passes run as one launch (one frame per grid row) for frames up to this many
// pixels, whose per-frame pre-pass is too small to fill the GPU (C2: 0.1666 -> 0.1645 ms per
// frame); larger frames keep one launch per frame (C3 at 60 frames: 2.810 vs 2.827 ms,
// profiles/history/r04pb_ab_prebatch.log).
constexpr uint32_t kPrepassBatchMaxPixels = 512u * 1024u;
constexpr uint64_t kSpecWideMinSamples = 256ull << 20;
constexpr int kOccupancyBvh = 100;          // rvcp_games101_occupancy code of the BVH kernel
#ifndef RVCP_TILE
#define RVCP_TILE 256
#endif
constexpr uint32_t kTile = RVCP_TILE;       // triangles per LDS tile (12 KiB at 256)
constexpr uint64_t kTiledDualMinSamples = 1ull << 19;   // auto: variant 4 rather than 5 from here
                                            // (4 wins at 512x512x4, 5 at 256x256x4)
constexpr uint32_t kTiledWideMinFaces = 64;   // auto: variant 4 above this many faces on
                                            // frames of kTiledDualMinSamples or more (F = 72:
                                            // 4 beats 3 and 6 from 2 Msamples)
constexpr uint32_t kTiledMinFaces = 256;   // auto: variant 5 from here (measured crossover
                                            // vs variant 3 at ~230 faces)

// One triangle as the brute-force scan reads it: v0, e1 = v1 - v0, e2 = v2 - v0, computed on
// the host with the same float subtractions the shader performs per test
// (ray_tracer_games101_branch.comp:247-248), so the scan is bit-identical while reading
// 36 algorithmic bytes per test.  Padded to 48 B (three 16-B rows).
struct alignas(16) TriRecord {
    float v0[3];
    float e1[3];
    float e2[3];
    float pad[3];
};
static_assert(sizeof(TriRecord) == 48, "TriRecord is 48 B");

// Scenes up to this many faces get the scene-specialised scan (rvcp_jit.cpp; the unrolled code
// grows with the face count, and the specialised kernels keep the scene in LDS arrays of this
// size).
constexpr uint32_t kJitMaxFaces = 64;

// One entry of the light table: a luminous face as sample_light_games101 sees it
// (ray_tracer_games101_branch.comp:384-404), with the std140 id quirk already applied.
struct alignas(16) LightRecord {
    float cum;          // running emit_area_sum after this entry (second loop, :396-399)
    uint32_t face;      // face index
    float pad0[2];
    float v0[4];        // positions of the face's three vertices (sample_in_face :315-317)
    float v1[4];
    float v2[4];
    float n[4];         // normalize(vertices[face.x].normal)  (:325)
    float le[4];        // materials[face.material_id].albedo  (:437)
};
static_assert(sizeof(LightRecord) == 96, "LightRecord is 96 B");

// A pixel whose primary ray hit a non-emissive surface, as the primary pre-pass hands it to
// the path kernel (variant 3): the cached primary hit record (:421-431 at depth 0) and the
// pixel's RNG seed.
struct alignas(16) SurfRecord {
    float pos[3];
    uint32_t pix;
    float nrm[3];
    float seed;         // srand's seed of the pixel (:153-155), computed once by the pre-pass
    float alb_pi[3];    // albedo / pi of the hit material
    uint32_t mat;
};
static_assert(sizeof(SurfRecord) == 48, "SurfRecord is 48 B");

// Per-face shading data, gathered by index once per traversal for the nearest face only:
// the three vertex normals (interpolated at :262-266), the face material (:272) with its type
// and albedo / PI.  One independent 64-B gather instead of face -> vertices -> material.
struct alignas(16) FaceShade {
    float n0[3];
    uint32_t mat;
    float n1[3];
    uint32_t ty;
    float n2[3];
    uint32_t pad0;
    float alb_pi[3];
    uint32_t pad1;
};
static_assert(sizeof(FaceShade) == 64, "FaceShade is 64 B");

// Per-material record: albedo + type (MaterialBuffer, :74-83) and albedo / PI, the value
// lambertian_brdf_eval returns (:346), divided once on the host with the same float division.
struct alignas(16) MatRecord {
    float albedo[3];
    uint32_t ty;
    float alb_pi[3];
    uint32_t pad;
};
static_assert(sizeof(MatRecord) == 32, "MatRecord is 32 B");

// Opt-in BVH (rvcp_config_t.accel = RVCP_ACCEL_BVH).  The builder makes a binary tree whose
// nodes hold both children's boxes; child reference: >= 0 an internal node, < 0 a leaf
// ~ref = first << 5 | (count - 1) over the leaf-ordered triangle array.  Boxes are enlarged at
// build time (bvh_build) so that a triangle the exact test accepts is never culled by rounding
// in the box test.  The device traverses the 4-wide tree bvh4_collapse makes of it.
struct alignas(16) BvhNode {
    float lbox[6];      // left child: lo xyz, hi xyz
    float rbox[6];      // right child
    int32_t left, right;
    int32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode is 64 B");
// at most this many triangles per BVH leaf: 2 since round 5 -- with the node-phase break
// (rvcp_kernels.hip) the 4-triangle leaves' tests cost more than the extra node steps of 2
// (C5 BVH 52.0 -> 47.0 ms; 1: 46.5 ms for 1.8x the nodes; profiles/history/r05zc_ab_bvhleaf.log,
// r05zd_ab_bvhleaf2.log)
#ifndef RVCP_BVH_LEAF_MAX
#define RVCP_BVH_LEAF_MAX 2
#endif
constexpr int kBvhLeafMax = RVCP_BVH_LEAF_MAX;
constexpr uint32_t kBvhPadId = 0xFFFFFFFFu;   // padding slot of the leaf order (even leaf starts)
constexpr int kBvhStack = 32;           // traversal stack entries per lane

// The traversed tree: up to 4 children per node, boxes stored per axis so one node is seven
// 16-byte loads; a step tests the four boxes, pushes the hit children but the nearest (farthest
// first) and descends into the nearest.  Unused child slots hold an unreachable box (a point
// at 3e38) and the leaf reference ~0 (triangle 0 again: a repeated test never changes the hit).
struct alignas(16) Bvh4Node {
    float lo[3][4];     // lo[axis][child]
    float hi[3][4];
    int32_t ref[4];
    int32_t pad[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node is 128 B");

// The same node with its child boxes quantised to bytes (bvh4_quantize): per axis the children's
// bounds are origin + q * scale with scale a power of two, lo rounded down and hi up (so every
// box contains its Bvh4Node box); byte c of qlo[axis] / qhi[axis] is child c.  Unused children
// are inverted (qlo = 255, qhi = 0), which the ordered slab test never enters.  64 B: four
// 16-B loads per traversal step instead of seven.
struct alignas(16) Bvh4QNode {
    float origin[3];
    float scale[3];
    uint32_t qlo[3];
    uint32_t qhi[3];
    int32_t ref[4];
};
static_assert(sizeof(Bvh4QNode) == 64, "Bvh4QNode is 64 B");

// Frame-constant parameters of one render launch.
struct FrameArgs {
    // camera, precomputed on the host exactly as sample_ray (:217-235) computes it
    float cam_pos[3];
    float u[3];          // normalize(cross(fwd, up)) * w
    float v[3];          // normalize(cross(fwd, u)) * h
    float pos[3];        // cam_pos + fwd * t_near
    float base_len;      // length(pos - cam_pos)
    float t_near, t_far;
    float time;          // push-constant time (RNG seed input)
    uint32_t width, height;
    uint32_t shard_index, shard_count;
    uint32_t n_pixels;   // pixels owned by this shard (rows * width)
    uint32_t spp, max_bounces;
    float att_stop, t_min, t_max, rr, eps;
    uint32_t n_faces, n_lights;
    float light_total, light_pdf;
    // the BRDF update's divisor max(0.1, pdf) * rr (:465-471) for pdf = 1/(2 pi) (cos > 0) and
    // pdf = 0, and their IEEE reciprocals: frame constants, so the update divides by a known
    // reciprocal (divs_y) instead of computing rcp_ieee per event
    float brdf_den[2], brdf_rcp[2];
    // every light record samples the same face (the std140 id quirk on the Cornell box maps
    // both entries to face 0): nee_sample's pick cannot change the sample, so it reads record 0
    uint32_t lights_same;
    // every triangle's scan denominator is +-0 or within [2^-126, 2^126] for rays passing
    // dir_fast_ok (scan_rcp_fast_scene): the generic scans may take 1/den without the class check
    uint32_t rcp_fast;
    // the scene has a metal material (type 1): mode 2's scatter needs the reflected direction
    uint32_t has_metal;
    uint32_t static_chunks;  // pixels handed out statically (one chunk per wave)
    uint32_t static_chunk;   // pixels of each wave's static chunk (<= kChunk)
    uint32_t n_simds;        // SIMDs of the device (CUs x 4), for static_split
    uint32_t want_linear;
    int32_t variant;         // kernel schedule (rvcp_config_t::kernel_variant, resolved)
    uint32_t n_spheres;      // integrator RVCP_INTEGRATOR_LEGACY only
    uint32_t n_mats;
    uint32_t dyn_chunk;      // largest frame-queue grab after the static chunk
    uint32_t chunk_min;      // smallest grab
    uint32_t chunk_window;   // grab = pixels this wave consumes in chunk_window ticks (10 ns)
    int32_t accel;           // RVCP_ACCEL_*
    int32_t bvh_root;        // root reference (see BvhNode) when accel == RVCP_ACCEL_BVH
    uint32_t bvh_n4;         // Bvh4Node offset of the quantised nodes in the node buffer (0)
    uint32_t bvh_slots;      // TriRecord offset of the packed 10-float leaf records (0: buffer start)
    // faces [0, bvh_prefix) are not in the BVH: every ray tests them first, with the
    // scene-specialised scan where the module has one, else the generic test (the hybrid of
    // DESIGN.md §4.6); 0 = the BVH holds every face
    uint32_t bvh_prefix;
    // small frames (path kernels of schedules 3/6): when the surface list fits the resident
    // lanes, spread it over every resident wave, at least spread_min pixels each (0 = off),
    // and let waves with <= 32 rays split each ray's scan over R lanes from the first
    // iteration (early_tail), not only once the queue is empty
    uint32_t spread_min;
    uint32_t early_tail;
    // index of this frame's first pixel in the outputs (rvcp_render_frames_async: frame k of a
    // batch starts at k x the largest shard's pixels; 0 for a single frame)
    uint32_t pix_base;
    // integrator mode 2 batches (one kernel over n frames; rvcp_render_frames_async): queue
    // pixel p is pixel p % frame_pixels of frame p / frame_pixels, whose camera and time are
    // the 16 floats at batch_cams + 16 * frame (FrameCam order: cam_pos, u, v, pos, base_len,
    // t_near, t_far, time) and whose outputs start frame_stride pixels after the previous
    // frame's; batch_cams == nullptr for a single frame
    uint32_t frame_pixels, frame_stride;
    const float *batch_cams;
    // debug build of the library only: per-wave {start, queue exhausted, end, iterations,
    // shader-clock start, shader-clock end}
    // of the path kernel, s_memrealtime ticks (100 MHz); nullptr otherwise
    unsigned long long *timeline;
};

#ifndef __HIPCC_RTC__
// rvcp_bvh.cpp: build the BVH over n faces (three vertex positions each); returns the depth.
int bvh_build(const float (*pos)[3][3], uint32_t n, std::vector<BvhNode> &nodes,
              std::vector<uint32_t> &order, int32_t &root);
// Collapse the binary tree into the 4-wide one, keeping the traversal stack within
// kBvhStack entries; returns that stack bound.
int bvh4_collapse(const std::vector<BvhNode> &nodes, int32_t root, std::vector<Bvh4Node> &out,
                  int32_t &root4);
// rvcp_bvh.cpp: the byte-quantised copy of a collapsed tree (same indices and refs).
void bvh4_quantize(const std::vector<Bvh4Node> &in, std::vector<Bvh4QNode> &out);
// rvcp_bvh.cpp: how many leading faces are "big" (box extent above the split-clipping
// threshold: max(8 x the median extent, scene diagonal / 16)), at most `cap`; the hybrid tests
// them with the specialised scan and builds the BVH over the rest.
uint32_t bvh_big_prefix(const float (*pos)[3][3], uint32_t n, uint32_t cap);

#endif  // __HIPCC_RTC__
}  // namespace rvcp

#ifndef __HIPCC_RTC__
// Launchers (defined in rvcp_kernels.hip), called by rvcp_host.cpp.
extern "C" {
int rvcp_launch_games101(const rvcp::FrameArgs *args, const rvcp::TriRecord *tri,
                         const void *faces, const void *verts, const rvcp::MatRecord *mats,
                         const rvcp::LightRecord *lights, const float *gamma_t,
                         uint32_t *out_rgba, float *out_lin, unsigned long long *counters,
                         uint32_t grid_blocks, void *stream);
// args[0 .. n_frames): one FrameArgs per frame of the batch (pix_base = k x frame_stride);
// one pre-pass per frame into one surface list, one path kernel, one tone map over
// n_frames x frame_stride pixels (n_pixels when n_frames == 1).  spec_path_fn / spec_pre_fn:
// the scene-specialised path kernel and pre-pass (rvcp_jit.cpp), or null for the built-in ones
int rvcp_launch_games101_v3(const rvcp::FrameArgs *args, uint32_t n_frames, uint32_t frame_stride,
                            const rvcp::TriRecord *tri,
                            const void *faces, const void *verts, const rvcp::MatRecord *mats,
                            const rvcp::LightRecord *lights, const float *gamma_t,
                            uint32_t *out_rgba, float *out_lin, unsigned long long *counters,
                            rvcp::SurfRecord *surf, const rvcp::FaceShade *shade,
                            const rvcp::Bvh4Node *bvh_nodes, const rvcp::TriRecord *bvh_tris,
                            uint32_t grid_blocks, void *stream, void *main_event,
                            void *spec_path_fn, const float *cams, void *spec_pre_fn = nullptr);
// Integrator RVCP_INTEGRATOR_LEGACY (ray_tracer.comp): materials / spheres are the raw
// rvcp_material_t / rvcp_sphere_t arrays, unorm_t the UNORM8 threshold table.
int rvcp_launch_legacy(const rvcp::FrameArgs *args, const rvcp::TriRecord *tri,
                       const rvcp::FaceShade *shade, const void *spheres, const void *materials,
                       const float *unorm_t, uint32_t *out_rgba, float *out_lin,
                       unsigned long long *counters, uint32_t grid_blocks, void *stream,
                       void *spec_legacy_fn);
int rvcp_legacy_occupancy(int *blocks_per_cu);
// mandelbrot.comp (rvcp_mandelbrot.hip)
int rvcp_launch_mandelbrot(float pos_x, float pos_y, float scale, uint32_t width,
                           uint32_t height, const float *unorm_t, uint32_t *out_rgba,
                           float *out_value, void *stream);
int rvcp_launch_assemble(const uint32_t *gathered, uint32_t slot_rows, uint32_t width,
                         uint32_t height, uint32_t shard_count, uint32_t *frame, void *stream);
int rvcp_launch_fill(uint32_t *out_rgba, float *out_lin, uint32_t n_pixels, uint32_t rgba,
                     void *stream);
int rvcp_games101_occupancy(int variant, int *blocks_per_cu);
void rvcp_static_split(uint32_t n, uint32_t grid_waves, uint32_t n_simds, uint32_t *waves,
                       uint32_t *chunk);
}
#endif  // __HIPCC_RTC__
