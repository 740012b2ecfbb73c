// rvcp_jit.h -- scene-specialised path kernels compiled at upload with hipRTC (rvcp_jit.cpp,
// DESIGN.md §4.7).  Host-side only; not part of the C-ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/rvcp.h"
#include "rvcp_internal.h"

namespace rvcp {

struct JitKernels {
    int device = 0;
    hipModule_t module = nullptr;
    hipFunction_t path5 = nullptr;     // schedule 3 (5 waves per SIMD)
    hipFunction_t path6 = nullptr;     // schedule 6 (6 waves per SIMD)
    hipFunction_t legacy = nullptr;    // integrator mode 2 (modules compiled with `legacy`)
    hipFunction_t primary = nullptr;   // the schedule-3/6 pre-pass with the specialised scan
    // the BVH hybrid (modules compiled with `bvh`): the BVH path kernel and pre-pass, the scan
    // covering the scene's first FrameArgs::bvh_prefix faces
    hipFunction_t bvh_path = nullptr, bvh_primary = nullptr;
    int blocks_per_cu5 = 0, blocks_per_cu6 = 0, blocks_per_cu_legacy = 0, blocks_per_cu_bvh = 0;
    // fnv1a of the module's whole compile input (hipRTC version, options, embedded sources,
    // generated scan): the disk-cache key, and the identity bench.py binds PMC summaries to
    uint64_t key_hash = 0;
    ~JitKernels();
};

// Every |v0| <= 2^40 and |e1|, |e2| <= 2^41 (finite): the range in which dropping the products
// with exact-zero components cannot turn the generic test's inf * 0 = NaN into a finite value.
bool jit_scene_in_range(const TriRecord *tri, uint32_t n);
// Every triangle's denominator, for any ray direction passing the kernel's dir_fast_ok (each
// component +-0 or at least 2^-40, |d|_1 <= 16), is +-0 or within [2^-126, 2^126] in magnitude
// with no overflow on the way: the generic scan may then take 1/den without the class check
// (FrameArgs::rcp_fast).
bool scan_rcp_fast_scene(const TriRecord *tri, uint32_t n);
// Extra hipRTC options (debug build only; empty in the product library).
std::vector<std::string> jit_extra_flags();
// The generated scan (spec_scan1 / spec_scan2) for n triangle records.
// opts: kScanSkipB | kScanEagerSplit (experiment knobs, jit_scan_opts)
constexpr unsigned kScanSkipB = 1u, kScanEagerSplit = 2u;
std::string jit_scan_source(const TriRecord *tri, uint32_t n, unsigned opts = 0);
// Compile rvcp_kernels.hip with the given scan for gfx950 (hipRTC); 0 or -1 with err set.
// `legacy` also builds the mode-2 kernel (RVCP_JIT_LEGACY).
// `lds_scene`: the mode-2 kernel copies the scene into LDS (RVCP_LEGACY_LDS_SCENE).
int jit_compile_code(const std::string &scan, std::vector<char> &code, std::string &err,
                     bool legacy = false, int legacy_waves = 0, bool lds_scene = false,
                     bool bvh = false);
// jit_compile_code behind the on-disk code-object cache (rvcp_set_code_cache_dir): a verified
// entry for exactly this compile is read (*from_disk = true), else the module is compiled and
// stored; force_compile counts the entry rejected and recompiles it (the runtime refused it).
int jit_cached_code(const std::string &scan, std::vector<char> &code, std::string &err,
                    bool legacy, int legacy_waves, bool lds_scene, bool bvh, bool *from_disk,
                    bool force_compile);
// Compiled + loaded kernels for the scene on `device` (process-wide cache keyed by the scan
// source and `legacy`); nullptr with err set when hipRTC is unavailable or compilation fails.
// `sphereless`: the mode-2 kernel is built for 6 waves per SIMD.
// `lds_fits`: at most 64 spheres and 64 materials (and, as always here, 64 faces): the mode-2
// kernel reads its hit records, spheres and materials from LDS copies.
// `bvh`: also the BVH hybrid's kernels (RVCP_JIT_BVH; tri / n are then the prefix faces).
// `spheres` (legacy modules): the scene's sphere records, written into the module as literals
// (jit_sphere_source) -- the module is then valid for these spheres only, like its scan.
std::shared_ptr<JitKernels> jit_path_kernels(int device, const TriRecord *tri, uint32_t n,
                                             std::string &err, bool legacy = false,
                                             bool sphereless = false, bool lds_fits = false,
                                             bool bvh = false, const rvcp_sphere_t *spheres = nullptr,
                                             uint32_t n_spheres = 0, uint32_t n_materials = 64);
// The sphere X-macro of a mode-2 module ("" for none or more than kJitMaxSpheres).
constexpr uint32_t kJitMaxSpheres = 64;
std::string jit_sphere_source(const rvcp_sphere_t *sph, uint32_t n);
// The LDS sizes of a mode-2 module with the scene in LDS, and its LDS primary-hit columns.
std::string jit_legacy_lds_source(uint32_t n_faces, uint32_t n_spheres, uint32_t n_materials);

}  // namespace rvcp
