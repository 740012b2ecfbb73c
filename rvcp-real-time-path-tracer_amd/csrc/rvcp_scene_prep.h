// rvcp_scene_prep.h -- host-only scene preparation of librvcp: upload validation, the
// device tables derived from the reference's upload arrays, and the .rvcpscn file reader.
// Pure C++ (no HIP), so the same source is built into librvcp.so and, for the sanitizer
// tests, into a plain g++ checker (tools/scene_prep_check.cpp).  Not part of the C-ABI.
#pragma once

#include <cmath>
#include <string>
#include <vector>

#include "../../include/rvcp.h"
#include "rvcp_internal.h"

namespace rvcp {

// ---- host-side vec3 with the shader's evaluation order (compile with -ffp-contract=off) ----
struct h3 { float x, y, z; };
inline h3 mk3(float x, float y, float z) { return h3{x, y, z}; }
inline h3 ld3h(const float *p) { return mk3(p[0], p[1], p[2]); }
inline h3 add(h3 a, h3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline h3 sub(h3 a, h3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline h3 muls(h3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
// the shader builtins, fused as in DESIGN.md §3.1 (these restate shader code, not glam)
inline float dot(h3 a, h3 b) { return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x)); }
inline h3 cross(h3 a, h3 b) {
    return mk3(std::fma(a.y, b.z, -(a.z * b.y)), std::fma(a.z, b.x, -(a.x * b.z)),
               std::fma(a.x, b.y, -(a.y * b.x)));
}
inline float length(h3 a) { return std::sqrt(dot(a, a)); }
inline h3 normalize(h3 a) { return muls(a, 1.0f / std::sqrt(dot(a, a))); }
inline void st3(float *d, h3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

// The upload arrays of rvcp_upload_scene (the reference's descriptor-set buffers).
struct SceneInput {
    const rvcp_material_t *materials = nullptr;
    uint32_t n_materials = 0;
    const rvcp_vertex_t *vertices = nullptr;
    uint32_t n_vertices = 0;
    const rvcp_face_t *faces = nullptr;
    uint32_t n_faces = 0;
    const rvcp_sphere_t *spheres = nullptr;
    uint32_t n_spheres = 0;
    const uint32_t *lum_face_ids = nullptr;
    uint32_t n_lum_face_ids = 0;
};

// What the device receives: the scan's triangle records, per-material and per-face shading
// records and the light table (sample_light_games101 with the std140 id quirk applied).
struct SceneTables {
    std::vector<TriRecord> tri;
    std::vector<MatRecord> mats;
    std::vector<FaceShade> shade;
    std::vector<LightRecord> lights;     // at least one entry (a zero record if no lights)
    float light_total = 0.0f;
};

// Validate `in` and build its tables.  RVCP_OK, or RVCP_E_INVALID with `err` set (every
// index the kernels follow is bounds-checked here; the reference checks none).
int prepare_scene(const SceneInput &in, bool lum_id_std140_quirk, SceneTables &out,
                  std::string &err);

// A .rvcpscn file ("RVCPSCN1", format in scene_io.py) read into arrays of their own types.
struct SceneFile {
    rvcp_lengths_t lengths{};
    rvcp_camera_t camera{};
    std::vector<rvcp_material_t> materials;
    std::vector<rvcp_sphere_t> spheres;
    std::vector<rvcp_vertex_t> vertices;
    std::vector<rvcp_face_t> faces;
    std::vector<uint32_t> lum_sphere_ids, lum_face_ids;
};

// RVCP_OK, or RVCP_E_INVALID with `err` set for an unreadable, truncated or malformed file
// (the header's lengths must account for the file's size exactly).
int read_scene_file(const char *path, SceneFile &out, std::string &err);

}  // namespace rvcp
