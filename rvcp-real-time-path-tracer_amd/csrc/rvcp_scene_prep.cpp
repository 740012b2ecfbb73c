// rvcp_scene_prep.cpp -- host-only scene preparation (rvcp_scene_prep.h): the part of
// Vk::create_descriptor_set_0s (src/ray_tracer/vulkan.rs:454-574) that turns the Rust upload
// arrays into device tables, plus the .rvcpscn reader.  Compiled with -ffp-contract=off: the
// derived constants (edges, light areas, albedo / PI) use the shader's float operations.
#include "rvcp_scene_prep.h"

#include <cstdio>
#include <cstring>

namespace rvcp {

namespace {

// get_face_area, ray_tracer_games101_branch.comp:302-307
float face_area(const rvcp_vertex_t *v, const rvcp_face_t &f)
{
    const h3 v0 = ld3h(v[f.vertices[0]].position), v1 = ld3h(v[f.vertices[1]].position);
    const h3 v2 = ld3h(v[f.vertices[2]].position);
    return 0.5f * length(cross(sub(v1, v0), sub(v2, v0)));
}

}  // namespace

int prepare_scene(const SceneInput &in, bool quirk, SceneTables &out, std::string &err)
{
    if (!in.materials || in.n_materials == 0) { err = "need >= 1 material"; return RVCP_E_INVALID; }
    if ((in.n_vertices && !in.vertices) || (in.n_faces && !in.faces) ||
        (in.n_lum_face_ids && !in.lum_face_ids) || (in.n_spheres && !in.spheres)) {
        err = "null array with nonzero length";
        return RVCP_E_INVALID;
    }
    for (uint32_t i = 0; i < in.n_spheres; i++)
        if (in.spheres[i].material_id >= in.n_materials) {
            err = "sphere " + std::to_string(i) + " material out of range";
            return RVCP_E_INVALID;
        }
    for (uint32_t i = 0; i < in.n_faces; i++) {
        for (int k = 0; k < 3; k++)
            if (in.faces[i].vertices[k] >= in.n_vertices) {
                err = "face " + std::to_string(i) + " vertex index out of range";
                return RVCP_E_INVALID;
            }
        if (in.faces[i].material_id >= in.n_materials) {
            err = "face " + std::to_string(i) + " material out of range";
            return RVCP_E_INVALID;
        }
    }
    for (uint32_t i = 0; i < in.n_lum_face_ids; i++)
        if (in.lum_face_ids[i] >= in.n_faces) {
            err = "luminous face id " + std::to_string(i) + " out of range";
            return RVCP_E_INVALID;
        }

    // triangles: v0, e1 = v1 - v0, e2 = v2 - v0 (:243-248)
    out.tri.assign(in.n_faces, TriRecord{});
    for (uint32_t i = 0; i < in.n_faces; i++) {
        const rvcp_face_t &f = in.faces[i];
        const h3 v0 = ld3h(in.vertices[f.vertices[0]].position);
        const h3 v1 = ld3h(in.vertices[f.vertices[1]].position);
        const h3 v2 = ld3h(in.vertices[f.vertices[2]].position);
        st3(out.tri[i].v0, v0);
        st3(out.tri[i].e1, sub(v1, v0));
        st3(out.tri[i].e2, sub(v2, v0));
    }
    out.mats.assign(in.n_materials, MatRecord{});
    for (uint32_t i = 0; i < in.n_materials; i++) {
        std::memcpy(out.mats[i].albedo, in.materials[i].albedo, sizeof(float) * 3);
        out.mats[i].ty = in.materials[i].ty;
        for (int c = 0; c < 3; c++) out.mats[i].alb_pi[c] = in.materials[i].albedo[c] / 3.1415926f;
    }
    out.shade.assign(in.n_faces, FaceShade{});
    for (uint32_t i = 0; i < in.n_faces; i++) {
        FaceShade &fs = out.shade[i];
        const rvcp_face_t &f = in.faces[i];
        std::memcpy(fs.n0, in.vertices[f.vertices[0]].normal, 12);
        std::memcpy(fs.n1, in.vertices[f.vertices[1]].normal, 12);
        std::memcpy(fs.n2, in.vertices[f.vertices[2]].normal, 12);
        fs.mat = f.material_id;
        fs.ty = out.mats[fs.mat].ty;
        std::memcpy(fs.alb_pi, out.mats[fs.mat].alb_pi, 12);
    }
    // light table (sample_light_games101, :384-404) with the std140 id quirk (:109-111):
    // element i of the std140 `uint v[100]` reads the packed u32 at 4i (0 past the end)
    const uint32_t nl = in.n_lum_face_ids;
    auto light_id = [&](uint32_t i) {
        return quirk ? ((4ull * i < nl) ? in.lum_face_ids[4u * i] : 0u) : in.lum_face_ids[i];
    };
    out.lights.assign(nl ? nl : 1u, LightRecord{});
    float total = 0.0f;
    for (uint32_t i = 0; i < nl; i++) total += face_area(in.vertices, in.faces[light_id(i)]);
    float run = 0.0f;
    for (uint32_t i = 0; i < nl; i++) {
        const uint32_t id = light_id(i);
        const rvcp_face_t &f = in.faces[id];
        run += face_area(in.vertices, f);
        LightRecord &L = out.lights[i];
        L.cum = run;
        L.face = id;
        std::memcpy(L.v0, in.vertices[f.vertices[0]].position, 12);
        std::memcpy(L.v1, in.vertices[f.vertices[1]].position, 12);
        std::memcpy(L.v2, in.vertices[f.vertices[2]].position, 12);
        st3(L.n, normalize(ld3h(in.vertices[f.vertices[0]].normal)));
        std::memcpy(L.le, in.materials[f.material_id].albedo, 12);
    }
    out.light_total = total;
    return RVCP_OK;
}

int read_scene_file(const char *path, SceneFile &out, std::string &err)
{
    if (!path) { err = "null path"; return RVCP_E_INVALID; }
    FILE *f = std::fopen(path, "rb");
    if (!f) { err = std::string("cannot open scene file ") + path; return RVCP_E_INVALID; }
    struct Closer { FILE *f; ~Closer() { std::fclose(f); } } closer{f};
    constexpr size_t kHeader = 128;
    unsigned char head[kHeader];
    if (std::fread(head, 1, kHeader, f) != kHeader || std::memcmp(head, "RVCPSCN1", 8) != 0) {
        err = "not an RVCPSCN1 scene file";
        return RVCP_E_INVALID;
    }
    uint32_t version, header_bytes;
    std::memcpy(&version, head + 8, 4);
    std::memcpy(&header_bytes, head + 12, 4);
    std::memcpy(&out.lengths, head + 16, sizeof(out.lengths));
    std::memcpy(&out.camera, head + 40, sizeof(out.camera));
    if (version != 1 || header_bytes != kHeader) {
        err = "unsupported scene file version";
        return RVCP_E_INVALID;
    }
    const rvcp_lengths_t &L = out.lengths;
    // 6 lengths < 2^32 times <= 32 B: the sum fits in 64 bits
    const uint64_t body = 32ull * L.materials_len + 32ull * L.spheres_len + 32ull * L.vertices_len +
                          16ull * L.faces_len + 4ull * L.luminous_sphere_id_len +
                          4ull * L.luminous_face_id_len;
    if (std::fseek(f, 0, SEEK_END) != 0) { err = "cannot seek scene file"; return RVCP_E_INVALID; }
    const long size = std::ftell(f);
    if (size < 0 || (uint64_t)size != kHeader + body) {
        err = "scene file size does not match its lengths";
        return RVCP_E_INVALID;
    }
    if (std::fseek(f, (long)kHeader, SEEK_SET) != 0) { err = "cannot seek scene file"; return RVCP_E_INVALID; }
    // each array into storage of its own type, in file order
    bool ok = true;
    auto take = [&](auto &vec, uint32_t n) {
        vec.resize(n);
        if (ok && n) ok = std::fread(vec.data(), sizeof(vec[0]), n, f) == n;
    };
    take(out.materials, L.materials_len);
    take(out.spheres, L.spheres_len);
    take(out.vertices, L.vertices_len);
    take(out.faces, L.faces_len);
    take(out.lum_sphere_ids, L.luminous_sphere_id_len);
    take(out.lum_face_ids, L.luminous_face_id_len);
    if (!ok) { err = "error reading scene file"; return RVCP_E_INVALID; }
    return RVCP_OK;
}

}  // namespace rvcp
