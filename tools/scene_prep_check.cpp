// scene_prep_check.cpp -- CPU driver of librvcp's host-only scene preparation
// (csrc/rvcp_scene_prep.cpp: .rvcpscn reader, upload validation, device tables), built with
// g++ under AddressSanitizer / UBSan by tests/test_scene_prep_cpu.py and fed damaged files.
//   scene_prep_check FILE [quirk=1]
// Prints one line: "rc=<code> faces=<n> lights=<n> total=<light area> err=<message>".
#include <cstdio>
#include <cstdlib>
#include <string>

#include "rvcp_scene_prep.h"

int main(int argc, char **argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s FILE [quirk]\n", argv[0]);
        return 2;
    }
    const bool quirk = argc < 3 || std::atoi(argv[2]) != 0;
    rvcp::SceneFile sf;
    std::string err;
    int rc = rvcp::read_scene_file(argv[1], sf, err);
    rvcp::SceneTables tab;
    if (rc == RVCP_OK) {
        rvcp::SceneInput in;
        in.materials = sf.materials.data(); in.n_materials = sf.lengths.materials_len;
        in.vertices = sf.vertices.data(); in.n_vertices = sf.lengths.vertices_len;
        in.faces = sf.faces.data(); in.n_faces = sf.lengths.faces_len;
        in.spheres = sf.spheres.data(); in.n_spheres = sf.lengths.spheres_len;
        in.lum_face_ids = sf.lum_face_ids.data(); in.n_lum_face_ids = sf.lengths.luminous_face_id_len;
        rc = rvcp::prepare_scene(in, quirk, tab, err);
    }
    std::printf("rc=%d faces=%zu lights=%zu total=%.9g err=%s\n", rc, tab.tri.size(),
                tab.lights.size(), (double)tab.light_total, err.c_str());
    return 0;
}
