"""librvcp's host-side scene preparation on the CPU, under AddressSanitizer / UBSan.

csrc/rvcp_scene_prep.cpp holds everything rvcp_upload_scene / rvcp_upload_scene_file do on the
host before any HIP call: the .rvcpscn reader, the bounds checks of every index the kernels
follow (face vertices, material ids, luminous face ids) and the device tables.  It is built
here with g++ -fsanitize=address,undefined together with tools/scene_prep_check.cpp and fed
valid and damaged files: every damaged file must be rejected with RVCP_E_INVALID and a
message, with no sanitizer report (the reference does no validation at all,
src/ray_tracer/vulkan.rs:454-574)."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import rvcp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rvcp-real-time-path-tracer_amd", "csrc")
HDR = 128
LEN_OFF = 16            # six u32 lengths: materials, spheres, vertices, faces, lum spheres, lum faces


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("prep") / "scene_prep_check")
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-ffp-contract=off",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                        "-I", CSRC, os.path.join(ROOT, "tools", "scene_prep_check.cpp"),
                        os.path.join(CSRC, "rvcp_scene_prep.cpp"), "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer build unavailable: " + r.stderr[-300:])
    return exe


def _run(exe, path, quirk=1):
    r = subprocess.run([exe, str(path), str(quirk)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
    out = r.stdout.strip()
    fields = dict(kv.split("=", 1) for kv in out.split(" ", 4))
    return int(fields["rc"]), fields


@pytest.fixture(scope="module")
def cornell_file(tmp_path_factory):
    p = tmp_path_factory.mktemp("scn") / "cornell.rvcpscn"
    rvcp_amd.scene_io.save(str(p), rvcp_amd.Scene.default())
    return p.read_bytes()


def _lengths(data):
    return list(struct.unpack_from("<6I", data, LEN_OFF))


def _with_lengths(data, L):
    b = bytearray(data)
    struct.pack_into("<6I", b, LEN_OFF, *L)
    return bytes(b)


def _body_offsets(data):
    L = _lengths(data)
    sizes = [32, 32, 32, 16, 4, 4]
    off, out = HDR, []
    for n, s in zip(L, sizes):
        out.append(off)
        off += n * s
    return out


def test_valid_files(checker, cornell_file, tmp_path):
    p = tmp_path / "ok.rvcpscn"
    p.write_bytes(cornell_file)
    rc, f = _run(checker, p)
    assert rc == 0 and f["faces"] == "32" and f["lights"] == "2", f
    rc0, f0 = _run(checker, p, quirk=0)
    assert rc0 == 0 and float(f0["total"]) > 0
    big = tmp_path / "big.rvcpscn"
    rvcp_amd.scene_io.save(str(big), rvcp_amd.scene.with_random_triangles(rvcp_amd.Scene.default(), 3000))
    rc, f = _run(checker, big)
    assert rc == 0 and f["faces"] == "3032", f


def _damaged(data):
    """(name, bytes, expected message fragment)"""
    L = _lengths(data)
    off_mat, off_sph, off_vtx, off_face, off_ls, off_lf = _body_offsets(data)
    cases = [
        ("empty", b"", "not an RVCPSCN1"),
        ("short_header", data[:50], "not an RVCPSCN1"),
        ("bad_magic", b"RVCPSCN2" + data[8:], "not an RVCPSCN1"),
        ("bad_version", data[:8] + struct.pack("<I", 2) + data[12:], "version"),
        ("bad_header_bytes", data[:12] + struct.pack("<I", 64) + data[16:], "version"),
        ("truncated_body", data[:-5], "size does not match"),
        ("appended_junk", data + b"\0" * 16, "size does not match"),
        ("faces_len_plus_one", _with_lengths(data, L[:3] + [L[3] + 1] + L[4:]), "size does not match"),
        ("materials_len_huge", _with_lengths(data, [0xFFFFFFFF] + L[1:]), "size does not match"),
        ("all_lengths_huge", _with_lengths(data, [0xFFFFFFFF] * 6), "size does not match"),
        ("zero_materials_consistent",
         _with_lengths(data[:off_mat] + data[off_sph:], [0] + L[1:]), "material"),
    ]
    b = bytearray(data)
    struct.pack_into("<I", b, off_face + 16 * 5 + 4, 10 ** 6)         # face 5, vertex 1
    cases.append(("vertex_index_oob", bytes(b), "vertex index out of range"))
    b = bytearray(data)
    struct.pack_into("<I", b, off_face + 16 * 7 + 12, L[0])            # face 7 material
    cases.append(("material_id_oob", bytes(b), "material out of range"))
    b = bytearray(data)
    struct.pack_into("<I", b, off_lf, L[3])                            # luminous id == F
    cases.append(("lum_id_oob", bytes(b), "luminous face id"))
    return cases


def test_damaged_files_rejected(checker, cornell_file, tmp_path):
    for name, blob, frag in _damaged(cornell_file):
        p = tmp_path / f"{name}.rvcpscn"
        p.write_bytes(blob)
        rc, f = _run(checker, p)
        assert rc == rvcp_amd.abi.RVCP_E_INVALID, (name, f)
        assert frag in f["err"], (name, f["err"])


def test_missing_and_directory_paths(checker, tmp_path):
    rc, f = _run(checker, tmp_path / "does_not_exist.rvcpscn")
    assert rc == rvcp_amd.abi.RVCP_E_INVALID and "cannot open" in f["err"]
    rc, f = _run(checker, tmp_path)                                    # a directory
    assert rc == rvcp_amd.abi.RVCP_E_INVALID


def test_random_byte_corruption(checker, cornell_file, tmp_path):
    """Seeded random corruption of header and body bytes: any outcome but a crash or a
    sanitizer report is acceptable (a flipped float is still a valid scene)."""
    rng = np.random.default_rng(11)
    for i in range(40):
        b = bytearray(cornell_file)
        for _ in range(int(rng.integers(1, 9))):
            k = int(rng.integers(0, len(b)))
            b[k] = int(rng.integers(0, 256))
        p = tmp_path / f"r{i}.rvcpscn"
        p.write_bytes(bytes(b))
        rc, _ = _run(checker, p)
        assert rc in (0, rvcp_amd.abi.RVCP_E_INVALID)
