"""rand()'s fract as one v_fract_f32 is exact on every argument the RNG can
form: the C check (tests/rand_fract_check.c, linked with the CPU oracle's software sin) runs all
2.1e8 floats y in [1, 2^25] and finds no x = sin(y) * 43758.5453 for which x - floor(x) rounds
to 1.0, the only input where v_fract_f32 differs.  (The GPU side of the same check, with the
kernel's own sin and the instruction itself: tools/sqrt_check.hip, profiles/history/r04c_sqrt_check.log.)"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_rand_fract_never_rounds_to_one(tmp_path):
    exe = tmp_path / "fract_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-msse4.1", "-mfma", "-o", str(exe),
                    os.path.join(HERE, "rand_fract_check.c"),
                    os.path.join(ROOT, "oracle", "rvcp_oracle.c"), "-lm", "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fract == 1.0 in 0" in r.stdout
    assert "checked 209715201 rand arguments" in r.stdout
