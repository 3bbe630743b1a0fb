"""The device libm replicas / RNG form (csrc/tpt_devmath.h) against this image's
glibc, compiled as host code.  Stride 1 = exhaustive (every float of each domain,
~15 s); the default stride keeps the CPU suite fast."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_devmath_matches_glibc(tmp_path):
    exe = str(tmp_path / "devmath_check")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off",
                           os.path.join(ROOT, "tests", "native", "devmath_check.cpp"), "-o", exe])
    stride = os.environ.get("TPT_DEVMATH_STRIDE", "61")
    r = subprocess.run([exe, stride], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    for line in r.stdout.strip().splitlines():
        assert line.endswith("bad=0"), line


@pytest.mark.gpu
def test_fast_reciprocal_exhaustive():
    """rcp_fast_f32 (make_ray's 1/d) equals IEEE 1.0f / x for every float it is used on."""
    exe = os.path.join(ROOT, "tests", "native", "build", "rcpf_check")
    assert os.path.exists(exe), "built by __graft_entry__.build()"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
