"""The BDPT gen hand-off protocol on the host (VERDICT r3 Next #8): the device's own
sequence-word functions (csrc/tpt_genseq.h) driven by two emulated gen streams with
a limited number of resident slots (tests/native/genseq_check.cpp).  CPU only: never
run as a GPU stress test."""
import os
import subprocess

from conftest import ROOT


def test_gen_handoff_protocol(tmp_path):
    exe = str(tmp_path / "genseq_check")
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-pthread", "-I",
                           os.path.join(ROOT, "toypathtracer-games101-assignment7_amd", "csrc"),
                           os.path.join(ROOT, "tests", "native", "genseq_check.cpp"), "-o", exe])
    p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(p.stdout)
    assert p.returncode == 0 and "ALL OK" in p.stdout, p.stdout + p.stderr
