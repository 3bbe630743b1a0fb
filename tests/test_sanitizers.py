"""Race detection on the CPU restatement ("Run the CPU restatement under
TSan"; the reference's own split is Renderer.cpp:86-114 with a thread_local RNG,
README.md:45-47).  tests/native/tsan_render.cpp renders a 64x64 frame, PT and BDPT,
through oracle_render on 8 threads, built with -fsanitize=thread; the run must report
no race and the threaded frames must equal the 1-thread ones (PT bit for bit, BDPT
within the splat merge's rounding)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "native", "tsan_render.cpp")
ORACLE = os.path.join(ROOT, "oracle", "tpt_oracle.cpp")
MODELS = os.path.join(ROOT, "toypathtracer-games101-assignment7_amd", "models")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_oracle_render_under_tsan(tmp_path):
    exe = str(tmp_path / "tsan_render")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-ffp-contract=off",
                           "-I", os.path.join(ROOT, "include"), SRC, ORACLE, "-o", exe, "-lpthread"])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1")
    r = subprocess.run(["setarch", "-R", exe, MODELS], capture_output=True, text=True, timeout=600, env=env)
    if "unexpected memory mapping" in r.stderr:  # kernels whose ASLR layout TSan cannot use
        r = subprocess.run([exe, MODELS], capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-2000:])
