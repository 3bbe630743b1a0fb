"""The gen kernel's stealing walk, and connect's stealing shadow walk, on the host (VERDICT r5
Next #2, ADVICE r5 tie fixture; round 6 TPT_CONN_STEAL).

tests/native/steal_check.cpp runs the shipped device function itself -- walk4_steal
(csrc/tpt_bdpt.h), with its mailbox, job list and per-ray merge -- unmodified on an
emulated 64-lane wavefront (tests/native/wave_emu.h), on rays through the bunny's walk
group and through a mesh of duplicate triangles (every hit an exact two-leaf distance
tie), and requires every lane's answer to equal, bit for bit, the per-lane 4-wide walk and
the threaded binary walk (BVHAccel::Intersect's DFS with the strict `>`, BVH.cpp:103-143).
It also checks that HostScene::grank follows the DFS leaf order, and restates the
LDS-atomic merge the round-5 build first tried (not shipped) to show it losing hits
(DESIGN.md §5.2).  Connect's walk4_shadow_steal (csrc/tpt_device.h) runs the same way on
segments of random length with ShadowCheck's threshold, against the per-lane any-hit walk
and the closest-hit criterion (Scene.cpp:37-48).  CPU only."""
import os
import re
import subprocess

from conftest import PKG, ROOT


def test_stealing_walk_equals_the_sequential_fold(tmp_path):
    exe = str(tmp_path / "steal_check")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-std=c++17", "-O2", "-x", "c++", "-D__HIP_PLATFORM_AMD__",
                           "-I/opt/rocm/include", "-I", os.path.join(PKG, "csrc"),
                           os.path.join(ROOT, "tests", "native", "steal_check.cpp"), "-L", PKG, "-ltpt",
                           "-Wl,-rpath," + PKG, "-o", exe])
    p = subprocess.run([exe, os.path.join(PKG, "models")], capture_output=True, text=True, timeout=300)
    print(p.stdout)
    assert p.returncode == 0 and "ALL OK" in p.stdout, p.stdout + p.stderr
    m = re.search(r"bunny: \d+ waves, \d+ rays, (\d+) walked the group, (\d+) hits; stealing walk != DFS: (\d+)",
                  p.stdout)
    assert m and int(m.group(2)) > 10000 and int(m.group(3)) == 0
    # connect's stealing shadow walk (TPT_CONN_STEAL, uncapped): the any-hit answer of every
    # lane equals the per-lane walk's and ShadowCheck's closest-hit criterion
    for scene in ("bunny", "ties"):
        sh = re.search(scene + r" shadow: \d+ rays, (\d+) walked the group, (\d+) shadowed; stealing shadow walk != DFS: "
                       r"(\d+), per-lane any-hit walk != DFS: (\d+)", p.stdout)
        assert sh and int(sh.group(2)) > 100 and int(sh.group(3)) == 0 and int(sh.group(4)) == 0, scene
    # the not-shipped atomic-minimum merge (form 0) must be seen to fail: the check can
    # tell a right merge from a wrong one on these rays
    bad = re.search(r"bunny, LDS atomic-minimum merge form 0 \(not shipped\): (\d+) of", p.stdout)
    assert bad and int(bad.group(1)) > 0
