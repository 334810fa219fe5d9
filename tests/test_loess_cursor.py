"""The planner's loess contours are evaluated with a leaf cursor
(LoessFit::eval_seq, sg_loess.cpp) instead of a k-d tree walk per point; this
compiles the host planner's loess unit with g++ and checks the two bit for bit
on random anchor sets, integer and half-integer z, repeated z (CPU only)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "soundgen_beta_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_loess_cursor_equals_tree_walk(tmp_path):
    exe = str(tmp_path / "loess_cursor")
    cmd = ["g++", "-O2", "-std=c++17", "-I" + CSRC, "-I" + os.path.join(HERE, "..", "include"),
           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", os.path.join(HERE, "cpp", "loess_cursor.cpp"),
           os.path.join(CSRC, "sg_loess.cpp"), os.path.join(CSRC, "sg_rrng.cpp"), os.path.join(CSRC, "sg_scratch.cpp"), "-o", exe]
    subprocess.run(cmd, check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    tot, bad = (int(v) for v in r.stdout.split()[1::2])
    assert tot > 1_000_000 and bad == 0
