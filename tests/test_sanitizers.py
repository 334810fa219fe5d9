"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
§5): tests/sanitize/run.sh builds the planner (soundgen_beta_amd/csrc/*.cpp)
and the oracle with -fsanitize=address,undefined, preloads the runtime into a
pytest process and runs the CPU planner tests there -- parallel planning and
the part merge, the scratch pools, the bulk-block cache and its trim, the
uniform gather, the device amplitude formula evaluated on the host, the loess
cursor, R's RNG, the sharded planning of tests/test_dist.py. Any report fails."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(1500)
def test_planner_and_oracle_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "tests", "sanitize", "run.sh"), "tests/sanitize/test_canary.py",
                        "tests/test_planner.py", "tests/test_amp_build.py", "tests/test_oracle.py",
                        "tests/test_loess_cursor.py", "tests/test_api_helpers.py", "tests/test_rrng.py",
                        "tests/test_dist.py", "-m", "not gpu"],
                       cwd=ROOT, capture_output=True, text=True, timeout=1400)
    if r.returncode != 0:  # keep the whole report (pytest shows only the tail)
        os.makedirs(os.path.join(ROOT, "tests", "sanitize", "_build"), exist_ok=True)
        with open(os.path.join(ROOT, "tests", "sanitize", "_build", "last_failure.log"), "w") as f:
            f.write(r.stdout + "\n----- stderr -----\n" + r.stderr)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert " passed" in r.stdout and "skipped" not in r.stdout.split("\n")[-2], r.stdout[-2000:]
