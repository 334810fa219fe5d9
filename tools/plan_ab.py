"""Planning-time A/B on the C5 workload: python tools/plan_ab.py N_CALLS
(SG_HIP_LIB picks the library; SG_PLAN_THREADS the host threads). Prints the
wall time of sg_plan_batch and a fingerprint of the plan (lengths, kernel
stats, device bytes) so two libraries can be checked for identical plans."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402

native.lib()
calls = bench.c5_calls(int(sys.argv[1]))
t = time.time()
p = batch.Plan(calls, None)
dt = time.time() - t
st = p.stats()
fp = hashlib.md5((repr(sorted(st.items())) + repr(p.total) + p.lengths.tobytes().hex()).encode()).hexdigest()
print("lib %s threads %s calls %d plan_s %.2f failed %d fingerprint %s" % (
    os.path.basename(native.LIB_PATH), os.environ.get("SG_PLAN_THREADS", "auto"), len(calls), dt,
    int((p.status != 0).sum()), fp), flush=True)
