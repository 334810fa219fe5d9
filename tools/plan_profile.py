"""Where the host planner spends its time: samples the planning threads
(tools/sampler.c, SIGPROF at 2 kHz) while batch.Plan plans C5 calls, and
attributes each sample to the innermost planner function on its stack
(addr2line on libsoundgen_hip.so; inline chains when built with -g), so time
inside libc (memcpy, memset, malloc) or libm is charged to the planner code
that called it.

    python tools/plan_profile.py [calls] [top]
    (SG_PP_RNG=1: the calls draw from one RRng stream through callbacks, as from R)

Development tool; CPU only.
"""
import collections
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# llvm's addr2line reads the DWARF 5 line tables clang emits (binutils' may not)
_SYMB = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
ADDR2LINE = [_SYMB, "--output-style=GNU"] if os.path.exists(_SYMB) else ["addr2line"]


def _maps():
    rows = []
    for ln in open("/proc/self/maps"):
        f = ln.split()
        if len(f) < 6:
            continue
        a, b = (int(x, 16) for x in f[0].split("-"))
        rows.append((a, b, f[1], int(f[2], 16), f[5]))
    base = {}
    for a, b, perm, off, path in rows:
        if off == 0 and path not in base:
            base[path] = a
    return [(a, b, path, base.get(path, a)) for a, b, perm, off, path in rows if "x" in perm]


def _locate(maps, pc):
    for a, b, path, base in maps:
        if a <= pc < b:
            return path, pc - base
    return None, 0


def _symbolize(path, offs):
    """{offset: [(function, file:line), ...] innermost first}"""
    out, cur, addr = {}, [], None
    res = subprocess.run(ADDR2LINE + ["-a", "-f", "-i", "-C", "-e", path] + ["0x%x" % o for o in sorted(offs)],
                         capture_output=True, text=True).stdout.splitlines()
    for ln in res:
        if ln.startswith("0x") and len(ln.split()) == 1:
            if addr is not None:
                out[addr] = list(zip(cur[0::2], cur[1::2]))
            addr, cur = int(ln, 16), []
        else:
            cur.append(ln)
    if addr is not None:
        out[addr] = list(zip(cur[0::2], cur[1::2]))
    return out


def _short(fn):
    return fn.replace("(anonymous namespace)", "anon").split("(")[0]


def main(n_calls=4096, top=40):
    import bench
    from soundgen_beta_amd import batch
    so = os.path.join(ROOT, "tools", "_sampler.so")
    if not os.path.exists(so):
        subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "sampler.c")])
    S = C.CDLL(so)
    S.sg_sampler_pcs.restype = C.POINTER(C.c_uint64)
    S.sg_sampler_stacks.restype = C.POINTER(C.c_uint64)
    depth = S.sg_sampler_depth()
    calls = bench.c5_calls(int(n_calls))
    if os.environ.get("SG_PP_RNG"):  # one R-RNG stream through callbacks (the R shim's path): serial planning
        from soundgen_beta_amd.rrng import RRng
        g = RRng(7)
        calls = [{"kind": "soundgen", "args": c["args"], "rng": g} for c in calls]
    # load the library, warm the size estimates (SG_PP_WARM=1: a whole plan first, so that the
    # host block cache is as warm as for bench.py's later chunks)
    batch.Plan(calls if os.environ.get("SG_PP_WARM") else calls[:max(64, len(calls) // 4)], None).close()
    node = None
    if os.environ.get("SG_PP_NODE"):  # the node path (with SG_PP_RNG: draws-only recording + replay)
        from soundgen_beta_amd import native
        node = native.Node([0])
    S.sg_sampler_start(2000, 1)
    t0 = time.perf_counter()
    p = batch.NodePlan(calls, node) if node else batch.Plan(calls, None)
    wall = time.perf_counter() - t0
    n = S.sg_sampler_stop()
    p.close()
    P, ST = S.sg_sampler_pcs(), S.sg_sampler_stacks()
    maps = _maps()
    lib = None
    samples = []  # (leaf object, leaf offset, [planner offsets innermost first])
    for i in range(n):
        leaf_path, leaf_off = _locate(maps, P[i])
        frames = [P[i]] + [ST[i * depth + k] for k in range(depth) if ST[i * depth + k]]
        mine = []
        for j, pc in enumerate(frames):
            path, off = _locate(maps, pc)
            if path and "libsoundgen_hip" in path:
                lib = path
                mine.append(off if j == 0 else off - 1)  # return address -> call site
        samples.append((leaf_path, leaf_off, mine))
    sym = _symbolize(lib, {o for _, _, m in samples for o in m}) if lib else {}
    self_fn, incl_fn, leaf_obj = collections.Counter(), collections.Counter(), collections.Counter()
    self_line = collections.Counter()
    under = os.environ.get("SG_PP_UNDER")  # only samples with this planner frame on the stack
    if under:
        samples = [x for x in samples if any(under in _short(fn) for o in x[2] for fn, _ in sym.get(o, []))]
        n = len(samples)
    for leaf_path, leaf_off, mine in samples:
        leaf_obj[os.path.basename(leaf_path or "?")] += 1
        if not mine:
            self_fn["<outside the planner library>"] += 1
            continue
        chain = sym.get(mine[0], [("??", "")])
        where = "" if leaf_path and "libsoundgen_hip" in leaf_path else "  [in %s]" % os.path.basename(leaf_path or "?")
        self_fn[_short(chain[0][0]) + where] += 1
        self_line["%s @ %s%s" % (_short(chain[0][0]), chain[0][1].split("/")[-1], where)] += 1
        seen = set()
        for o in mine:
            for fn, _ in sym.get(o, []):
                f = _short(fn)
                if f not in seen:
                    seen.add(f)
                    incl_fn[f] += 1
    tot = max(n, 1)
    print("calls %d, wall %.2f s, samples %d" % (int(n_calls), wall, n))
    for title, ctr in (("self (innermost planner frame; [in X] = time inside library X)", self_fn),
                       ("self by source line", self_line),
                       ("inclusive (any planner frame on the stack)", incl_fn), ("leaf object", leaf_obj)):
        print("\n== %s" % title)
        for k, v in ctr.most_common(int(top)):
            print("%6.2f%%  %s" % (100.0 * v / tot, k[:150]))


if __name__ == "__main__":
    main(*sys.argv[1:])
