"""Per-step kernel table from a rocprofv3 kernel-stats CSV of bench.py
(--steps S --warmup W --device-steps 0 --no-d2h: S + W + S executes of every plan).
    python tools/kstats_table.py <run_kernel_stats.csv> <executes> [top]"""
import csv
import sys

path, ex = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
rows = [r for r in csv.DictReader(open(path)) if r["Name"].startswith("sg_") and "amp_build" not in r["Name"]
        and "ugather" not in r["Name"]]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / ex / 1e6
print("| kernel | ms/step | launches/step × avg |")
print("|---|---|---|")
for r in rows[:top]:
    n = int(r["Calls"]) // ex
    print("| `%s` | %.1f | %d × %.2f ms |" % (r["Name"], float(r["TotalDurationNs"]) / ex / 1e6, n,
                                        float(r["AverageNs"]) / 1e6))
print("\nsum of kernels: %.1f ms/step" % tot)
