"""Summarise rocprofv3 --pmc passes: mean counter value per (kernel, grid size)."""
import collections
import csv
import glob
import json
import sys

tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob("gpurun_out/%s_*/run_counter_collection.csv" % tag)):
    for r in csv.DictReader(open(path)):
        key = "%s grid=%s" % (r["Kernel_Name"][:40], r["Grid_Size"])
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in sorted(d.items())} for k, d in acc.items() if k.startswith("sg_")}
json.dump(out, sys.stdout, indent=1)
