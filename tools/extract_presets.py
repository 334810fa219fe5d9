"""Extract the soundgen() argument sets of presets$<speaker>$<name>
(R/presets.R:156-410 of the reference) into soundgen_beta_amd/presets.json.

Each preset is an R call string such as
    'soundgen(sylLen = 250, pitchAnchors = list(time = c(0, 1), value = c(147, 150)), ...)'
This script evaluates the small R subset those strings use (soundgen(), list(),
c(), numbers, strings, NA/TRUE/FALSE/NULL) into JSON data: the parameter
values are inputs for the C5 workload, not code. Runs in the build container
(where /root/reference exists); the JSON travels with the repo.

    python tools/extract_presets.py [/root/reference/R/presets.R]
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/R/presets.R"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "soundgen_beta_amd", "presets.json")

from soundgen_beta_amd.rcall import Parser, tokens  # noqa: E402,F401  (the R literal evaluator)


def main():
    text = open(SRC).read()
    start = text.index("presets = list(")
    body = text[start:]
    speakers = [(m.start(), m.group(1)) for m in re.finditer(r"\n  ([A-Za-z0-9]+) = list\(", body)]
    out = {}
    for m in re.finditer(r"\n\s+([A-Za-z0-9_]+) = '(soundgen\((?:[^']*)\))'", body):
        speaker = [s for p, s in speakers if p < m.start()][-1]
        call = " ".join(m.group(2).split())
        args = Parser(tokens(call)).expr()
        out.setdefault(speaker, {})[m.group(1)] = args if isinstance(args, dict) else {}
    n = sum(len(v) for v in out.values())
    json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)
    print("wrote %d presets (%s) to %s" % (n, ", ".join("%s %d" % (k, len(v)) for k, v in out.items()), OUT))


if __name__ == "__main__":
    main()
