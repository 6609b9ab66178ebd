#!/usr/bin/env python3
"""Per-kernel counter totals of the LAST frame of a `rocprofv3 --pmc ... --kernel-trace` run of bench.py
(one frame: --steps 1 --warmup 0 --settle-s 0): for each kernel name, the counters of its last dispatch
(the timed frame's; bench.py's stats frames come first).  Used for the Grid / BVH chain-pass comparison
(DESIGN.md §7, round 6).

    python tools/pmc_passes.py PMC_DIR [PMC_DIR ...]  -> one JSON object {kernel: {counter: value}}
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def last_dispatch_counters(d):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> summed value
    for r in rows:
        per[(r["Kernel_Name"], int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    last = {}
    for (k, disp), cs in per.items():
        if k not in last or disp > last[k][0]:
            last[k] = (disp, cs)
    return {k: dict(v[1]) for k, v in last.items()}


def main():
    out = defaultdict(dict)
    for d in sys.argv[1:]:
        for k, cs in last_dispatch_counters(d).items():
            out[k].update(cs)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
