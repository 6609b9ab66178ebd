#!/usr/bin/env python3
"""Run tools/bin/gather_ceiling (1 and 2 dependent chains per lane) and write
profiles/gather_ceiling.json: every table size's rate and the ceiling bench.py's roofline uses —
the fastest table with ONE record in flight per lane (the path kernel's node-step shape).

usage: python tools/ceiling.py [out.json]
"""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
BIN = ROOT / "tools" / "bin" / "gather_ceiling"


def main():
    out = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "gather_ceiling.json"
    rows = []
    for chains in (1, 2):
        r = subprocess.run([str(BIN), str(chains)], capture_output=True, text=True, timeout=300, check=True)
        rows += [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    one = [x for x in rows if x["chains"] == 1]
    best = max(one, key=lambda x: x["GB_per_s"])
    res = {"what": "dependent 64-B per-lane record gathers (4 x global_load_dwordx4), 6 waves/SIMD, "
                   "one chain per lane = the path kernel's node step; tools/gather_ceiling.hip",
           "peak_GB_per_s": best["GB_per_s"], "peak_table_bytes": best["table_bytes"], "rows": rows}
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}))
    for x in rows:
        print(json.dumps(x))


if __name__ == "__main__":
    main()
