#!/usr/bin/env python3
"""Run tools/bin/gather_ceiling (1 and 2 dependent chains per lane, and the quad-cooperative
fetch) and write
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
    for chains in (1, 2, 0):  # 0: the quad-cooperative fetch
        r = subprocess.run([str(BIN), str(chains)], capture_output=True, text=True, timeout=300, check=True)
        rows += [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    one = [x for x in rows if x["chains"] == 1 and x.get("fetch", "lane") == "lane"]
    best = max(one, key=lambda x: x["GB_per_s"])
    res = {"what": "dependent 64-B per-lane record gathers (4 x global_load_dwordx4), 6 waves/SIMD, "
                   "one chain per lane = the path kernel's node step; every dword consumed (round 3: the round-1/2 "
                   "kernel consumed 7 of 16 dwords and the compiler narrowed its loads to 6 per record, "
                   "understating the ceiling ~1.45x); tools/gather_ceiling.hip. fetch quad_coop rows: "
                   "the same records fetched by the 4 lanes of a quad together (one 64-B segment per "
                   "quad per load) and transposed with DPP",
           "peak_GB_per_s": best["GB_per_s"], "peak_table_bytes": best["table_bytes"], "rows": rows}
    big = max(one, key=lambda x: x["table_bytes"])
    # the 1 GiB table misses the L2 on every record and each miss is one 128-B fabric read
    # (tools/fetch_calib.py: TCC_EA0_RDREQ_128B per record ~1.0), so the fabric line rate is twice
    # the record-byte rate there
    res["fabric_line_GB_per_s"] = round(2.0 * big["GB_per_s"], 1)
    res["fabric_note"] = ("L2 <-> fabric line rate of the same gathers from the largest table: every 64-B "
                          "record costs one 128-B fabric read, so fabric bytes/s = 2 x record bytes/s")
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "rows"}))
    for x in rows:
        print(json.dumps(x))


if __name__ == "__main__":
    main()
