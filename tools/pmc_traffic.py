#!/usr/bin/env python3
"""Per-launch HBM traffic of the path kernel from rocprofv3 --pmc passes (tools/pmc.sh).

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, "HBM [CDNA4]" and "rocprofv3 PMC slots"):
FETCH_SIZE and WRITE_SIZE are collected in separate passes (3 + 2 TCC slots do not fit one
pass); FETCH_SIZE (KiB) reports half the bytes of 128-B requests on gfx950, so it is doubled;
WRITE_SIZE (KiB) is taken as is.  hbm_bytes_per_launch = 2*FETCH + WRITE, in bytes, for the
timed (non-stats) dispatch of path_persistent.  The ray tracer's loads are 16-B-per-lane
gathers, a width the guide lists as uncalibrated, so the figure is recorded together with the
raw counter values and the TCC hit rate.

usage: python tools/pmc_traffic.py gpurun_out/pmc <workload-key> [out.json]
"""
import csv
import json
import sys
from pathlib import Path


def dispatch_counters(pass_dir: Path):
    """{(dispatch_id, kernel): {counter: value}} summed over the dispatch's rows."""
    out = {}
    for f in pass_dir.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            d = out.setdefault(key, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def timed_path_dispatch(counters):
    # the timed frame is the LAST path_persistent dispatch of the non-stats instantiation
    # (rocprofv3 reports demangled names: path_persistent<TRI_ONLY, STATS=false, MODE, WAVES>)
    keys = sorted(k for k in counters
                  if "path_persistent<" in k[1] and k[1].split("<", 2)[1].split(",")[1].strip() == "false")
    return keys[-1] if keys else None


def main():
    root = Path(sys.argv[1])
    workload = sys.argv[2]
    out = Path(sys.argv[3]) if len(sys.argv) > 3 else Path("profiles/pmc_traffic.json")
    vals, kernel = {}, None
    for p in sorted(x for x in root.iterdir() if x.is_dir()):
        c = dispatch_counters(p)
        k = timed_path_dispatch(c)
        if k is None:
            continue
        kernel = k[1]
        vals.update(c[k])
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        sys.exit(f"FETCH_SIZE/WRITE_SIZE not found under {root}: {sorted(vals)}")
    fetch = vals["FETCH_SIZE"] * 1024.0
    write = vals["WRITE_SIZE"] * 1024.0
    res = {
        "workload": workload,
        "kernel": kernel,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "fetch_size_bytes_raw": fetch,
        "write_size_bytes": write,
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); 16-B gathers are an uncalibrated width",
        "raw": vals,
    }
    if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
        res["tcc_hit_rate"] = vals["TCC_HIT_sum"] / max(1.0, vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps({k: v for k, v in res.items() if k != "raw"}))


if __name__ == "__main__":
    main()
