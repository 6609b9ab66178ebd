#!/usr/bin/env python3
"""FETCH_SIZE calibration for the path kernel's access shape.

tools/gather_ceiling.hip issues dependent 64-B per-lane record gathers (4 x global_load_dwordx4)
over tables of known size; its byte count is exact: blocks x 256 lanes x iters records of 64 B
per timed dispatch.  From the 1 GiB table (past the 256 MiB Infinity Cache and the L2s) nearly
every record misses the L2, so FETCH_SIZE of that dispatch against those bytes gives the factor
that turns FETCH_SIZE into fabric bytes for this shape — instead of the x2 the guide states for
coalesced streaming reads.  TCC_HIT/TCC_MISS (another pass) give the L2 hit rate per table, and
TCC_EA0_RDREQ (a third pass) the fabric requests, so bytes per request follow as well.

usage: python tools/fetch_calib.py <dir with pass subdirs p1 p2 ...> <gather_ceiling stdout jsonl> [out.json]
"""
import csv
import json
import sys
from pathlib import Path


def dispatches(pass_dir: Path):
    """[(dispatch_id, kernel, {counter: value})] of the pass, in dispatch order."""
    out = {}
    for f in pass_dir.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            d = out.setdefault(key, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k[0], k[1], v) for k, v in sorted(out.items())]


def main():
    root, runs = Path(sys.argv[1]), Path(sys.argv[2])
    out = Path(sys.argv[3]) if len(sys.argv) > 3 else Path("profiles/r03_fetch_calibration.json")
    tables = [json.loads(l) for l in runs.read_text().splitlines() if l.startswith("{")]
    vals = [{} for _ in tables]
    for p in sorted(x for x in root.iterdir() if x.is_dir()):
        ds = [d for d in dispatches(p) if "gather" in d[1]]
        timed = ds[1::2]  # warm-up, timed, warm-up, timed, ... one pair per table
        for i, d in enumerate(timed[:len(tables)]):
            vals[i].update(d[2])
    rows = []
    for t, v in zip(tables, vals):
        iters = 3000 if t["table_bytes"] <= (1 << 15) * 64 else 2000
        alg = t["blocks"] * 256.0 * iters * 64.0
        row = {"table_bytes": t["table_bytes"], "algorithmic_bytes": alg}
        if "FETCH_SIZE" in v:
            row["fetch_size_bytes"] = v["FETCH_SIZE"] * 1024.0
            row["fetch_over_algorithmic"] = row["fetch_size_bytes"] / alg
        if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
            row["tcc_hit_rate"] = v["TCC_HIT_sum"] / max(1.0, v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
            row["tcc_requests"] = v["TCC_HIT_sum"] + v["TCC_MISS_sum"]
        if all(k in v for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
            row["rdreq_by_size"] = {"32B": v["TCC_EA0_RDREQ_32B_sum"], "64B": v["TCC_EA0_RDREQ_64B_sum"],
                                    "128B": v["TCC_EA0_RDREQ_128B_sum"]}
            row["read_bytes_by_size"] = (32.0 * v["TCC_EA0_RDREQ_32B_sum"] + 64.0 * v["TCC_EA0_RDREQ_64B_sum"] +
                                         128.0 * v["TCC_EA0_RDREQ_128B_sum"])
        if "TCC_EA0_RDREQ_sum" in v:
            row["ea_rdreq"] = v["TCC_EA0_RDREQ_sum"]
            row["ea_rdreq_per_record"] = v["TCC_EA0_RDREQ_sum"] / (alg / 64.0)
        rows.append(row)
    big = max(rows, key=lambda r: r["table_bytes"])
    res = {"what": "FETCH_SIZE against the known bytes of dependent 64-B per-lane record gathers "
                   "(tools/gather_ceiling.hip, one chain per lane, 6 waves/SIMD)",
           "rows": rows}
    if "fetch_over_algorithmic" in big and "tcc_hit_rate" in big:
        miss = 1.0 - big["tcc_hit_rate"]
        # fabric bytes of the L2 misses = algorithmic bytes x miss rate (every missed record is a
        # whole 64-B record): the factor that scales FETCH_SIZE to them
        res["fetch_factor_from_misses"] = big["algorithmic_bytes"] * miss / max(1.0, big["fetch_size_bytes"])
        res["fetch_factor"] = res["fetch_factor_from_misses"]
        res["fetch_factor_note"] = ("fabric read bytes = FETCH_SIZE x fetch_factor for 64-B record gathers, "
                                    f"from the {big['table_bytes'] >> 20} MiB table (L2 miss rate {miss:.3f})")
        if big.get("read_bytes_by_size"):
            # the request sizes the L2 actually issued: the direct byte count
            res["fetch_factor_from_request_sizes"] = big["read_bytes_by_size"] / max(1.0, big["fetch_size_bytes"])
            res["fetch_factor"] = res["fetch_factor_from_request_sizes"]
            res["fetch_factor_note"] += "; factor from the TCC_EA0_RDREQ_{32,64,128}B request sizes"
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
