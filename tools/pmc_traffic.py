#!/usr/bin/env python3
"""Per-launch fabric traffic and pipe counters of the path kernel from rocprofv3 --pmc passes
(tools/pmc.sh), recorded per workload key in one JSON (bench.py reads its key's record).

Recipe (/opt/skills/guides/MI355X_MICROARCH.md, "HBM [CDNA4]" and "rocprofv3 PMC slots"):
FETCH_SIZE and WRITE_SIZE come from separate passes (3 + 2 TCC slots do not fit one pass).
FETCH_SIZE = TCC_EA0_RDREQ x 64 B; the guide's x2 holds for coalesced 16-B/lane streams, and
other shapes need their own calibration.  The path kernel's reads are 64-B record gathers:
tools/fetch_calib.py calibrates them on tools/gather_ceiling.hip's known byte count, and when a
pass collected the read requests by size (TCC_EA0_RDREQ_32B/64B/128B_sum) the read bytes are
counted from them directly (32 n32 + 64 n64 + 128 n128).  Otherwise FETCH_SIZE is scaled by the
calibrated factor (profiles/r03_fetch_calibration.json).  WRITE_SIZE is taken as is (exact for
16-B-per-lane stores).  These are L2 <-> fabric bytes: Infinity-Cache hits are included.

usage: python tools/pmc_traffic.py gpurun_out/pmc <workload-key> [out.json] [kernel-substring]
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CALIB = ROOT / "profiles" / "r03_fetch_calibration.json"


def dispatch_counters(pass_dir: Path):
    """{(dispatch_id, kernel): {counter: value}} summed over the dispatch's rows."""
    out = {}
    for f in pass_dir.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            d = out.setdefault(key, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def timed_path_dispatch(counters, sub=None):
    # the timed frame is the LAST path_persistent dispatch of the non-stats instantiation
    # (rocprofv3 reports demangled names: path_persistent<TRI_ONLY, STATS=false, MODE, WAVES, ACC>)
    if sub:
        keys = sorted(k for k in counters if sub in k[1])
    else:
        keys = sorted(k for k in counters
                      if "path_persistent<" in k[1] and k[1].split("<", 2)[1].split(",")[1].strip() == "false")
    return keys[-1] if keys else None


def _targs(name):
    try:
        return [a.strip() for a in name.split("<", 2)[1].split(">")[0].split(",")]
    except IndexError:
        return []


def _mode(name):
    a = _targs(name)
    return int(a[2]) if "path_persistent<" in name and len(a) > 2 and a[2].isdigit() else None


def _stats(name):
    a = _targs(name)
    return len(a) > 1 and a[1] == "true"


def derive(vals):
    """Fabric bytes and the pipe ratios bench.py reports, from the merged counters."""
    res = {}
    write = vals.get("WRITE_SIZE", 0.0) * 1024.0
    if all(k in vals for k in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
        read = (32.0 * vals["TCC_EA0_RDREQ_32B_sum"] + 64.0 * vals["TCC_EA0_RDREQ_64B_sum"] +
                128.0 * vals["TCC_EA0_RDREQ_128B_sum"])
        res["read_bytes_method"] = "TCC_EA0_RDREQ_{32,64,128}B request sizes"
    elif "FETCH_SIZE" in vals:
        factor = 2.0
        src = "guide x2 (coalesced streams; no calibration record)"
        if CALIB.exists():
            c = json.loads(CALIB.read_text())
            if c.get("fetch_factor"):
                factor, src = c["fetch_factor"], f"calibrated on 64-B record gathers ({CALIB.name})"
        read = vals["FETCH_SIZE"] * 1024.0 * factor
        res["read_bytes_method"] = f"FETCH_SIZE x {factor:.3f}: {src}"
    else:
        return res
    res.update({"hbm_bytes_per_launch": read + write, "read_bytes": read, "write_size_bytes": write})
    if "FETCH_SIZE" in vals:
        res["fetch_size_bytes_raw"] = vals["FETCH_SIZE"] * 1024.0
    if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
        res["tcc_hit_rate"] = vals["TCC_HIT_sum"] / max(1.0, vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])
    if "TCP_TOTAL_CACHE_ACCESSES" in vals and "TCP_TCC_READ_REQ" in vals:
        res["l1_hit_rate"] = 1.0 - vals["TCP_TCC_READ_REQ"] / max(1.0, vals["TCP_TOTAL_CACHE_ACCESSES"])
    if "GRBM_GUI_ACTIVE" in vals:
        cyc = vals["GRBM_GUI_ACTIVE"] / 8.0  # the counter sums the 8 XCDs
        cus = 256.0
        if "SQ_INSTS_VALU" in vals:
            # a wave64 VALU instruction occupies a SIMD for 2 cycles (32 lanes/cycle)
            res["valu_busy"] = 2.0 * vals["SQ_INSTS_VALU"] / (1024.0 * cyc)
        for k, name in (("TA_TA_BUSY", "ta_busy"), ("TD_TD_BUSY", "td_busy")):
            if k in vals:
                res[name] = vals[k] / (cus * cyc)
    if "SQ_INSTS_SALU" in vals and "SQ_INSTS_VALU" in vals:
        res["salu_per_valu"] = vals["SQ_INSTS_SALU"] / max(1.0, vals["SQ_INSTS_VALU"])
    return res


def main():
    root = Path(sys.argv[1])
    workload = sys.argv[2]
    out = Path(sys.argv[3]) if len(sys.argv) > 3 else ROOT / "profiles" / "pmc_traffic.json"
    sub = sys.argv[4] if len(sys.argv) > 4 else None
    vals, kernel = {}, None
    pass_vals = [{}, {}]  # a two-pass frame's launches: the closest-chain pass, the replay pass
    pass_kernels = [None, None]
    for p in sorted(x for x in root.iterdir() if x.is_dir()):
        c = dispatch_counters(p)
        k = timed_path_dispatch(c, sub)
        if k is None:
            continue
        kernel = k[1]
        cur = dict(c[k])
        # a two-pass frame (FrameMode 5 or 7, then 6, drt_capi.hip): the frame is both launches
        if _mode(k[1]) in (6, 8):
            prev = [d for d in c if d[0] < k[0] and _mode(d[1]) in (5, 7) and not _stats(d[1])]
            if prev:
                p5 = max(prev)  # the frame's first pass
                kernel = p5[1] + " + " + k[1]
                pass_vals[0].update(c[p5])
                pass_vals[1].update(c[k])
                pass_kernels = [p5[1], k[1]]
                for n, v in c[p5].items():
                    cur[n] = cur.get(n, 0.0) + v
        vals.update(cur)
    rec = derive(vals)
    if "hbm_bytes_per_launch" not in rec:
        sys.exit(f"no read-byte counters under {root}: {sorted(vals)}")
    rec = {"kernel": kernel, **rec, "raw": vals}
    if pass_kernels[0]:
        # per pass (bench.py roofline.passes): the same derived figures for each launch on its own
        rec["passes"] = [{"kernel": kn, **derive(pv), "raw": pv} for kn, pv in zip(pass_kernels, pass_vals)]
    db = {"workloads": {}}
    if out.exists():
        old = json.loads(out.read_text())
        db = old if "workloads" in old else {"workloads": {}}
    db["workloads"][workload] = rec
    db["note"] = ("per workload key (bench.py config.key): fabric (L2 <-> Infinity Cache / HBM) bytes per "
                  "launch of the timed path-kernel dispatch and pipe ratios; tools/pmc.sh + tools/pmc_traffic.py")
    out.write_text(json.dumps(db, indent=1) + "\n")
    print(json.dumps({workload: {k: v for k, v in rec.items() if k != "raw"}}))


if __name__ == "__main__":
    main()
