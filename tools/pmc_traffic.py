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
    """{(dispatch_id, kernel): {counter: value}} summed over the dispatch's rows; the dispatch's queue
    is kept under the key "__queue"."""
    out = {}
    for f in pass_dir.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), r["Kernel_Name"])
            d = out.setdefault(key, {"__queue": r.get("Queue_Id", "0")})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def last_frame(counters, sub=None):
    """Dispatch keys of the last timed frame: its non-stats path_persistent dispatch (pass 1, or the
    whole one-pass frame), then on the same queue its second pass — the persistent replay (FrameMode
    6 / 8 / 10) or the wavefront replay (wf_gen_kernel, the non-stats trace_stream, the Grid's
    non-stats grid_stream or its MODE_QSTREAM (11) dispatch, wf_combine_kernel or, reduce folded in, wf_combine_reduce_kernel; per chunk of sample slots).
    With `sub`, the last dispatch whose name holds it."""
    if sub:
        keys = sorted(k for k in counters if sub in k[1])
        return [keys[-1]] if keys else []
    frames, cur = [], {}
    for k in sorted(counters):
        q, name, a = counters[k]["__queue"], k[1], _targs(k[1])
        if "path_persistent<" in name:
            if _stats(name):
                cur[q] = None
            elif _mode(name) in (6, 8, 10, 11) and cur.get(q) is not None:
                cur[q].append(k)
            else:
                cur[q] = [k]
                frames.append(cur[q])
        elif ("wf_gen_kernel" in name or "wf_combine" in name or
              (("trace_stream<" in name and len(a) > 3 and a[3] == "false") or (
               "grid_stream<" in name and len(a) > 2 and a[2] == "false"))) and cur.get(q) is not None:
            cur[q].append(k)
    return frames[-1] if frames else []


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


def _sum(counters, keys):
    out = {}
    for k in keys:
        for n, v in counters[k].items():
            if n != "__queue":
                out[n] = out.get(n, 0.0) + v
    return out


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
    pass_vals = [{}, {}]  # a two-pass frame's launches: the closest-chain pass, the replay pass (all its launches)
    pass_kernels = [None, None]
    for p in sorted(x for x in root.iterdir() if x.is_dir()):
        c = dispatch_counters(p)
        fr = last_frame(c, sub)
        if not fr:
            continue
        kernel = " + ".join(k[1] for k in fr)
        # this pass's counters summed over the frame's launches (each counter group is its own pass)
        vals.update(_sum(c, fr))
        if len(fr) > 1:
            pass_kernels = [fr[0][1], " + ".join(k[1] for k in fr[1:])]
            pass_vals[0].update(_sum(c, fr[:1]))
            pass_vals[1].update(_sum(c, fr[1:]))
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
