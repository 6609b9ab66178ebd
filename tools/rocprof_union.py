#!/usr/bin/env python3
"""Path-kernel device time per step from a rocprofv3 kernel trace of `bench.py --steps K --warmup W`,
computed the way bench.py computes roofline.kernel_ms from HIP events: the union of the timed
dispatches' [start, end] spans divided by K.  Also the mean duration of the serial frames rendered
after the timed region (roofline.kernel_ms_serial).

Dispatch order of the non-stats path_persistent instantiation in bench.py: S clock-settle frames
(the bench line's config.settle_frames), W warmup, K timed, 3 serial, then (one GPU) 2 drt_render
frames.

usage: python tools/rocprof_union.py TRACE_DIR --steps K --warmup W [--settle S | --bench-json F]
"""
import argparse
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import interval_union  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--settle", type=int, default=None, help="clock-settle frames before the warmup")
    ap.add_argument("--bench-json", default=None, help="the profiled run's bench line (settle_frames)")
    a = ap.parse_args()
    settle = a.settle
    if settle is None and a.bench_json:
        settle = json.loads(Path(a.bench_json).read_text())["config"].get("settle_frames", 0)
    settle = settle or 0
    rows = []
    for f in Path(a.trace_dir).rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "path_persistent<" in k and k.split("<", 2)[1].split(",")[1].strip() == "false":
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    # A two-pass frame (in-order frames, and AA frames of refraction-free BVH scenes since round 4)
    # is two dispatches of two instantiations (MODE_SKEL / MODE_CHAIN, then MODE_REPLAY): P passes.
    names = sorted({k for _, _, k in rows})
    P = len(names) if len(names) in (1, 2) else 1
    w0 = settle + a.warmup
    timed = rows[w0 * P:(w0 + a.steps) * P]
    serial = rows[(w0 + a.steps) * P:(w0 + a.steps + 3) * P]
    union_ms = interval_union([s for s, _, _ in timed], [e for _, e, _ in timed]) / 1e6
    frames = [serial[i:i + P] for i in range(0, len(serial), P)]
    per_pass = {k: round(sum(e - s for s, e, kk in timed if kk == k) / max(1, sum(1 for *_, kk in timed if kk == k))
                         / 1e6, 3) for k in names}
    res = {"kernel": timed[0][2] if timed else None, "kernels": names, "passes": P, "dispatches": len(rows),
           "settle_frames": settle,
           "kernel_ms_per_step_union": round(union_ms / max(1, a.steps), 3),
           "pass_ms_mean_timed": per_pass,
           "kernel_ms_serial_mean": round(sum(f[-1][1] - f[0][0] for f in frames) / max(1, len(frames)) / 1e6, 3),
           "timed_span_ms": round((timed[-1][1] - timed[0][0]) / 1e6, 3) if timed else None}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
