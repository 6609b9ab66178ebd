#!/usr/bin/env python3
"""Path-kernel device time per step from a rocprofv3 kernel trace of `bench.py --steps K --warmup W`,
computed the way bench.py computes roofline.kernel_ms from HIP events: the union of the timed
dispatches' [start, end] spans divided by K.  Also the mean duration of the serial frames rendered
after the timed region (roofline.kernel_ms_serial).

Frame order in bench.py (a frame: its non-stats path_persistent dispatch and its second pass's
dispatches): S clock-settle frames (the bench line's config.settle_frames), W warmup, K timed, 3
serial, then (one GPU) 2 drt_render frames.

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
    # A frame is its non-stats path_persistent dispatch plus, on the same stream, the dispatches of its
    # second pass: the persistent replay (FrameMode 6 / 8 / 10) or the wavefront replay (wf_gen_kernel, the
    # non-stats trace_stream, the Grid's non-stats grid_stream or its MODE_QSTREAM (11) dispatch, wf_combine_kernel or, reduce folded in, wf_combine_reduce_kernel; per chunk of
    # sample slots).  Frames in flight interleave across streams.
    rows = []
    for f in Path(a.trace_dir).rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Dispatch_Id"]), r.get("Stream_Id", "0"), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    frames, cur = [], {}
    for _, stream, s0, e0, k in rows:
        targs = k.split("<", 2)[1].split(">")[0].split(",") if "<" in k else []
        if "path_persistent<" in k:
            stats = targs[1].strip() == "true"
            mode = int(targs[2]) if targs[2].strip().isdigit() else -1
            if stats:
                cur[stream] = None
            elif mode in (6, 8, 10, 11) and cur.get(stream) is not None:
                cur[stream].append((s0, e0, k))
            else:
                cur[stream] = [(s0, e0, k)]
                frames.append(cur[stream])
        elif ("wf_gen_kernel" in k or "wf_combine" in k or
              (("trace_stream<" in k and targs[3].strip() == "false") or (
               "grid_stream<" in k and targs[2].strip() == "false"))) and cur.get(stream) is not None:
            cur[stream].append((s0, e0, k))
    names = sorted({k for fr in frames for _, _, k in fr})
    P = max((len(fr) for fr in frames), default=1)
    w0 = settle + a.warmup
    timed_frames = frames[w0:w0 + a.steps]
    timed = [d for fr in timed_frames for d in fr]
    serial_frames = frames[w0 + a.steps:w0 + a.steps + 3]
    union_ms = interval_union([s for s, _, _ in timed], [e for _, e, _ in timed]) / 1e6
    per_pass = {k: round(sum(e - s for s, e, kk in timed if kk == k) / max(1, sum(1 for *_, kk in timed if kk == k))
                         / 1e6, 3) for k in names}
    res = {"kernel": timed[0][2] if timed else None, "kernels": names, "dispatches_per_frame": P, "frames": len(frames),
           "settle_frames": settle,
           "kernel_ms_per_step_union": round(union_ms / max(1, a.steps), 3),
           "pass_ms_mean_timed": per_pass,
           "kernel_ms_serial_mean": round(sum(max(e for _, e, _ in f) - min(s for s, _, _ in f) for f in serial_frames)
                                          / max(1, len(serial_frames)) / 1e6, 3),
           "timed_span_ms": round((max(e for _, e, _ in timed) - min(s for s, _, _ in timed)) / 1e6, 3) if timed else None}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
