"""The profile tools that turn rocprofv3 output into the bench line's figures (CPU only, synthetic CSV).

tools/rocprof_union.py (roofline.kernel_ms against the trace) and tools/pmc_traffic.py (per-pass fabric
bytes) must group a frame's dispatches the way run_frame issues them: the non-stats path_persistent
dispatch of pass 1, then on the same stream / queue its second pass — the persistent replay
(FrameMode 6 / 8 / 10) or the wavefront replay (wf_gen, the non-stats trace_stream, grid_stream or the Grid's
MODE_QSTREAM dispatch, wf_combine; per chunk of sample slots).  Stats frames are skipped, and frames in
flight interleave across streams.
"""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

CHAIN = "void drt::path_persistent<true, false, 7, 6, 2>(drt::SceneArgs, drt::FrameArgs)"
CHAIN_ST = "void drt::path_persistent<true, true, 7, 6, 2>(drt::SceneArgs, drt::FrameArgs)"
GEN = "drt::wf_gen_kernel(drt::SceneArgs, drt::FrameArgs, drt::WfArgs)"
TRACE = "void drt::trace_stream<true, 2, 7, false>(drt::SceneArgs, drt::TraceArgs)"
TRACE_ST = "void drt::trace_stream<true, 2, 7, true>(drt::SceneArgs, drt::TraceArgs)"
COMB = "drt::wf_combine_kernel(drt::SceneArgs, drt::FrameArgs, drt::WfArgs)"
# round 6: the combine with the frame's reduce folded in (the default)
COMBR = "drt::wf_combine_reduce_kernel(drt::SceneArgs, drt::FrameArgs, drt::WfArgs, drt::ReduceArgs, unsigned int)"
QSTREAM = "void drt::path_persistent<true, false, 11, 5, 1>(drt::SceneArgs, drt::FrameArgs)"
GCHAIN = "void drt::path_persistent<true, false, 7, 5, 1>(drt::SceneArgs, drt::FrameArgs)"
REDUCE = "drt::reduce_kernel(drt::ReduceArgs)"


def frame(chain, second, stream, t0, ms=(10, 1, 8, 1)):
    """Dispatches (name, stream, start ns, end ns) of one frame starting at t0 (ms per dispatch)."""
    out, t = [], t0
    for name, d in zip([chain] + second + [REDUCE], list(ms) + [0.1]):
        out.append((name, stream, t, t + int(d * 1e6)))
        t += int(d * 1e6) + 1000
    return out


def write_trace(path: Path, dispatches):
    path.mkdir(parents=True, exist_ok=True)
    with open(path / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Stream_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for i, (name, stream, s, e) in enumerate(dispatches):
            w.writerow([i + 1, stream, name, s, e])


def test_rocprof_union_groups_wavefront_frames(tmp_path):
    wf = [GEN, TRACE, COMB]
    d = []
    d += frame(CHAIN_ST, [GEN, TRACE_ST, COMB], 0, 0)            # the stats frame: skipped
    for k in range(3):                                          # 1 settle + 1 warmup + 1 timed
        d += frame(CHAIN, wf, 0, 100_000_000 * (k + 1))
    d += frame(CHAIN, wf, 0, 500_000_000)                       # serial frame after the timed region
    write_trace(tmp_path / "t", d)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "rocprof_union.py"), str(tmp_path / "t"), "--steps", "1",
                          "--warmup", "1", "--settle", "1"], capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["frames"] == 4 and r["dispatches_per_frame"] == 4
    # the timed frame: 10 + 1 + 8 + 1 ms of dispatches, 3 µs of gaps between them
    assert abs(r["kernel_ms_per_step_union"] - 20.0) < 0.01
    assert abs(r["kernel_ms_serial_mean"] - 20.003) < 0.01
    assert abs(r["pass_ms_mean_timed"][TRACE] - 8.0) < 1e-6


def test_rocprof_union_interleaved_streams_and_grid_qstream(tmp_path):
    # two frames in flight on streams 1 and 2, their dispatches interleaved in issue order; Grid frames
    # whose second pass is MODE_QSTREAM, two chunks each
    wf = [GEN, QSTREAM, COMB, GEN, QSTREAM, COMB]
    a = frame(GCHAIN, wf, 1, 0, ms=(10, 1, 5, 1, 1, 5, 1))
    b = frame(GCHAIN, wf, 2, 3_000_000, ms=(10, 1, 5, 1, 1, 5, 1))
    d = [x for pair in zip(a, b) for x in pair]
    write_trace(tmp_path / "t", d)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "rocprof_union.py"), str(tmp_path / "t"), "--steps", "2",
                          "--warmup", "0", "--settle", "0"], capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["frames"] == 2 and r["dispatches_per_frame"] == 7
    assert r["kernel"] == GCHAIN


def test_pmc_traffic_last_frame_sums_the_second_pass(tmp_path):
    import pmc_traffic

    def row(did, name, q, counter, value):
        return {"Dispatch_Id": did, "Kernel_Name": name, "Queue_Id": q, "Counter_Name": counter, "Counter_Value": value}

    p = tmp_path / "p1"
    p.mkdir()
    rows = []
    did = 0
    for frame_names in ([CHAIN_ST, GEN, TRACE_ST, COMB], [CHAIN, GEN, TRACE, COMB], [CHAIN, GEN, TRACE, COMB]):
        for n in frame_names:
            did += 1
            rows.append(row(did, n, 6, "WRITE_SIZE", 1.0 * did))
    with open(p / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    c = pmc_traffic.dispatch_counters(p)
    fr = pmc_traffic.last_frame(c)
    assert [k[0] for k in fr] == [9, 10, 11, 12]          # the last non-stats frame, all four dispatches
    assert pmc_traffic._sum(c, fr[1:])["WRITE_SIZE"] == 10 + 11 + 12


def test_rocprof_union_counts_the_folded_combine(tmp_path):
    """Round 6: a wavefront frame ends with wf_combine_reduce_kernel (no reduce launch); it is part of the frame."""
    d = []
    for k in range(2):  # 1 warmup + 1 timed
        d += [x for x in frame(CHAIN, [GEN, TRACE, COMBR], 0, 100_000_000 * (k + 1)) if x[0] != REDUCE]
    write_trace(tmp_path / "t", d)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "rocprof_union.py"), str(tmp_path / "t"), "--steps", "1",
                          "--warmup", "1", "--settle", "0"], capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["dispatches_per_frame"] == 4
    assert abs(r["kernel_ms_per_step_union"] - 20.0) < 0.01 and COMBR in r["kernels"]


def test_profile_tools_count_grid_stream(tmp_path):
    """Round 6: a Grid wavefront frame's shadow queries run on grid_stream (non-stats dispatch: last template
    argument false); both tools count it as part of the frame, and skip the stats instantiation."""
    import pmc_traffic

    gs = "void drt::grid_stream<true, 7, false>(drt::SceneArgs, drt::TraceArgs, int, int)"
    gs_st = "void drt::grid_stream<true, 7, true>(drt::SceneArgs, drt::TraceArgs, int, int)"
    gchain_st = GCHAIN.replace("true, false", "true, true")
    d = [x for x in frame(gchain_st, [GEN, gs_st, COMBR], 0, 0) if x[0] != REDUCE]
    for k in range(2):  # 1 warmup + 1 timed
        d += [x for x in frame(GCHAIN, [GEN, gs, COMBR], 0, 100_000_000 * (k + 1)) if x[0] != REDUCE]
    write_trace(tmp_path / "t", d)
    out = subprocess.run([sys.executable, str(ROOT / "tools" / "rocprof_union.py"), str(tmp_path / "t"), "--steps", "1",
                          "--warmup", "1", "--settle", "0"], capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["frames"] == 2 and r["dispatches_per_frame"] == 4 and gs in r["kernels"] and gs_st not in r["kernels"]
    assert abs(r["kernel_ms_per_step_union"] - 20.0) < 0.01

    p = tmp_path / "p1"
    p.mkdir()
    rows = []
    for did, (name, *_rest) in enumerate(d, 1):
        rows.append({"Dispatch_Id": did, "Kernel_Name": name, "Queue_Id": 6, "Counter_Name": "WRITE_SIZE",
                     "Counter_Value": 1.0 * did})
    with open(p / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    c = pmc_traffic.dispatch_counters(p)
    fr = pmc_traffic.last_frame(c)
    assert [k[0] for k in fr] == [9, 10, 11, 12] and fr[2][1] == gs
