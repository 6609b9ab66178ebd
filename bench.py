#!/usr/bin/env python3
"""Headline benchmark: Mrays/s + frame ms, synthetic 1M-triangle BVH scene, 512x512x64spp.

BASELINE.json metric: "Mrays/s + frame ms at 512x512x64spp, 1M-tri BVH scene, 1/2/4/8 MI355X".
Workload: N random triangles (centres U[-1,1]^3, vertices c + U[-h,h]^3,
h = N^-1/3, numpy default_rng(seed)), a 2-triangle floor, mirror material (Ks .5), one quad
+ one point light, balls_low camera, accel bvh, reference semantics (MAX_DEPTH 4, no glossy).

One step = one frame (renderScene, main.cpp:525-738) of the whole hot path on device-resident
inputs: every pixel sample, every closest-hit and shadow ray, the per-pixel ordered reduce and,
for N > 1, the RCCL gather of the tile shards to rank 0 plus their reassembly.  Frames are
tile-sharded (16x16 tiles, tile t -> rank t mod N), so scaling is STRONG (fixed frame).

Rays = closest-hit + shadow traversals per frame, counted by the kernel in an untimed stats
frame (identical every frame: the keyed RNG makes the frame deterministic).

Prints ONE JSON line on rank 0.  Launch for N > 1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
# the vector-memory ceiling of the path kernel's access shape (dependent 64-B per-lane record
# gathers at 6 waves/SIMD), measured by tools/gather_ceiling.hip on one MI355X
CEILING_JSON = ROOT / "profiles" / "gather_ceiling.json"
NODE_BYTES, PRIM_BYTES = 64, 48  # one inner-node record (both child boxes), one primitive record
# shadow tree (drt_layout.hpp): one 4-ary record (four quantised child boxes + descriptors), and the
# exact leaf-box record an in-range shadow hit is checked against
WIDE_BYTES, LEAFBOX_BYTES = 64, 32
CAMERA = dict(eye=(2.1, 1.3, 1.7), at=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0), fovy=45.0, hither=0.01)
FLOOR = np.array([[-4, -4, -1.2, 4, -4, -1.2, 4, 4, -1.2], [-4, -4, -1.2, 4, 4, -1.2, -4, 4, -1.2]], np.float32)


def synthetic_triangles(n, seed=1):
    rng = np.random.default_rng(seed)
    h = n ** (-1.0 / 3.0)
    c = rng.uniform(-1.0, 1.0, size=(n, 1, 3))
    v = c + rng.uniform(-h, h, size=(n, 3, 3))
    return np.concatenate([v.astype(np.float32).reshape(n, 9), FLOOR])


def populate(scene, tris, res, spp, aperture=0.0, focal=1.0, accel="bvh", ks=0.5):
    """Same calls for the product scene and the oracle scene (P3F-equivalent content)."""
    scene.set_camera(CAMERA["eye"], CAMERA["at"], CAMERA["up"], CAMERA["fovy"], CAMERA["hither"], res, res,
                     aperture, focal)
    scene.set_background((0.078, 0.361, 0.753))
    scene.set_accel(accel)
    scene.set_spp(spp)
    scene.add_light_quad((4, 3, 2), (1, 1, 1), (4, 2, 2), (3, 3, 2), 16)
    scene.add_light_point((-3, 1, 5), (1, 1, 1))
    scene.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), ks, 30.0827, 0, 1)
    scene.add_triangles(tris)


def balls_low_path(res, spp, accel):
    """BASELINE config C2: P3D_Scenes/balls_low (spheres + plane, 2 quad + 1 point light) as P3F
    text with resolution / spp / accel set (tests/scenegen.py restates the scene file)."""
    import tempfile

    from tests import scenegen

    d = Path(tempfile.mkdtemp(prefix="drt_bench_"))
    return scenegen.write(d, "balls_low.p3f", scenegen.balls_low_text(res=(res, res), spp=spp, accel=accel))


def make_scene(mod, args, tris, ext):
    """The bench scene for the product (mod = distributionraytracer_amd) or the oracle."""
    if args.scene == "balls_low":
        return mod.Scene.load_p3f(balls_low_path(args.res, args.spp, ext["accel"]))
    s = mod.Scene.new() if hasattr(mod.Scene, "new") else mod.Scene()
    populate(s, tris, args.res, args.spp, ext["aperture"], ext["focal"], ext["accel"], ext["ks"])
    return s


def cpu_baseline(args, tris, res, spp, seed, target_s, threads, ext):
    """The CPU oracle (C++/OpenMP restatement of the reference, oracle/) timed on this host on a
    bounded sample: a band of full rows of the SAME frame."""
    from oracle import oracle as O

    O.build()
    s = make_scene(O, args, tris, ext)
    kw = {k: ext[k] for k in ("max_depth", "roughness", "light_spp")}
    t0 = time.time()
    s.build()
    build_s = time.time() - t0
    mid = res // 2
    t0 = time.time()
    _, st = s.render(seed=seed, threads=threads, rows=(mid, mid + 1), **kw)
    per_row = max(time.time() - t0, 1e-3)
    rows = int(max(1, min(res, target_s / per_row)))
    y0 = max(0, mid - rows // 2)
    t0 = time.time()
    _, st = s.render(seed=seed, threads=threads, rows=(y0, y0 + rows), **kw)
    dt = time.time() - t0
    rays = st["closest_calls"] + st["shadow_calls"]
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"rows {y0}-{y0 + rows - 1} of the {res}x{res}x{spp}spp frame ({rows * res * spp} samples, "
                      f"{rays} rays) in {dt:.1f} s; oracle BVH build {build_s:.1f} s",
            "seconds": round(dt, 2), **host_cpu_info(),
            # the oracle against the reference itself, same scenes, measured in the build container
            # (DESIGN.md §5): per thread the oracle is 1.2-1.3x the reference and it scales better
            # (the reference opens a nested OpenMP region and allocates per pixel)
            "calibration": {"oracle_over_reference_1_thread": {"1M_tris": 1.30, "100k_tris": 1.18},
                            "oracle_over_reference_8_threads": {"1M_tris": 2.46, "100k_tris": 1.44},
                            "source": "DESIGN.md §5 (512^2 x 1 spp BVH frames, 8-core container, BASELINE.md)"}}


def host_cpu_info():
    """The host's CPUs as this process sees them: nproc, the affinity set the oracle threads run
    on, and the cgroup CPU quota (cpu.max) that may cap them below that."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    return info


def interval_union(starts, ends):
    """Total length of the union of [start, end) intervals."""
    tot, cur_s, cur_e = 0.0, None, None
    for a, b in sorted(zip(starts, ends)):
        if cur_e is None or a > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = a, b
        else:
            cur_e = max(cur_e, b)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def load_ceiling():
    """The measured ceilings of the path kernel's access shape (profiles/gather_ceiling.json,
    tools/gather_ceiling.hip): dependent 64-B per-lane record gathers from an L1/L2-resident table
    (the vector-memory path's own rate, the bound) and the L2 <-> fabric line rate of the same
    gathers from a table past the caches (every record a 128-B line read)."""
    try:
        c = json.loads(CEILING_JSON.read_text())
        return {"peak_GB_per_s": c["peak_GB_per_s"], "table_bytes": c["peak_table_bytes"],
                "fabric_line_GB_per_s": c.get("fabric_line_GB_per_s"),
                "source": "profiles/gather_ceiling.json (tools/gather_ceiling.hip)"}
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="synthetic", choices=["synthetic", "balls_low"],
                    help="synthetic triangle soup (headline, C3, C4) or P3D_Scenes balls_low (C2)")
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--seed", type=int, default=1)
    # BASELINE configs C3/C4; defaults are the headline workload
    ap.add_argument("--aperture", type=float, default=0.0, help="thin-lens aperture ratio (C4: 8)")
    ap.add_argument("--focal", type=float, default=1.0, help="focal ratio (C4: 1)")
    ap.add_argument("--roughness", type=float, default=0.0, help="glossy reflection (C4: 0.1)")
    ap.add_argument("--max-depth", type=int, default=4, help="MAX_DEPTH (C4: 8)")
    ap.add_argument("--light-spp", type=int, default=1, help="shadow samples per quad light (C3: 4)")
    ap.add_argument("--accel", default="bvh", choices=["bvh", "grid", "none"], help="accelerator (scene.h:22)")
    ap.add_argument("--ks", type=float, default=0.5, help="material Ks (0: no mirror bounces; diagnostics)")
    ap.add_argument("--check-frame", action="store_true",
                    help="after timing, rank 0 checks the assembled frame against a whole-frame render (bitwise)")
    ap.add_argument("--frames-in-flight", type=int, default=0, choices=[0, 1, 2, 3, 4],
                    help="frames pipelined on separate streams and scratch slots, so that a frame's start "
                         "overlaps the previous frame's tail (0: 1 for a wavefront AA / Whitted frame on one "
                         "GPU, 2 otherwise.  Round 5, "
                         "wavefront replay: a whole frame alone 62.4 ms, two in flight 65.3 ms per frame — "
                         "the next frame's persistent chain pass holds the CUs the replay launches wait for; "
                         "a rank's 1/8 shard 10.1 ms alone, 8.87 ms with two in flight, 8.83 with three, "
                         "profiles/r05_frames_in_flight.jsonl, r05_shard_scaling_pipe*.json)")
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="untimed frames before the warmup steps until this much wall time has passed: the "
                         "GPU's clocks settle after the idle scene build (measured: with 2 warmup frames the "
                         "timed frames ran 3 %% slower than the steady 87.8 ms)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-load-timing", action="store_true",
                    help="skip the P3F leg: the synthetic scene written as a .p3f file (by a child process "
                         "during the scene build and the stats frames, waited for before the timed frames) and "
                         "parsed + built after the timed region (f1: Scene::load_p3f + BVH::Build, "
                         "scene.cpp:565-594, bvh.cpp:27-227)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    # f1 leg: the same scene as a P3F file, written by a child process during the scene build and the stats
    # frames (np.savetxt of 3M vertices takes ~10 s of one core), waited for before the settle frames, and
    # parsed and built after the timed region
    p3f_writer, p3f_path = None, None
    # Started before anything touches the GPU, and not under a profiler (rocprofv3 preloads its
    # library into every child, and with --pmc that library would initialise the GPU in the writer).
    profiled = "rocprof" in os.environ.get("LD_PRELOAD", "")
    if rank == 0 and args.scene == "synthetic" and not args.no_load_timing and not profiled:
        import subprocess
        import tempfile

        p3f_path = Path(tempfile.gettempdir()) / f"drt_bench_{os.getpid()}_{args.tris}.p3f"
        code = ("import sys; sys.path.insert(0, %r); from tests import scenegen as sg; "
                "sg.write_synthetic_p3f(%r, %d, res=(%d, %d), spp=%d, accel=%r, seed=%d, aperture=%r, focal=%r)"
                % (str(ROOT), str(p3f_path), args.tris, args.res, args.res, args.spp, args.accel, args.seed,
                   args.aperture, args.focal))
        p3f_writer = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.DEVNULL)
    import torch
    import torch.distributed as dist

    import distributionraytracer_amd as drt
    from distributionraytracer_amd.sharding import FrameGather, TileLayout

    # one process per GPU; DRT_DIST_BACKEND=gloo (with ranks folded onto the visible devices) only
    # rehearses the multi-rank script path on a box with fewer GPUs than ranks
    backend = os.environ.get("DRT_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count()) if backend != "nccl" else local
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            # RCCL's all-gather kernel needs CU room like any kernel: on a high-priority stream it
            # is dispatched ahead of the other frames' pending persistent blocks
            opts = dist.ProcessGroupNCCL.Options(is_high_priority_stream=True)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev), pg_options=opts)
        else:
            dist.init_process_group(backend)

    def log(*a):
        if rank == 0:
            print(*a, file=sys.stderr, flush=True)

    t0 = time.time()
    tris = synthetic_triangles(args.tris, args.seed) if args.scene == "synthetic" else None
    ext = {"aperture": args.aperture, "focal": args.focal, "roughness": args.roughness,
           "max_depth": args.max_depth, "light_spp": args.light_spp, "accel": args.accel, "ks": args.ks}
    scene = make_scene(drt, args, tris, ext)
    scene.build()
    info = scene.info()
    build_s = time.time() - t0
    log(f"[bench] scene: {info.n_objects} objects, BVH {info.bvh_nodes} nodes, host build {info.build_ms / 1e3:.2f} s "
        f"(total setup {build_s:.1f} s)")
    r = drt.Renderer(dev)
    r.upload(scene)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream

    fkw = {"max_depth": args.max_depth, "roughness": args.roughness, "light_spp": args.light_spp}
    plan = r.plan(r.frame_params(seed=args.seed, shard=rank, n_shards=world, **fkw))
    passes = plan["passes"]
    wavefront = bool(plan.get("wavefront"))
    # frames in flight (--frames-in-flight 0): one on one GPU for a wavefront AA / Whitted frame, whose next
    # frame's chain pass would hold the CUs its replay launches wait for; two otherwise — one-pass frames
    # (C2, 1 ms: launch gaps) and in-order frames (C4: the chain pass's in-order tail) gain from the overlap,
    # and so does a rank's shard on several GPUs (profiles/r05_frames_in_flight.jsonl, r05_configs_pipe*.jsonl)
    pipe = args.frames_in_flight or (1 if world == 1 and wavefront and plan["mode"] != 1 else 2)
    shard_ps = [r.frame_params(seed=args.seed, shard=rank, n_shards=world, slot=j, **fkw) for j in range(pipe)]
    shard_p = shard_ps[0]
    stats_p = r.frame_params(seed=args.seed, shard=rank, n_shards=world, stats=True, **fkw)
    ref_p = r.frame_params(seed=args.seed, shard=rank, n_shards=world, stats=True, reference_order=True, **fkw)
    frame = torch.empty((args.res, args.res, 3), dtype=torch.float32, device="cuda")
    # frames in flight: frame i runs on stream / scratch slot / output buffers i % pipe, so the next
    # frame's kernel fills the CUs the previous frame's tail leaves idle
    streams = [stream] + [torch.cuda.Stream() for _ in range(pipe - 1)]
    frames = [frame] + [torch.empty_like(frame) for _ in range(pipe - 1)]
    if world > 1:
        layout = TileLayout(args.res, args.res, 16, world)
        tiles, floats = r.shard_layout(shard_p)
        if floats != layout.floats_per_shard or tiles != len(layout.tiles_of(rank)):
            raise RuntimeError(f"shard layout mismatch: library {tiles} tiles / {floats} floats, "
                               f"host {len(layout.tiles_of(rank))} / {layout.floats_per_shard}")
        fgs = [FrameGather(layout, device="cuda") for _ in range(pipe)]

    def step(p, j=0):
        s = streams[j]
        with torch.cuda.stream(s):
            if world == 1:
                r.render_device(p, frames[j].data_ptr(), s.cuda_stream)
            else:
                r.render_device(p, fgs[j].shard.data_ptr(), s.cuda_stream)
                gathered = fgs[j].gather()  # RCCL all-gather of the shard buffers over xGMI
                if rank == 0:
                    r.unshard_device(p, gathered.data_ptr(), frames[j].data_ptr(), s.cuda_stream)

    # untimed stats frame: rays, node visits and primitive tests of this rank's shard
    step(stats_p)
    torch.cuda.synchronize()
    st = r.stats()
    keys = ["closest_rays", "shadow_rays", "closest_inner", "shadow_inner", "closest_prims", "shadow_prims",
            "closest_leaf", "shadow_leaf", "samples", "wave_node_iters", "wave_path_iters", "lane_path_iters",
            "cycles_refill", "cycles_node", "cycles_shade", "stack_pushes", "stack_spills",
            "wave_leaf_iters", "cycles_leaf", "wide_shadow_rays", "wide_inner", "wide_leaf", "wide_prims",
            "wide_verify"]
    # untimed reference-order stats frame (every shadow query on the reference's binary tree, one
    # pass): §8(d)'s algorithmic bytes on the reference tree, the basis of rounds 1-3's roofline
    step(ref_p)
    torch.cuda.synchronize()
    st_ref = r.stats()
    bytes_ref_tree = NODE_BYTES * (st_ref["closest_inner"] + st_ref["shadow_inner"]) + \
        PRIM_BYTES * (st_ref["closest_prims"] + st_ref["shadow_prims"])
    mine = torch.tensor([st[k] for k in keys], dtype=torch.float64, device="cuda")
    tot = mine.clone()
    if world > 1:
        dist.all_reduce(tot)
    tot = dict(zip(keys, tot.tolist()))
    mine = dict(zip(keys, mine.tolist()))
    rays_frame = tot["closest_rays"] + tot["shadow_rays"]

    # the f1 leg's P3F writer (one core, ~10 s at 1M triangles) finishes before the settle, warmup and
    # timed frames, so that nothing else of this run shares the host while they run
    p3f_wait_s = 0.0
    if p3f_writer is not None:
        t_w = time.perf_counter()
        try:
            p3f_writer.wait(timeout=300)
        except Exception:  # noqa: BLE001 (the f1 leg reports the failure below)
            pass
        p3f_wait_s = time.perf_counter() - t_w
        log(f"[bench] waited {p3f_wait_s:.1f} s for the P3F writer before the timed frames")
    # clock settle: as many untimed frames as fill --settle-s (one frame timed first; the count is
    # the max over ranks, since every frame of a multi-rank run holds a collective)
    settle = 0
    if args.settle_s > 0:
        t_s = time.perf_counter()
        step(shard_ps[0], 0)
        torch.cuda.synchronize()
        n_t = torch.tensor([int(args.settle_s / max(1e-3, time.perf_counter() - t_s))], device="cuda")
        if world > 1:
            dist.all_reduce(n_t, op=dist.ReduceOp.MAX)
        settle = 1 + int(n_t.item())
        for i in range(1, settle):
            step(shard_ps[i % pipe], i % pipe)
    for i in range(args.warmup):
        step(shard_ps[i % pipe], i % pipe)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(shard_ps[i % pipe], i % pipe)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    # roofline.kernel_ms: device time the path kernel held per step over the timed region — the
    # union of the timed frames' path-kernel spans (HIP events on each frame's stream, one device
    # clock) divided by the steps.  Frames in flight overlap, so a single frame's span also holds
    # its wait for the other frame's blocks; the union counts every instant once.
    try:
        ps, pe, _ = r.frame_spans(args.steps)
        kernel_ms = interval_union(ps, pe) / max(1, len(ps))
    except AttributeError:  # an A/B build (DRT_LIBRARY) older than drt_frame_spans
        kernel_ms = None

    # the path kernel of frames rendered one at a time (untimed, after the timed region): its
    # launch duration alone, for the rocprof per-dispatch average
    serial = 3
    for _ in range(serial):
        r.render_device(shard_p, (frames[0] if world == 1 else fgs[0].shard).data_ptr(), sptr)
    torch.cuda.synchronize()
    path_ms, total_ms = r.frame_times(serial)
    try:
        pass1_ms, pass2_ms = r.frame_pass_times(serial)
    except AttributeError:  # an A/B build (DRT_LIBRARY) older than drt_frame_pass_times
        pass1_ms, pass2_ms = [], []
    stage_ms = None  # the last serial frame's pass-2 launches (wf_gen, stream, wf_combine), HIP events
    if wavefront:
        try:
            stage_ms = r.frame_stage_times()
        except (AttributeError, RuntimeError):  # (an A/B build older than drt_frame_stage_times)
            stage_ms = None
    frame_check = None
    if args.check_frame:
        step(shard_p)  # assemble one more frame, then compare it with a one-shot whole frame
        torch.cuda.synchronize()
        if rank == 0:
            whole = torch.empty_like(frame)
            r.render_device(r.frame_params(seed=args.seed, **fkw), whole.data_ptr(), sptr)
            torch.cuda.synchronize()
            frame_check = bool(torch.equal(whole.view(torch.int32), frame.view(torch.int32)))
        if world > 1:
            dist.barrier()
    host_frame_ms = None
    if world == 1:
        # PCIe-inclusive variant (not `value`): drt_render with the frame copied to host memory
        r.render(seed=args.seed, **fkw)  # first call allocates the context's host-path buffers
        t_h = time.perf_counter()
        r.render(seed=args.seed, **fkw)
        host_frame_ms = (time.perf_counter() - t_h) * 1e3
    serial_ms = float(np.mean(path_ms)) if len(path_ms) else float("nan")
    if kernel_ms is None:
        kernel_ms = serial_ms
    bytes_launch = NODE_BYTES * (mine["closest_inner"] + mine["shadow_inner"]) + \
        PRIM_BYTES * (mine["closest_prims"] + mine["shadow_prims"] + mine["wide_prims"]) + \
        WIDE_BYTES * mine["wide_inner"] + LEAFBOX_BYTES * mine["wide_verify"]
    achieved = bytes_launch / (kernel_ms * 1e-3) / 1e9
    ceiling = load_ceiling()
    traffic = None
    valu_busy = None
    dflt = {"aperture": 0.0, "focal": 1.0, "roughness": 0.0, "max_depth": 4, "light_spp": 1, "accel": "bvh", "ks": 0.5}
    extras = [f"{k}{v if isinstance(v, str) else format(v, 'g')}" for k, v in ext.items() if v != dflt[k]]
    head = f"tris{args.tris}" if args.scene == "synthetic" else args.scene
    workload_key = "_".join([f"{head}_res{args.res}_spp{args.spp}"] + extras)
    tj = Path(args.traffic_json)
    pmc = {}
    read_bytes = None
    tr_rec = None
    if world == 1 and tj.exists():
        try:
            # tools/pmc_traffic.py records one entry per workload key: fabric bytes per launch and the
            # pipe ratios (VALU busy against the gfx950 issue peak: a wave64 VALU instruction occupies
            # a SIMD for 2 cycles; kernel cycles = GRBM_GUI_ACTIVE / 8, the counter sums the 8 XCDs)
            tr = json.loads(tj.read_text()).get("workloads", {}).get(workload_key)
            tr_rec = tr
            if tr:
                traffic = tr.get("hbm_bytes_per_launch")
                valu_busy = tr.get("valu_busy")
                pmc = {k: round(tr[k], 4) for k in ("l1_hit_rate", "tcc_hit_rate", "ta_busy", "td_busy", "salu_per_valu")
                       if tr.get(k) is not None}
                pmc["read_bytes_method"] = tr.get("read_bytes_method")
                read_bytes = tr.get("read_bytes")
        except Exception:
            traffic = None

    # Two-level gather model of the path kernel: every record read costs the
    # vector-memory path's L1/L2-resident gather rate, except the records that miss the L2, which
    # cost the rate measured for gathers from a table past the caches.  Missed records = fabric line
    # reads (128 B each, PMC) — one per missed 64-B record, as the calibration table measured.
    model = None
    if read_bytes and ceiling and ceiling.get("fabric_line_GB_per_s"):
        miss = read_bytes / 128.0
        hit_bytes = max(0.0, bytes_launch - 64.0 * miss)
        t_hit = hit_bytes / (ceiling["peak_GB_per_s"] * 1e9) * 1e3
        t_miss = 64.0 * miss / (ceiling["fabric_line_GB_per_s"] / 2.0 * 1e9) * 1e3
        model = {"t_ms": round(t_hit + t_miss, 3), "t_l2_resident_ms": round(t_hit, 3),
                 "t_fabric_ms": round(t_miss, 3), "missed_records": int(miss),
                 "frac": round((t_hit + t_miss) / kernel_ms, 4)}
    # Per pass (a two-pass frame: the closest-chain launch, then the replay launch): device time of
    # each launch in the frames rendered alone after the timed region, its executed algorithmic bytes
    # (pass 1 traverses the closest-hit queries, pass 2 the shadow queries), its fabric reads from
    # the PMC record's per-launch entries, and its place against the same ceilings.
    pass_rows = None
    if passes == 2 and len(pass1_ms):
        b1 = NODE_BYTES * mine["closest_inner"] + PRIM_BYTES * mine["closest_prims"]
        b2 = bytes_launch - b1
        pmc_passes = (tr_rec or {}).get("passes") or [None, None]
        pass_rows = []
        for name, ms, b, pp in (("closest_chain", float(np.mean(pass1_ms)), b1, pmc_passes[0]),
                                ("replay", float(np.mean(pass2_ms)), b2, pmc_passes[1])):
            row = {"pass": name, "ms": round(ms, 3), "bytes": int(b), "achieved": round(b / (ms * 1e-3) / 1e9, 1)}
            if name == "replay":
                # the stream kernel: trace_stream (BVH), grid_stream over the compact queries (Grid, round 6) or
                # the path kernel's MODE_QSTREAM over the marker layout (DRT_GRID_STREAM=0 / DRT_WAVEFRONT_COMPACT=0)
                compact = os.environ.get("DRT_WAVEFRONT_COMPACT", "1") != "0" and (
                    args.accel == "bvh" or os.environ.get("DRT_GRID_STREAM", "1") != "0")
                # (round 6: a triangle scene's Grid frame answers them on its shadow tree, trace_stream GV, and
                # the undecided ones on grid_stream; DRT_GRID_SHADOW_TREE=0 keeps grid_stream for all)
                gv = compact and args.accel == "grid" and os.environ.get("DRT_GRID_SHADOW_TREE", "1") != "0"
                stream_name = ("trace_stream<shadow>" if args.accel == "bvh" else
                               "trace_stream<Grid shadow tree> + grid_stream<undecided>" if gv else
                               "grid_stream" if compact else "path_persistent<GRID> query stream")
                row["kernels"] = (f"wf_gen + {stream_name} + wf_combine" if wavefront else
                                  f"path_persistent<{args.accel.upper()}> replay")
                if stage_ms:
                    # each launch of the wavefront pass 2 on its own: its device time in
                    # the last serial frame, and the bytes it streams — wf_gen writes the query records (32 B;
                    # BVH: real queries only, packed per 64-slot group) and every (level, pair)'s Phong factors
                    # (8 B) plus a 16-B record per level; the
                    # stream moves the pass's algorithmic shadow-tree bytes; wf_combine reads the answers
                    # (1 B), factors and level records and writes the frame (12 B per pixel)
                    levels = args.max_depth + 1
                    n_quad = 1 if args.scene == "synthetic" else 2
                    pairs = n_quad * max(1, args.light_spp) + 1
                    slots = plan["sample_slots"]
                    if compact:  # compact queries: records of the real queries only (WfArgs::compact)
                        gen_b = mine["shadow_rays"] * 32 + slots * levels * (pairs * 8 + 16)
                    else:  # the marker layout: every (level, pair) slot
                        gen_b = slots * levels * (pairs * 40 + 16)
                    comb_b = slots * levels * (pairs * 9 + 16) + 12 * slots // max(1, args.spp)
                    la = {}
                    for key, label, bb in (("wf_gen", "wf_gen", gen_b), ("stream", stream_name, b),
                                           ("wf_combine", "wf_combine (reduce folded in)", comb_b)):
                        lm = float(stage_ms[key])
                        e = {"kernel": label, "ms": round(lm, 3), "bytes": int(bb),
                             "achieved": round(bb / max(1e-9, lm * 1e-3) / 1e9, 1)}
                        if key == "stream" and ceiling:
                            e["frac"] = round(e["achieved"] / ceiling["peak_GB_per_s"], 4)
                        elif key != "stream":
                            e["hbm_frac"] = round(e["achieved"] / HBM_PEAK_GBS, 4)
                        la[key] = e
                    row["launches"] = la
            if ceiling:
                row["frac"] = round(row["achieved"] / ceiling["peak_GB_per_s"], 4)
            if pp and pp.get("read_bytes") is not None:
                row["fabric_read_bytes"] = pp["read_bytes"]
                row["write_bytes"] = pp.get("write_size_bytes")
                if ceiling and ceiling.get("fabric_line_GB_per_s"):
                    miss = pp["read_bytes"] / 128.0
                    th = max(0.0, b - 64.0 * miss) / (ceiling["peak_GB_per_s"] * 1e9) * 1e3
                    tm = 64.0 * miss / (ceiling["fabric_line_GB_per_s"] / 2.0 * 1e9) * 1e3
                    row["two_level_model_ms"] = round(th + tm, 3)
                    row["two_level_frac"] = round((th + tm) / ms, 4)
                for k in ("valu_busy", "tcc_hit_rate"):
                    if pp.get(k) is not None:
                        row[k] = round(pp[k], 4)
            pass_rows.append(row)
    value = rays_frame * args.steps / dt / 1e6
    out = {
        "metric": "Mrays/s + frame ms at 512x512x64spp, 1M-tri BVH scene, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic (seeded random triangle soup, SURVEY.md §8d)" if args.scene == "synthetic" else
                 "balls_low scene (reference P3F content, tests/scenegen.py)"),
        "config": {"workload": (f"synthetic {args.tris} triangles + floor" if args.scene == "synthetic" else
                                "P3D_Scenes balls_low (10 spheres + plane)")
                               + f", {args.accel.upper()}, {args.res}x{args.res}, {args.spp} spp, MAX_DEPTH {args.max_depth}, "
                               + ("1 quad + 1 point light" if args.scene == "synthetic" else "2 quad + 1 point light")
                               + (f", DoF aperture {args.aperture:g} focal {args.focal:g}" if args.aperture else "")
                               + (f", roughness {args.roughness:g}" if args.roughness else "")
                               + (f", {args.light_spp} quad-light samples" if args.light_spp > 1 else ""),
                   "scene": args.scene, "tris": args.tris if args.scene == "synthetic" else 0, "res": args.res, "spp": args.spp, "accel": args.accel, "key": workload_key,
                   "parallelism": f"tile-shard x{world}" + (" + RCCL all-gather" if world > 1 else ""),
                   "frames_in_flight": pipe, "settle_frames": settle},
        # bound: the per-CU vector-memory path serving dependent 64-B per-lane record gathers (TD
        # busy 98 %), peak = tools/gather_ceiling.hip's L1/L2-resident rate; achieved =
        # algorithmic record bytes (64 B per inner-node visit + 48 B per primitive test) per second
        # of path-kernel device time.  traffic: PMC-measured L2 <-> fabric bytes per launch (reads
        # from the request-size counters, tools/pmc_traffic.py); fabric_frac against the measured
        # fabric line rate of the same gathers, hbm_frac against the 8 TB/s HBM figure.
        "roofline": {"bound": "vmem_gather", "achieved": round(achieved, 1),
                     "peak": ceiling["peak_GB_per_s"] if ceiling else None, "unit": "GB/s",
                     "frac": round(achieved / ceiling["peak_GB_per_s"], 4) if ceiling else None,
                     "traffic": traffic,
                     "fabric_frac": round(traffic / (kernel_ms * 1e-3) / 1e9 / ceiling["fabric_line_GB_per_s"], 4)
                     if traffic and ceiling and ceiling.get("fabric_line_GB_per_s") else None,
                     "hbm_frac": round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                     "valu_busy": round(valu_busy, 4) if valu_busy else None,
                     "pmc": pmc or None,
                     "two_level_model": model,
                     "kernel": f"path_persistent<{args.accel.upper()}>" + (
                         (" closest chain + wavefront replay (wf_gen, trace_stream, wf_combine)" if args.accel == "bvh" else
                          (" closest chain + wavefront replay (wf_gen, trace_stream on the Grid's shadow tree + grid_stream, "
                           "wf_combine)" if os.environ.get("DRT_GRID_SHADOW_TREE", "1") != "0" else
                           " closest chain + wavefront replay (wf_gen, grid_stream, wf_combine)")) if wavefront else
                         " closest chain + replay" if passes == 2 else ""),
                     "bytes_per_launch": int(bytes_launch),
                     "kernel_ms": round(kernel_ms, 3), "kernel_ms_serial": round(serial_ms, 3),
                     # §8(d)'s bytes (64 B per inner visit + 48 B per primitive test) on the reference's
                     # binary tree for every query (a DRT_FRAME_REFERENCE_ORDER stats frame): the basis
                     # rounds 1-3 quoted, over the same kernel time
                     "bytes_ref_tree": int(bytes_ref_tree),
                     "frac_ref_tree": round(bytes_ref_tree / (kernel_ms * 1e-3) / 1e9 / ceiling["peak_GB_per_s"], 4)
                     if ceiling else None,
                     "passes": pass_rows,
                     "pass_sum_ms": round(float(np.mean(pass1_ms) + np.mean(pass2_ms)), 3) if len(pass1_ms) else None,
                     "ceiling": ceiling},
        "host_output_frame_ms": None if host_frame_ms is None else round(host_frame_ms, 3),
        **({"frame_check_vs_whole_frame": frame_check} if args.check_frame else {}),
        "rays_per_frame": int(rays_frame),
        "samples_per_frame": int(tot["samples"]),
        "msamples_per_s": round(tot["samples"] * args.steps / dt / 1e6, 2),
        "bytes_per_ray": round(bytes_launch / max(1.0, mine["closest_rays"] + mine["shadow_rays"]), 1),
        "node_visits_per_ray": round((tot["closest_inner"] + tot["shadow_inner"] + tot["closest_leaf"] +
                                      tot["shadow_leaf"] + tot["wide_inner"] + tot["wide_leaf"]) / max(1.0, rays_frame), 2),
        # shadow queries on the 4-ary shadow tree: their share and records per query
        "shadow_tree": {"share": round(tot["wide_shadow_rays"] / max(1.0, tot["shadow_rays"]), 4),
                        "inner_per_query": round(tot["wide_inner"] / max(1.0, tot["wide_shadow_rays"]), 2),
                        "leaf_per_query": round(tot["wide_leaf"] / max(1.0, tot["wide_shadow_rays"]), 2),
                        "prims_per_query": round(tot["wide_prims"] / max(1.0, tot["wide_shadow_rays"]), 2),
                        "verify_per_query": round(tot["wide_verify"] / max(1.0, tot["wide_shadow_rays"]), 3)},
        "setup_s": round(build_s, 2),  # scene from in-memory triangles + BVH build (the P3F path: "load")
        # fraction of lanes doing useful work in the node loop / in the path loop (wave64)
        # (Grid: a wave iteration also walks empty cells, several per lane, so visits per wave
        # iteration is not a lane fraction there; tools/grid_diag.py has the Grid's own counters)
        "simd_eff": {"node_loop": round((tot["closest_inner"] + tot["shadow_inner"] + tot["closest_leaf"] +
                                         tot["shadow_leaf"] + tot["wide_inner"] + tot["wide_leaf"] + tot["wide_verify"])
                                        / max(1.0, 64 * tot["wave_node_iters"]), 3)
                     if args.accel != "grid" else None,
                     "path_loop": round(tot["lane_path_iters"] / max(1.0, 64 * tot["wave_path_iters"]), 3),
                     # BVH leaf block only (the Grid stepper has no separate leaf block)
                     "leaf_block": round((tot["closest_leaf"] + tot["shadow_leaf"] + tot["wide_leaf"]) /
                                         (64 * tot["wave_leaf_iters"]), 3) if tot["wave_leaf_iters"] else None},
        # traversal-stack pushes per ray and the share that went past the LDS part (scratch)
        "stack": {"pushes_per_ray": round(tot["stack_pushes"] / max(1.0, rays_frame), 2),
                  "spill_frac": round(tot["stack_spills"] / max(1.0, tot["stack_pushes"]), 4)},
        # share of the persistent kernel's wave cycles per loop section (stats frame)
        "cycle_share": {k: round(tot["cycles_" + k] / max(1.0, tot["cycles_refill"] + tot["cycles_node"] +
                                                           tot["cycles_shade"]), 3)
                        for k in ("refill", "node", "shade")},
        # share of the node section spent in the leaf (primitive test) block
        "leaf_share_of_node": round(tot["cycles_leaf"] / max(1.0, tot["cycles_node"]), 3),
        "leaf_iter_frac": round(tot["wave_leaf_iters"] / max(1.0, tot["wave_node_iters"]), 3),
        # s_memtime cycles per wave-level iteration (stats frame; stamps cost some cycles themselves)
        "cycles_per_iter": {"node": round(tot["cycles_node"] / max(1.0, tot["wave_node_iters"]), 1),
                            "leaf_block": round(tot["cycles_leaf"] / max(1.0, tot["wave_leaf_iters"]), 1),
                            "shade": round(tot["cycles_shade"] / max(1.0, tot["wave_path_iters"]), 1)},
    }
    if p3f_writer is not None:  # f1: Scene::load_p3f + BVH::Build of the file (the reference: 65 s)
        try:
            p3f_writer.wait(timeout=300)
            drt_scene_bytes = p3f_path.stat().st_size
            t_l = time.perf_counter()
            fs = drt.Scene.load_p3f(p3f_path)
            parse_s = time.perf_counter() - t_l
            t_l = time.perf_counter()
            fs.build()
            fbuild_s = time.perf_counter() - t_l
            same = fs.info().n_objects == info.n_objects and fs.info().bvh_nodes == info.bvh_nodes
            out["load"] = {"p3f_bytes": drt_scene_bytes, "parse_s": round(parse_s, 2), "build_s": round(fbuild_s, 2),
                           "load_build_s": round(parse_s + fbuild_s, 2), "same_scene": bool(same),
                           "writer_wait_s": round(p3f_wait_s, 1),
                           "note": "setup_s builds from in-memory triangles; this is the P3F file path"}
            log(f"[bench] P3F {drt_scene_bytes / 1e6:.0f} MB: parse {parse_s:.2f} s, BVH build {fbuild_s:.2f} s")
            del fs
        except Exception as e:  # reported, never required
            out["load"] = {"error": repr(e)}
            p3f_writer.kill()
        finally:
            p3f_path.unlink(missing_ok=True)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        threads = O.host_threads()  # every host core this process may run on (nproc stated in the line)
        try:
            out["cpu_baseline"] = cpu_baseline(args, tris, args.res, args.spp, args.seed, args.cpu_seconds, threads,
                                               ext)
            out["cpu_baseline"]["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        except Exception as e:  # the baseline is reported, never required
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
