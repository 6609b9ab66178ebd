"""Tile-sharded frames across ranks on CPU: the host half of the N>1 path.

Each rank renders with the CPU oracle (standing in for its GPU; the oracle is the parity
checker, see oracle/README), packs its tiles into the shard-compact buffer that
drt_render_device fills on the GPU, and the ranks exchange buffers through the same
FrameGather (all_gather_into_tensor) bench.py uses over RCCL — here over gloo, world size 2.
Rank 0 reassembles the frame with the layout's host mirror of drt_unshard_device and must get
the whole-frame render back bit for bit.  The device-side pack (render_device with n_shards > 1)
and unshard kernels are checked against the same layout by tests/test_gpu_parity.py.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from distributionraytracer_amd.sharding import TileLayout  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_oracle(res, spp, seed):
    import scenegen
    from oracle import oracle as O

    path = Path(os.environ["DRT_TEST_TMP"]) / f"mixed_{res[0]}x{res[1]}.p3f"
    if not path.exists():
        scenegen.write(path.parent, path.name, scenegen.mixed_scene_text(res=res, spp=spp))
    sc = O.Scene.load_p3f(str(path))
    sc.build()
    return sc.render(seed=seed, threads=2)[0]


def _rank_main(rank, world, port, res, spp, seed, tile, out_dir):
    import torch.distributed as dist

    from distributionraytracer_amd.sharding import FrameGather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frame = _render_oracle(res, spp, seed)
        layout = TileLayout(res[0], res[1], tile, world)
        fg = FrameGather(layout, device="cpu")
        fg.shard.copy_(__import__("torch").from_numpy(layout.pack_host(frame, rank)))
        gathered = fg.gather().numpy().copy()
        if rank == 0:
            np.save(os.path.join(out_dir, "frame.npy"), frame)
            np.save(os.path.join(out_dir, "reassembled.npy"), layout.unshard_host(gathered))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("res,tile", [((48, 40), 16), ((37, 29), 8)])
def test_two_rank_gather_reassembles_frame(oracle_mod, tmp_path, res, tile):
    import torch.multiprocessing as mp

    os.environ["DRT_TEST_TMP"] = str(tmp_path)
    # the first render builds the scene file (both ranks then read it)
    _render_oracle(res, 4, 11)
    mp.spawn(_rank_main, args=(2, _free_port(), res, 4, 11, tile, str(tmp_path)), nprocs=2, join=True)
    frame = np.load(tmp_path / "frame.npy")
    back = np.load(tmp_path / "reassembled.npy")
    assert frame.shape == (res[1], res[0], 3)
    assert np.array_equal(frame, back)


@pytest.mark.parametrize("res_x,res_y,tile,n", [(512, 512, 16, 1), (512, 512, 16, 8), (100, 37, 16, 3),
                                                (17, 5, 4, 7), (1024, 1024, 16, 8)])
def test_layout_pack_unshard_roundtrip(res_x, res_y, tile, n):
    rng = np.random.default_rng(res_x * 31 + n)
    frame = rng.random((res_y, res_x, 3), dtype=np.float32)
    lay = TileLayout(res_x, res_y, tile, n)
    # every tile belongs to exactly one shard, shards differ by at most one tile
    owned = sorted(t for s in range(n) for t in lay.tiles_of(s))
    assert owned == list(range(lay.n_tiles))
    counts = [len(lay.tiles_of(s)) for s in range(n)]
    assert max(counts) - min(counts) <= 1 and max(counts) == lay.tiles_per_shard
    gathered = np.concatenate([lay.pack_host(frame, s) for s in range(n)])
    assert gathered.size == n * lay.floats_per_shard
    assert np.array_equal(lay.unshard_host(gathered), frame)


def test_layout_rejects_bad_arguments():
    with pytest.raises(ValueError):
        TileLayout(0, 10)
    with pytest.raises(ValueError):
        TileLayout(10, 10, 16, 0)
