"""Tile sharding of one frame across ranks, and the framebuffer gather.

Pixels are independent (main.cpp:603: the reference parallelises the pixel loop) and the keyed
RNG depends only on (seed, pixel, call index), so a frame splits into square tiles dealt
round-robin over a dealing order in which tile row ty is rotated by ty tiles: tile (tx, ty) has
position p = ty * tiles_x + (tx + ty) % tiles_x and belongs to rank p % n_shards, so every rank
takes diagonal stripes of the image rather than the same columns in every row.  Each rank
renders its tiles into a shard-compact buffer (drt_render_device with n_shards > 1): its k-th
tile (position p = shard + k * n_shards) occupies floats [k * tile^2 * 3, (k + 1) * tile^2 * 3),
pixel (px, py) of the tile at (py * tile + px) * 3.
Every shard buffer has the same length (tiles_per_shard = ceil(n_tiles / n_shards) tiles), so
the gather is one all_gather_into_tensor (RCCL over xGMI on GPUs, gloo on CPU) and the frame is
reassembled by drt_unshard_device.  The numpy pack/unshard mirrors below define that layout for
host code and tests; the device path never goes through them.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass(frozen=True)
class TileLayout:
    res_x: int
    res_y: int
    tile: int = 16
    n_shards: int = 1

    def __post_init__(self):
        if self.res_x <= 0 or self.res_y <= 0 or self.tile <= 0 or self.n_shards <= 0:
            raise ValueError(f"invalid tile layout {self}")

    @property
    def tiles_x(self) -> int:
        return (self.res_x + self.tile - 1) // self.tile

    @property
    def tiles_y(self) -> int:
        return (self.res_y + self.tile - 1) // self.tile

    @property
    def n_tiles(self) -> int:
        return self.tiles_x * self.tiles_y

    @property
    def tiles_per_shard(self) -> int:
        return (self.n_tiles + self.n_shards - 1) // self.n_shards

    @property
    def floats_per_shard(self) -> int:
        return self.tiles_per_shard * self.tile * self.tile * 3

    def position_of_tile(self, t: int) -> int:
        """Dealing position of row-major tile t (tile_of_position in drt_kernels.hip)."""
        tx, ty = t % self.tiles_x, t // self.tiles_x
        return ty * self.tiles_x + (tx + ty) % self.tiles_x

    def tile_of_position(self, p: int) -> int:
        ty, r = divmod(p, self.tiles_x)
        return ty * self.tiles_x + (r - ty) % self.tiles_x

    def tiles_of(self, shard: int) -> list[int]:
        """Row-major tile indices rendered by `shard` (drt_frame_params.shard), in buffer order."""
        return [self.tile_of_position(p) for p in range(shard, self.n_tiles, self.n_shards)]

    def tile_origin(self, t: int) -> tuple[int, int]:
        return (t % self.tiles_x) * self.tile, (t // self.tiles_x) * self.tile

    def pack_host(self, frame: np.ndarray, shard: int) -> np.ndarray:
        """Shard-compact buffer of `shard` cut from a full (res_y, res_x, 3) frame; pixels of
        partial edge tiles that fall outside the frame are 0 (the device writes 0 there too)."""
        out = np.zeros((self.tiles_per_shard, self.tile, self.tile, 3), np.float32)
        for k, t in enumerate(self.tiles_of(shard)):
            x0, y0 = self.tile_origin(t)
            blk = frame[y0:y0 + self.tile, x0:x0 + self.tile]
            out[k, :blk.shape[0], :blk.shape[1]] = blk
        return out.reshape(-1)

    def unshard_host(self, gathered: np.ndarray) -> np.ndarray:
        """Full frame from n_shards shard buffers laid end to end (host mirror of
        drt_unshard_device)."""
        g = np.asarray(gathered, np.float32).reshape(self.n_shards, self.tiles_per_shard, self.tile, self.tile, 3)
        frame = np.zeros((self.res_y, self.res_x, 3), np.float32)
        for t in range(self.n_tiles):
            x0, y0 = self.tile_origin(t)
            h = min(self.tile, self.res_y - y0)
            w = min(self.tile, self.res_x - x0)
            p = self.position_of_tile(t)
            frame[y0:y0 + h, x0:x0 + w] = g[p % self.n_shards, p // self.n_shards, :h, :w]
        return frame


class FrameGather:
    """The one collective of a sharded frame: all ranks' shard buffers, end to end, on every
    rank (rank 0 then reassembles the frame).  Buffers are allocated once and reused."""

    def __init__(self, layout: TileLayout, device=None, group=None):
        import torch

        self.layout = layout
        self.group = group
        self.shard = torch.empty(layout.floats_per_shard, dtype=torch.float32, device=device)
        self.gathered = torch.empty(layout.n_shards * layout.floats_per_shard, dtype=torch.float32, device=device)

    def gather(self):
        import torch.distributed as dist

        if self.layout.n_shards == 1:
            self.gathered.copy_(self.shard)
        else:
            dist.all_gather_into_tensor(self.gathered, self.shard, group=self.group)
        return self.gathered
