"""Frame partition used for multi-GPU renders (fs_render_params tiling).

The frame is cut into tile_size x tile_size tiles numbered row-major; rank r
of N owns tiles t with t % N == r (fs_trace.h). The device kernels
(render_kernel, pack_tiles/unpack_tiles in csrc/fs_device.hip) implement the
same mapping; this module restates it for host-side checks and tools.
"""
import numpy as np


def tile_grid(width, height, tile_size=64):
    return (width + tile_size - 1) // tile_size, (height + tile_size - 1) // tile_size


def owned_tiles(width, height, rank, world, tile_size=64):
    tx, ty = tile_grid(width, height, tile_size)
    return list(range(rank, tx * ty, world))


def owner_map(width, height, world, tile_size=64):
    """(height, width) array: rank that renders each pixel."""
    tx, _ = tile_grid(width, height, tile_size)
    y, x = np.mgrid[0:height, 0:width]
    return ((y // tile_size) * tx + (x // tile_size)) % world


def pack(plane, width, height, rank, world, tile_size=64):
    """Owned tiles of `plane` (H, W, ...) as a (max_owned, ts, ts, ...) block."""
    tx, ty = tile_grid(width, height, tile_size)
    max_owned = (tx * ty + world - 1) // world
    out = np.zeros((max_owned, tile_size, tile_size) + plane.shape[2:], plane.dtype)
    for k, t in enumerate(owned_tiles(width, height, rank, world, tile_size)):
        x0, y0 = (t % tx) * tile_size, (t // tx) * tile_size
        blk = plane[y0:y0 + tile_size, x0:x0 + tile_size]
        out[k, :blk.shape[0], :blk.shape[1]] = blk
    return out


def unpack(dest, packed, rank, world, tile_size=64):
    height, width = dest.shape[:2]
    tx, _ = tile_grid(width, height, tile_size)
    for k, t in enumerate(owned_tiles(width, height, rank, world, tile_size)):
        x0, y0 = (t % tx) * tile_size, (t // tx) * tile_size
        h = min(tile_size, height - y0)
        w = min(tile_size, width - x0)
        dest[y0:y0 + h, x0:x0 + w] = packed[k, :h, :w]
    return dest
