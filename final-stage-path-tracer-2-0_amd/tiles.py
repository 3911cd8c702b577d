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


# ---- the product's tile exchange format (pack_tiles / unpack_tiles) ---------
# fs_frame_gather moves PACK_WORDS uint32 words per pixel: colour (3 floats),
# count, normal (3 floats), depth, material id (low, high word). A rank's
# pack holds max_owned tiles (tile k of rank r is r + k * world) of
# tile_size^2 pixels, row-major inside the tile; pixels and tiles outside the
# frame are zero. ncclGather delivers the packs concatenated in rank order.
PACK_WORDS = 10


def _pack_grid(width, height, world, tile_size):
    tx, ty = tile_grid(width, height, tile_size)
    return tx, ty, (tx * ty + world - 1) // world


def pack_words(planes, width, height, rank, world, tile_size=64):
    """pack_tiles (fs_device.hip) restated on the host. planes: dict with the
    frame's color (H, W, 3) float32, count (H, W) uint32, normal (H, W, 3)
    float32, depth (H, W) float32 and material (H, W) uint64 arrays."""
    tx, ty, owned_max = _pack_grid(width, height, world, tile_size)
    px = np.zeros((height, width, PACK_WORDS), np.uint32)
    px[..., 0:3] = planes["color"].view(np.uint32)
    px[..., 3] = planes["count"]
    px[..., 4:7] = planes["normal"].view(np.uint32)
    px[..., 7] = planes["depth"].view(np.uint32)
    px[..., 8] = (planes["material"] & 0xFFFFFFFF).astype(np.uint32)
    px[..., 9] = (planes["material"] >> 32).astype(np.uint32)
    out = np.zeros((owned_max, tile_size, tile_size, PACK_WORDS), np.uint32)
    for k in range(owned_max):
        t = rank + k * world
        if t >= tx * ty:
            continue
        x0, y0 = (t % tx) * tile_size, (t // tx) * tile_size
        blk = px[y0:y0 + tile_size, x0:x0 + tile_size]
        out[k, :blk.shape[0], :blk.shape[1]] = blk
    return out.reshape(-1)


def gamma8(c):
    """frame.cpp:67-71 (the display bytes unpack_tiles rebuilds)."""
    s = np.clip(c.astype(np.float32), 0.0, 1.0).astype(np.float64)
    return (255.0 * np.power(s, 1.0 / 2.2) + 0.5).astype(np.uint8)


def unpack_words(planes, gathered, width, height, world, self_rank, tile_size=64):
    """unpack_tiles restated: scatters every rank's pack of the rank-ordered
    concatenation `gathered` except self_rank's into planes (the dict of
    pack_words plus display (H, W, 3) uint8, rebuilt from the colour)."""
    tx, ty, owned_max = _pack_grid(width, height, world, tile_size)
    packs = np.asarray(gathered, np.uint32).reshape(world, owned_max, tile_size, tile_size, PACK_WORDS)
    for r in range(world):
        if r == self_rank:
            continue
        for k in range(owned_max):
            t = r + k * world
            if t >= tx * ty:
                continue
            x0, y0 = (t % tx) * tile_size, (t // tx) * tile_size
            h, w = min(tile_size, height - y0), min(tile_size, width - x0)
            blk = packs[r, k, :h, :w]
            sl = (slice(y0, y0 + h), slice(x0, x0 + w))
            planes["color"][sl] = blk[..., 0:3].view(np.float32)
            planes["count"][sl] = blk[..., 3]
            planes["normal"][sl] = blk[..., 4:7].view(np.float32)
            planes["depth"][sl] = blk[..., 7].view(np.float32)
            planes["material"][sl] = blk[..., 8].astype(np.uint64) | (blk[..., 9].astype(np.uint64) << np.uint64(32))
            planes["display"][sl] = gamma8(planes["color"][sl])
    return planes
