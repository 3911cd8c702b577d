"""Multi-rank path on CPU: world_size 2 over gloo. Each rank renders its
round-robin tiles (the fs_render_params tiling) with the oracle, packs them,
all_gathers them over gloo and rank 0 reassembles; the result must equal the
single-rank render bit for bit (tiles are independent given the
per-(pixel,sample) seeds)."""
import os
import sys

import numpy as np
import pytest

from conftest import ORACLE, PKG, load_scene

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

W, H, SPP, TS = 40, 36, 2, 16


def _rank(rank, world, port, scene_dir, out_dir):
    sys.path[:0] = [PKG, ORACLE]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fsamd
    import oracle_py
    import tiles

    s = load_scene("c2", scene_dir)
    o = oracle_py.Scene(s.desc_ptr())
    p = fsamd.render_params(W, H, SPP, tile_size=TS, tile_offset=rank, tile_stride=world)
    f = o.render(s.camera(0), p, threads=2)
    own = tiles.owner_map(W, H, world, TS)
    assert np.all(f.count[own == rank] == SPP) and np.all(f.count[own != rank] == 0)
    mine = torch.from_numpy(tiles.pack(f.color, W, H, rank, world, TS))
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        img = np.zeros((H, W, 3), np.float32)
        for r, part in enumerate(parts):
            tiles.unpack(img, part.numpy(), r, world, TS)
        np.save(os.path.join(out_dir, "gathered.npy"), img)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tiles_equal_single_rank(scene_dir, tmp_path):
    import fsamd
    import oracle_py

    world, port = 2, 29500 + os.getpid() % 1000
    mp.spawn(_rank, args=(world, port, scene_dir, str(tmp_path)), nprocs=world, join=True)
    got = np.load(os.path.join(str(tmp_path), "gathered.npy"))
    s = load_scene("c2", scene_dir)
    ref = oracle_py.Scene(s.desc_ptr()).render(s.camera(0), fsamd.render_params(W, H, SPP, tile_size=TS),
                                               threads=2)
    np.testing.assert_array_equal(got, ref.color)


def test_partition_covers_every_pixel_once():
    sys.path.insert(0, PKG)
    import tiles

    for world in (1, 2, 3, 8):
        own = tiles.owner_map(1920, 1080, world, 64)
        counts = np.bincount(own.ravel(), minlength=world)
        assert counts.sum() == 1920 * 1080
        assert counts.max() - counts.min() <= 64 * 64
