"""Multi-rank path on CPU: world_size 2 over gloo. Each rank renders its
round-robin tiles (the fs_render_params tiling) with the oracle, packs them
in the product's tile exchange format (pack_tiles: 10 words = 40 B per pixel,
restated in tiles.pack_words), gathers the packs over gloo in rank order as
ncclGather delivers them, and rank 0 scatters them with unpack_tiles'
restatement; every plane (display bytes rebuilt) must equal the single-rank
render bit for bit (tiles are independent given the per-(pixel,sample)
seeds). tests/test_gpu_parity.py ties tiles.pack_words to fs_frame_pack."""
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
    planes = {k: getattr(f, k) for k in ("color", "count", "display", "normal", "depth", "material")}
    words = tiles.pack_words(planes, W, H, rank, world, TS)
    assert words.nbytes == 40 * ((tiles.tile_grid(W, H, TS)[0] * tiles.tile_grid(W, H, TS)[1] + world - 1)
                                 // world) * TS * TS
    mine = torch.from_numpy(words.view(np.int32))  # gloo carries the 32-bit words as int32
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    if rank == 0:
        gathered = np.concatenate([p.numpy().view(np.uint32) for p in parts])
        tiles.unpack_words(planes, gathered, W, H, world, 0, TS)
        np.savez(os.path.join(out_dir, "gathered.npz"), **planes)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tiles_equal_single_rank(scene_dir, tmp_path):
    import fsamd
    import oracle_py

    world, port = 2, 29500 + os.getpid() % 1000
    mp.spawn(_rank, args=(world, port, scene_dir, str(tmp_path)), nprocs=world, join=True)
    got = np.load(os.path.join(str(tmp_path), "gathered.npz"))
    s = load_scene("c2", scene_dir)
    ref = oracle_py.Scene(s.desc_ptr()).render(s.camera(0), fsamd.render_params(W, H, SPP, tile_size=TS),
                                               threads=2)
    for k in ("color", "count", "display", "normal", "depth", "material"):
        np.testing.assert_array_equal(got[k], getattr(ref, k), err_msg=k)


def test_partition_covers_every_pixel_once():
    sys.path.insert(0, PKG)
    import tiles

    for world in (1, 2, 3, 8):
        own = tiles.owner_map(1920, 1080, world, 64)
        counts = np.bincount(own.ravel(), minlength=world)
        assert counts.sum() == 1920 * 1080
        assert counts.max() - counts.min() <= 64 * 64
