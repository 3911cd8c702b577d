"""The bench's torch-free control plane (rendezvous.FileGroup): broadcast,
barrier, max and clean-up over world_size 2 and 4 CPU processes."""
import multiprocessing as mp
import os

import pytest


def _rank(rank, world, path, q):
    import rendezvous

    g = rendezvous.FileGroup(rank, world, path=path, timeout=60)
    uid = g.broadcast(bytes(range(128)) if rank == 0 else None, root=0)
    g.barrier()
    m = g.max(10.0 * rank + 0.5)
    uid2 = g.broadcast(b"second" if rank == world - 1 else None, root=world - 1)
    for _ in range(20):  # many small ops in a row
        g.barrier()
    m2 = g.max(-float(rank))
    g.close()
    q.put((rank, uid, m, uid2, m2))


@pytest.mark.parametrize("world", [2, 4])
def test_file_group_collectives(world, tmp_path):
    path = str(tmp_path / "rdzv")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, uid, m, uid2, m2 in got:
        assert uid == bytes(range(128))
        assert m == 10.0 * (world - 1) + 0.5
        assert uid2 == b"second"
        assert m2 == 0.0
    assert not os.path.exists(path)  # rank 0 removed the directory


def test_file_group_times_out_alone(tmp_path):
    import rendezvous

    g = rendezvous.FileGroup(0, 2, path=str(tmp_path / "r"), timeout=0.2)
    with pytest.raises(TimeoutError):
        g.barrier()
