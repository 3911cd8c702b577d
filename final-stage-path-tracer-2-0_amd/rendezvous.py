"""Control plane of a one-node multi-GPU render: broadcast, barrier and max
over the ranks a launcher (torchrun) started, through files in a directory
the ranks share.

The data path (the framebuffer gather) is RCCL inside libfsgpu.so
(fs_frame_gather). This module only moves the RCCL unique id and a few
floats, and it does so without torch: a process that loads libfsgpu.so must
not load a second HIP runtime (torch's wheel bundles its own libamdhip64),
so the bench's GPU processes never import torch.

All ranks must be on one host (the directory is local). The directory name
is derived from the launcher's environment (MASTER_PORT, TORCHELASTIC_RUN_ID,
the restart count), the parent process id, which every worker of one
torchrun agent shares, and that parent's start time (a per-launch nonce: a
reused pid, or a rerun with the same port and run id, gets a fresh
directory, so no rank can read files a failed earlier launch left behind).
"""
from __future__ import annotations

import os
import shutil
import struct
import tempfile
import time


def _start_time(pid: int) -> str:
    """Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat
    field 22), or "0" where /proc is unavailable."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            stat = f.read()
        return stat[stat.rindex(")") + 2:].split()[19]
    except (OSError, ValueError, IndexError):
        return "0"


def default_dir() -> str:
    ppid = os.getppid()
    key = "_".join([os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", "none"),
                    os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"), str(ppid), _start_time(ppid)])
    return os.path.join(tempfile.gettempdir(), f"fs_rdzv_{os.getuid()}_{key}")


class FileGroup:
    """Collectives over `world` ranks through files in `path`.

    Every operation is numbered; rank r's contribution to operation k is the
    file "k.r", written atomically (write + rename). An operation completes
    for a rank when the files it waits for exist. The files of operation k
    are deleted once operation k + 1 has completed (every rank has then left
    k); close() ends with a "done" file per rank, after which rank 0 removes
    the directory. abort() (a rank that fails) leaves an "abort" file and
    removes the rank's own files, and rank 0's removes the directory; a rank
    waiting in any operation sees either and raises at once, instead of
    waiting out its timeout.
    """

    def __init__(self, rank: int, world: int, path: str | None = None, timeout: float = 900.0,
                 poll: float = 0.002):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world = rank, world
        self.path = path or default_dir()
        self.timeout, self.poll = timeout, poll
        self.seq = 0
        os.makedirs(self.path, exist_ok=True)

    # -- primitives
    def _file(self, seq: int, rank: int) -> str:
        return os.path.join(self.path, f"{seq}.{rank}")

    def _put(self, seq: int, data: bytes) -> None:
        tmp = self._file(seq, self.rank) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, self._file(seq, self.rank))

    def _wait(self, seq: int, ranks) -> dict:
        deadline = time.monotonic() + self.timeout
        out = {}
        pending = list(ranks)
        while pending:
            still = []
            for r in pending:
                try:
                    with open(self._file(seq, r), "rb") as f:
                        out[r] = f.read()
                except FileNotFoundError:
                    still.append(r)
            pending = still
            if pending:
                self._check_abort()
                if time.monotonic() > deadline:
                    raise TimeoutError(f"rendezvous {self.path}: op {seq} still waits for ranks {pending}")
                time.sleep(self.poll)
        return out

    def _check_abort(self) -> None:
        marker = os.path.join(self.path, "abort")
        if os.path.exists(marker) or not os.path.isdir(self.path):
            try:
                with open(marker) as f:
                    who = f.read().strip()
            except OSError:
                who = "0"
            raise RuntimeError(f"rendezvous {self.path}: rank {who} aborted")

    def _done(self, seq: int) -> None:
        # every rank has completed seq, hence left seq - 1: drop our file of it
        if seq > 0:
            try:
                os.remove(self._file(seq - 1, self.rank))
            except FileNotFoundError:
                pass

    def _op(self, data: bytes, wait_for) -> dict:
        seq = self.seq
        self.seq += 1
        self._put(seq, data)
        out = self._wait(seq, wait_for)
        return out

    # -- collectives
    def barrier(self) -> None:
        seq = self.seq
        self._op(b"", range(self.world))
        self._done(seq)

    def broadcast(self, data: bytes | None, root: int = 0) -> bytes:
        """root's bytes on every rank (others pass None; only the root writes
        a file)."""
        if self.rank == root and data is None:
            raise ValueError("the root must pass the data")
        seq = self.seq
        self.seq += 1
        if self.rank == root:
            self._put(seq, data)
        got = self._wait(seq, [root])
        self.barrier()  # everyone has read the root's file (the root drops it)
        return got[root]

    def max(self, value: float) -> float:
        seq = self.seq
        got = self._op(struct.pack("<d", float(value)), range(self.world))
        self._done(seq)
        return max(struct.unpack("<d", v)[0] for v in got.values())

    def allgather(self, values) -> list:
        """Every rank's list of floats (all of one length), in rank order."""
        vals = [float(v) for v in values]
        seq = self.seq
        got = self._op(struct.pack(f"<{len(vals)}d", *vals), range(self.world))
        self._done(seq)
        return [list(struct.unpack(f"<{len(got[r]) // 8}d", got[r])) for r in range(self.world)]

    def allgather_bytes(self, data: bytes) -> list:
        """Every rank's bytes, in rank order."""
        seq = self.seq
        got = self._op(bytes(data), range(self.world))
        self._done(seq)
        return [got[r] for r in range(self.world)]

    def abort(self) -> None:
        """Clean-up of a rank that fails: an "abort" marker for the others,
        then its own files go; rank 0 removes the directory."""
        try:
            tmp = os.path.join(self.path, f"abort.{self.rank}.tmp")
            with open(tmp, "w") as f:
                f.write(str(self.rank))
            os.replace(tmp, os.path.join(self.path, "abort"))
        except OSError:
            pass
        try:
            for name in os.listdir(self.path):
                if name.split(".")[1:2] == [str(self.rank)]:
                    try:
                        os.remove(os.path.join(self.path, name))
                    except FileNotFoundError:
                        pass
        except OSError:
            pass
        if self.rank == 0:
            shutil.rmtree(self.path, ignore_errors=True)

    def close(self) -> None:
        """Every rank writes its "done" file after its last read; rank 0 waits
        for all of them and removes the directory."""
        self.barrier()
        seq = self.seq
        self.seq += 1
        self._put(seq, b"done")
        if self.rank == 0:
            self._wait(seq, range(self.world))
            shutil.rmtree(self.path, ignore_errors=True)
