"""Read side of an executor daemon's load table (``LoadTable`` in
csrc/executor/admission.hpp).

Every front-end replica of a node routes Executes to the node's per-GPU
executor daemons.  Admission itself -- the in-flight bound and the HBM
commitment -- is enforced by each daemon for all replicas at once
(``admission.cpp``); this table is what lets a replica *route* by the
node-wide load (admitted + waiting jobs, committed HBM, gang reservations)
rather than by the requests it happens to have sent itself.  The daemon
publishes it in a 4 KiB shared file under its private run directory; a
replica maps it read-only and reads it with the seqlock protocol (``seq`` odd
while the daemon writes, re-read on change).
"""

from __future__ import annotations

import mmap
import os
import struct
from dataclasses import dataclass
from typing import Optional

MAGIC = 0x3130444F4C454542  # "BEELOD01"
_FMT = "<QQ10q"
_SIZE = struct.calcsize(_FMT)


@dataclass
class Load:
    jobs: int
    waiting: int
    hbm_committed: int
    max_inflight: int
    hbm_capacity: int
    reserved: bool
    executions: int
    pid: int
    max_jobs_seen: int
    max_hbm_seen: int

    @property
    def depth(self) -> int:
        """Jobs this GPU holds or owes: what least-loaded routing minimises."""
        return self.jobs + self.waiting


class LoadTable:
    def __init__(self, path: str) -> None:
        self.path = path
        fd = os.open(path, os.O_RDONLY | os.O_CLOEXEC)
        try:
            self._map = mmap.mmap(fd, 4096, mmap.MAP_SHARED, mmap.PROT_READ)
        finally:
            os.close(fd)
        self._last: Optional[Load] = None

    def read(self) -> Optional[Load]:
        """The daemon's current load, or -- when every try saw a write in
        progress (a writer descheduled between its two sequence bumps, on a
        crowded host) -- the last load read.  Never "no table" for a torn
        read: routing treats a slot without a table as holding only this
        replica's requests, so a slot whose reads kept tearing drew more
        work (the 8-slot rehearsal once gave one slot 335 executions against
        ~220 for the others)."""
        for _ in range(64):
            seq0 = struct.unpack_from("<Q", self._map, 8)[0]
            if seq0 & 1:
                continue  # being written
            vals = struct.unpack_from(_FMT, self._map, 0)
            if struct.unpack_from("<Q", self._map, 8)[0] != seq0:
                continue
            if vals[0] != MAGIC:
                return None
            self._last = Load(vals[2], vals[3], vals[4], vals[5], vals[6], bool(vals[7]), vals[8], vals[9], vals[10],
                              vals[11])
            return self._last
        return self._last

    def close(self) -> None:
        try:
            self._map.close()
        except (BufferError, ValueError):
            pass


def open_table(path: Optional[str]) -> Optional[LoadTable]:
    if not path:
        return None
    try:
        return LoadTable(path)
    except (OSError, ValueError):
        return None
