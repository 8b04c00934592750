"""File-object store: a flat directory of opaque, immutable objects.

Parity: `src/code_interpreter/services/storage.py:34-101` — objects are named
by ``secrets.token_hex(32)`` (random, not a content hash: the reference's
docstring says SHA-256 but the code draws random ids, `storage.py:36,52`),
``reader`` raises FileNotFoundError for unknown ids, ``delete`` raises it
for missing ones.

Differences (MI355X-native service):

* writes land in a temp file and are ``rename``d into place, so a reader
  never sees a half-written object;
* the store exposes :meth:`path_of` / :meth:`adopt_file` so the local GPU
  pool can hand objects to sandboxes (and take results back) with in-kernel
  copies / hard links on the same filesystem instead of streaming bytes
  through Python.
"""

from __future__ import annotations

import contextlib
import os
import secrets
import time
from typing import AsyncIterator, Optional

import anyio

from ..utils.validation import check_hash

CHUNK = 1 << 20


def new_object_id() -> str:
    return secrets.token_hex(32)


class ObjectWriter:
    """Async writer handed out by :meth:`Storage.writer`; ``hash`` is the final id."""

    def __init__(self, fh, object_id: str) -> None:
        self._fh = fh
        self.hash = object_id
        self.size = 0

    async def write(self, data: bytes) -> None:
        if not data:
            return
        if len(data) > CHUNK:  # big buffers: keep the event loop responsive
            await anyio.to_thread.run_sync(self._fh.write, data)
        else:
            self._fh.write(data)
        self.size += len(data)


class ObjectReader:
    def __init__(self, fh) -> None:
        self._fh = fh

    async def read(self, size: int = -1) -> bytes:
        if size is None or size < 0 or size > CHUNK:
            return await anyio.to_thread.run_sync(self._fh.read, size)
        return self._fh.read(size)

    async def iter_chunks(self, chunk: int = CHUNK) -> AsyncIterator[bytes]:
        while True:
            data = await self.read(chunk)
            if not data:
                return
            yield data


class Storage:
    def __init__(self, storage_path: str) -> None:
        self.storage_path = os.path.abspath(storage_path)
        os.makedirs(self.storage_path, exist_ok=True)
        # the service's alone: sandboxes (other UIDs, or jailed) never list it
        try:
            os.chmod(self.storage_path, 0o700)
        except OSError:
            pass
        self._tmp = os.path.join(self.storage_path, ".incoming")
        os.makedirs(self._tmp, exist_ok=True)

    # -- paths -------------------------------------------------------------
    def path_of(self, object_id: str) -> str:
        return os.path.join(self.storage_path, check_hash(object_id, "object id"))

    def temp_path(self) -> str:
        return os.path.join(self._tmp, secrets.token_hex(16))

    # -- write -------------------------------------------------------------
    @contextlib.asynccontextmanager
    async def writer(self) -> AsyncIterator[ObjectWriter]:
        object_id = new_object_id()
        tmp = self.temp_path()
        fh = open(tmp, "wb")
        try:
            w = ObjectWriter(fh, object_id)
            yield w
            fh.close()
            os.replace(tmp, os.path.join(self.storage_path, object_id))
        except BaseException:
            fh.close()
            with contextlib.suppress(FileNotFoundError):
                os.unlink(tmp)
            raise

    async def write(self, data: bytes) -> str:
        async with self.writer() as w:
            await w.write(data)
        return w.hash

    def adopt_file(self, src: str, link: bool = True) -> str:
        """Store an existing file as a new object (hard link if possible, else copy)."""
        object_id = new_object_id()
        dst = os.path.join(self.storage_path, object_id)
        if link:
            try:
                os.link(src, dst)
                return object_id
            except OSError:
                pass
        tmp = self.temp_path()
        _copy_file(src, tmp)
        os.replace(tmp, dst)
        return object_id

    # -- read --------------------------------------------------------------
    @contextlib.asynccontextmanager
    async def reader(self, object_id: str) -> AsyncIterator[ObjectReader]:
        try:
            path = self.path_of(object_id)
        except ValueError:
            raise FileNotFoundError(f"File not found: {object_id}")
        try:
            fh = open(path, "rb")
        except (FileNotFoundError, IsADirectoryError):
            raise FileNotFoundError(f"File not found: {object_id}")
        try:
            yield ObjectReader(fh)
        finally:
            fh.close()

    async def read(self, object_id: str) -> bytes:
        async with self.reader(object_id) as r:
            return await r.read()

    async def exists(self, object_id: str) -> bool:
        try:
            return os.path.isfile(self.path_of(object_id))
        except ValueError:
            return False

    async def size(self, object_id: str) -> Optional[int]:
        try:
            return os.path.getsize(self.path_of(object_id))
        except (ValueError, OSError):
            return None

    async def delete(self, object_id: str) -> None:
        try:
            path = self.path_of(object_id)
            os.unlink(path)
        except (ValueError, FileNotFoundError, IsADirectoryError):
            raise FileNotFoundError(f"File not found: {object_id}")

    # -- retention -----------------------------------------------------------
    def sweep(self, max_age_s: float, now: Optional[float] = None) -> int:
        """Delete objects (and abandoned temp files) stored more than
        ``max_age_s`` seconds ago; returns how many were removed.

        The reference leaves retention to operators ("clean old objects
        periodically", `README.md:61`); ``APP_FILE_STORAGE_TTL_SECONDS`` runs
        this from the service.  Age is measured from the inode change time:
        ``rename`` (written objects) and ``link`` (adopted sandbox files) both
        set it, so an adopted file's own older mtime does not count."""
        now = time.time() if now is None else now
        removed = 0
        for d in (self.storage_path, self._tmp):
            try:
                entries = list(os.scandir(d))
            except FileNotFoundError:
                continue
            for e in entries:
                try:
                    if not e.is_file(follow_symlinks=False):
                        continue
                    st = e.stat(follow_symlinks=False)
                    if now - max(st.st_ctime, st.st_mtime) > max_age_s:
                        os.unlink(e.path)
                        removed += 1
                except FileNotFoundError:
                    continue  # deleted concurrently (another replica's sweep, a DELETE)
        return removed


def _copy_file(src: str, dst: str) -> None:
    """Copy with copy_file_range (in-kernel) when available."""
    with open(src, "rb") as fi, open(dst, "wb") as fo:
        remaining = os.fstat(fi.fileno()).st_size
        if hasattr(os, "copy_file_range"):
            try:
                while remaining > 0:
                    n = os.copy_file_range(fi.fileno(), fo.fileno(), remaining)
                    if n <= 0:
                        break
                    remaining -= n
                if remaining <= 0:
                    return
            except OSError:
                fi.seek(0)
                fo.seek(0)
                fo.truncate()
        while True:
            buf = fi.read(CHUNK)
            if not buf:
                break
            fo.write(buf)
