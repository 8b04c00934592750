"""Minimal keep-alive HTTP/1.1 client over a Unix socket, for the hot
service -> executor hop.

httpx costs ~0.3-0.5 ms of Python per request; this is a plain asyncio
stream pool that writes one request and reads a Content-Length response
(the executor daemon never chunks its responses).
"""

from __future__ import annotations

import asyncio
import json
from typing import List, Optional, Tuple


class UdsHttpError(ConnectionError):
    pass


class Response:
    __slots__ = ("status_code", "content")

    def __init__(self, status_code: int, content: bytes) -> None:
        self.status_code = status_code
        self.content = content

    @property
    def text(self) -> str:
        return self.content.decode(errors="replace")

    def json(self):
        return json.loads(self.content)


class UdsHttpClient:
    def __init__(self, path: str, max_idle: int = 64) -> None:
        self.path = path
        self.max_idle = max_idle
        self._idle: List[Tuple[asyncio.StreamReader, asyncio.StreamWriter]] = []

    async def _conn(self):
        while self._idle:
            r, w = self._idle.pop()
            if not w.is_closing() and not r.at_eof():
                return r, w
            w.close()
        return await asyncio.open_unix_connection(self.path, limit=1 << 22)

    def _release(self, r, w) -> None:
        if len(self._idle) < self.max_idle and not w.is_closing():
            self._idle.append((r, w))
        else:
            w.close()

    async def request(self, method: str, path: str, body: Optional[bytes] = None, timeout: Optional[float] = None) -> Response:
        return await asyncio.wait_for(self._request(method, path, body), timeout) if timeout else await self._request(method, path, body)

    async def _request(self, method: str, path: str, body: Optional[bytes]) -> Response:
        body = body or b""
        head = (
            f"{method} {path} HTTP/1.1\r\nHost: executor\r\nContent-Type: application/json\r\n"
            f"Content-Length: {len(body)}\r\n\r\n"
        ).encode()
        for attempt in (0, 1):
            r, w = await self._conn()
            try:
                w.write(head + body)
                await w.drain()
                status_line = await r.readline()
                if not status_line:
                    raise UdsHttpError("executor closed the connection")
                status = int(status_line.split(b" ", 2)[1])
                length = 0
                keep = True
                while True:
                    line = await r.readline()
                    if line in (b"\r\n", b"\n", b""):
                        break
                    k, _, v = line.partition(b":")
                    k = k.strip().lower()
                    if k == b"content-length":
                        length = int(v.strip())
                    elif k == b"connection" and v.strip().lower() == b"close":
                        keep = False
                content = await r.readexactly(length) if length else b""
            except (ConnectionError, asyncio.IncompleteReadError, OSError, ValueError, IndexError) as e:
                w.close()
                if attempt == 0 and not isinstance(e, asyncio.IncompleteReadError):
                    continue  # stale pooled connection: retry once on a fresh one
                raise UdsHttpError(str(e)) from e
            except BaseException:
                w.close()  # cancelled mid-request: the connection state is unknown
                raise
            if keep:
                self._release(r, w)
            else:
                w.close()
            return Response(status, content)
        raise UdsHttpError("unreachable")

    async def post_json(self, path: str, obj, timeout: Optional[float] = None) -> Response:
        return await self.request("POST", path, json.dumps(obj).encode(), timeout)

    async def get_json(self, path: str, timeout: Optional[float] = 10.0):
        resp = await self.request("GET", path, None, timeout)
        if resp.status_code != 200:
            raise UdsHttpError(f"GET {path}: {resp.status_code} {resp.text[:200]}")
        return resp.json()

    async def aclose(self) -> None:
        for _, w in self._idle:
            w.close()
        self._idle.clear()
