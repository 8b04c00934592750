"""Streaming ``multipart/form-data`` parser.

The reference's ``PUT /v1/files`` takes an ``UploadFile`` (`http_server.py:
128-141`), which needs python-multipart — not installed on the target image.
This parser streams each part's body to a sink as it arrives, so uploads of
any size never sit in memory.
"""

from __future__ import annotations

import re
from typing import AsyncIterator, Awaitable, Callable, Dict, Optional

_BOUNDARY_RE = re.compile(r'boundary="?([^";]+)"?', re.IGNORECASE)
_DISPOSITION_RE = re.compile(r'(\w+)="((?:[^"\\]|\\.)*)"')


class MultipartError(ValueError):
    pass


def boundary_of(content_type: str) -> str:
    m = _BOUNDARY_RE.search(content_type or "")
    if not m:
        raise MultipartError("multipart boundary missing")
    return m.group(1)


def _parse_headers(block: bytes) -> Dict[str, str]:
    headers = {}
    for line in block.decode("latin-1").split("\r\n"):
        if ":" in line:
            k, v = line.split(":", 1)
            headers[k.strip().lower()] = v.strip()
    return headers


async def parse_multipart(
    chunks: AsyncIterator[bytes],
    boundary: str,
    on_part: Callable[[str, Optional[str], Dict[str, str]], Awaitable[Optional[Callable[[bytes], Awaitable[None]]]]],
    max_header_bytes: int = 16384,
) -> int:
    """Feed each part to ``on_part(name, filename, headers)``, which returns a
    data sink (or None to discard).  Returns the number of parts."""
    dash = b"--" + boundary.encode()
    delim = b"\r\n" + dash
    buf = b""
    it = chunks.__aiter__()

    async def more() -> bool:
        nonlocal buf
        try:
            buf += await it.__anext__()
            return True
        except StopAsyncIteration:
            return False

    # preamble up to the first boundary
    while True:
        i = buf.find(dash)
        if i >= 0:
            buf = buf[i + len(dash) :]
            break
        if len(buf) > len(dash):
            buf = buf[-len(dash) :]
        if not await more():
            raise MultipartError("no multipart boundary in body")
    parts = 0
    while True:
        while len(buf) < 2:
            if not await more():
                raise MultipartError("truncated multipart body")
        if buf.startswith(b"--"):
            return parts  # closing boundary
        if not buf.startswith(b"\r\n"):
            raise MultipartError("malformed boundary line")
        buf = buf[2:]
        while b"\r\n\r\n" not in buf:
            if len(buf) > max_header_bytes or not await more():
                raise MultipartError("malformed part headers")
        head, buf = buf.split(b"\r\n\r\n", 1)
        headers = _parse_headers(head)
        disp = dict(_DISPOSITION_RE.findall(headers.get("content-disposition", "")))
        sink = await on_part(disp.get("name", ""), disp.get("filename"), headers)
        parts += 1
        # body until the next delimiter
        while True:
            i = buf.find(delim)
            if i >= 0:
                if sink is not None and i:
                    await sink(buf[:i])
                buf = buf[i + len(delim) :]
                break
            keep = len(delim) - 1
            if len(buf) > keep:
                if sink is not None:
                    await sink(buf[:-keep])
                buf = buf[-keep:]
            if not await more():
                raise MultipartError("truncated multipart part")
