"""Async retry with exponential backoff.

Parity: the reference wraps `execute` and `spawn_executor_pod` in tenacity
``@retry(retry_if_exception_type(RuntimeError), stop_after_attempt(3),
wait_exponential(multiplier=1, min=4, max=10))``
(`kubernetes_code_executor.py:76-80,203-207`).  tenacity is not on the target
image; this is the same policy as a small decorator with knobs for tests.
"""

from __future__ import annotations

import asyncio
import functools
import logging
from typing import Awaitable, Callable, Tuple, Type, TypeVar

T = TypeVar("T")
logger = logging.getLogger("retry")


def backoff_delays(attempts: int, multiplier: float = 1.0, minimum: float = 4.0, maximum: float = 10.0):
    """Delays between attempts: ``clamp(multiplier * 2**i, minimum, maximum)``."""
    return [min(max(multiplier * (2**i), minimum), maximum) for i in range(max(attempts - 1, 0))]


def async_retry(
    retry_on: Tuple[Type[BaseException], ...] = (RuntimeError,),
    attempts: int = 3,
    multiplier: float = 1.0,
    minimum: float = 4.0,
    maximum: float = 10.0,
    sleep: Callable[[float], Awaitable[None]] = asyncio.sleep,
):
    delays = backoff_delays(attempts, multiplier, minimum, maximum)

    def decorate(fn: Callable[..., Awaitable[T]]) -> Callable[..., Awaitable[T]]:
        @functools.wraps(fn)
        async def wrapper(*args, **kwargs) -> T:
            for i in range(attempts):
                try:
                    return await fn(*args, **kwargs)
                except retry_on as e:
                    if i == attempts - 1:
                        raise
                    logger.warning("%s failed (%s), retry %d/%d in %.1fs", fn.__name__, e, i + 1, attempts - 1, delays[i])
                    await sleep(delays[i])
            raise AssertionError("unreachable")

        return wrapper

    return decorate
