"""Logging with a per-request id.

Parity: `src/code_interpreter/application_context.py:40-57` installs a filter
on the root handlers that stamps ``record.request_id`` from a ContextVar
(all-zero UUID when unset); every RPC / HTTP route sets a fresh uuid4.
"""

from __future__ import annotations

import logging
import logging.config
import uuid
from contextvars import ContextVar
from typing import Any, Dict, Optional

NULL_REQUEST_ID = "00000000-0000-0000-0000-000000000000"

request_id_var: ContextVar[Optional[str]] = ContextVar("request_id", default=None)


class RequestIdFilter(logging.Filter):
    def __init__(self, var: ContextVar = request_id_var) -> None:
        super().__init__()
        self._var = var

    def filter(self, record: logging.LogRecord) -> bool:
        record.request_id = self._var.get() or NULL_REQUEST_ID
        return True


def setup_logging(config: Dict[str, Any], var: ContextVar = request_id_var) -> None:
    logging.config.dictConfig(config)
    for handler in logging.root.handlers:
        if not any(isinstance(f, RequestIdFilter) for f in handler.filters):
            handler.addFilter(RequestIdFilter(var))


def new_request_id(var: ContextVar = request_id_var) -> str:
    rid = str(uuid.uuid4())
    var.set(rid)
    return rid
