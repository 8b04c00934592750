"""Wire-level validation primitives.

Parity: the reference declares two constrained string types
(`src/code_interpreter/utils/validation.py:19-22`):

* object id ("Hash"): ``^[0-9a-zA-Z_-]{1,255}$``
* absolute path:      ``^/[^/].*$``

The reference's path regex accepts ``..`` segments and the executor joins
user paths onto its base without checks (`executor/server.rs:83`), so a file
key such as ``/workspace/../../etc/x`` escapes the sandbox.  Here every path
that touches a filesystem goes through :func:`resolve_logical_path`, which
rejects traversal (documented divergence).
"""

from __future__ import annotations

import os
import re
from typing import Dict, Mapping, Optional, Tuple

HASH_PATTERN = r"^[0-9a-zA-Z_-]{1,255}$"
ABSOLUTE_PATH_PATTERN = r"^/[^/].*$"

_HASH_RE = re.compile(HASH_PATTERN)
_ABS_RE = re.compile(ABSOLUTE_PATH_PATTERN, re.DOTALL)

WORKSPACE_ROOT = "/workspace"
RUNTIME_PACKAGES_ROOT = "/runtime-packages"


class ValidationError(ValueError):
    """A request field failed validation; ``errors`` lists human-readable causes."""

    def __init__(self, errors):
        if isinstance(errors, str):
            errors = [errors]
        self.errors = list(errors)
        super().__init__("; ".join(self.errors))


def is_hash(value: object) -> bool:
    return isinstance(value, str) and _HASH_RE.match(value) is not None


def is_absolute_path(value: object) -> bool:
    return isinstance(value, str) and _ABS_RE.match(value) is not None


def check_hash(value: object, field: str = "hash") -> str:
    if not is_hash(value):
        raise ValidationError(f"{field}: {value!r} does not match {HASH_PATTERN}")
    return value  # type: ignore[return-value]


def check_absolute_path(value: object, field: str = "path") -> str:
    if not is_absolute_path(value):
        raise ValidationError(f"{field}: {value!r} does not match {ABSOLUTE_PATH_PATTERN}")
    return value  # type: ignore[return-value]


def check_file_map(files: Optional[Mapping[str, str]], field: str = "files") -> Dict[str, str]:
    """Validate a ``{absolute_path: object_id}`` mapping, collecting every error."""
    out: Dict[str, str] = {}
    errors = []
    for path, obj in (files or {}).items():
        if not is_absolute_path(path):
            errors.append(f"{field}: key {path!r} does not match {ABSOLUTE_PATH_PATTERN}")
            continue
        if not is_hash(obj):
            errors.append(f"{field}[{path!r}]: value {obj!r} does not match {HASH_PATTERN}")
            continue
        try:
            split_logical_path(path)
        except ValidationError as e:
            errors.extend(e.errors)
            continue
        out[path] = obj
    if errors:
        raise ValidationError(errors)
    return out


def split_logical_path(path: str) -> Tuple[str, str]:
    """Map a logical sandbox path to ``(root, relative)``.

    Paths under ``/runtime-packages/`` go to the runtime-packages root (on the
    sandbox ``PYTHONPATH``); everything else is placed in the workspace — the
    reference does the same routing (`kubernetes_code_executor.py:111-114`).
    A path such as ``/data/x.csv`` therefore lands at ``<workspace>/data/x.csv``
    (the reference's PathBuf::join would instead have written the absolute
    path verbatim, `server.rs:83`).
    """
    check_absolute_path(path)
    norm = os.path.normpath(path)
    if norm != path.rstrip("/") or "/../" in path + "/" or path.endswith("/.."):
        # normpath collapses '..' — any difference means traversal or oddities
        # like '//' or '/./'; reject them all rather than guessing intent.
        raise ValidationError(f"path {path!r} is not normalised (no '..', '.', or '//')")
    for root in (RUNTIME_PACKAGES_ROOT, WORKSPACE_ROOT):
        if norm == root:
            raise ValidationError(f"path {path!r} names a root directory, not a file")
        if norm.startswith(root + "/"):
            return root, norm[len(root) + 1 :]
    return WORKSPACE_ROOT, norm.lstrip("/")


def resolve_logical_path(path: str, workspace_dir: str, runtime_packages_dir: str) -> str:
    """Resolve a logical path onto real sandbox directories, refusing escapes."""
    root, rel = split_logical_path(path)
    base = runtime_packages_dir if root == RUNTIME_PACKAGES_ROOT else workspace_dir
    real = os.path.normpath(os.path.join(base, rel))
    if not (real == base or real.startswith(base.rstrip("/") + "/")):
        raise ValidationError(f"path {path!r} escapes the sandbox")
    return real


# Environment a request may hand its sandbox (gang jobs: RCCL / torch tuning).
# An allow-list: anything else could steer the sandbox's own bootstrap (jail,
# quota, GPU pin, loader) before user code runs.
ENV_ALLOW_PREFIXES = ("NCCL_", "RCCL_", "TORCH_", "PYTORCH_", "OMP_", "MKL_", "OPENBLAS_", "NUMEXPR_", "MIOPEN_",
                      "HIPBLASLT_", "ROCBLAS_", "TENSILE_", "USER_")
ENV_ALLOW_NAMES = frozenset({"PYTHONHASHSEED", "TZ", "LANG", "LC_ALL", "OMP_NUM_THREADS"})
_ENV_NAME = re.compile(r"^[A-Za-z_][A-Za-z0-9_]{0,127}$")


def check_env(env: Optional[Mapping[str, str]], allow_prefixes=ENV_ALLOW_PREFIXES, field: str = "env") -> Dict[str, str]:
    out: Dict[str, str] = {}
    errors = []
    for k, v in (env or {}).items():
        if not isinstance(k, str) or not _ENV_NAME.match(k):
            errors.append(f"{field}: invalid variable name {k!r}")
        elif not (k in ENV_ALLOW_NAMES or k.startswith(tuple(allow_prefixes))):
            errors.append(f"{field}: {k} is not allowed (allowed: {', '.join(allow_prefixes)} and "
                          f"{', '.join(sorted(ENV_ALLOW_NAMES))})")
        elif not isinstance(v, str) or "\0" in v or len(v) > 4096:
            errors.append(f"{field}: {k} must be a string of at most 4096 characters")
        else:
            out[k] = v
    if errors:
        raise ValidationError(errors)
    return out
