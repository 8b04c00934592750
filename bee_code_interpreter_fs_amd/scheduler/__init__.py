"""Execution backends: local GPU-pinned pools (native executor per MI355X),
Kubernetes executor pods, and an in-process fake for tests."""
from .backend import CodeExecutor, ExecuteRequest, ExecutionResult  # noqa: F401
