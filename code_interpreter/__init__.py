"""Compatibility entry points for deployments of the reference service.

``python -m code_interpreter`` and ``python -m code_interpreter.health_check``
keep working; the implementation is :mod:`bee_code_interpreter_fs_amd`.
"""
