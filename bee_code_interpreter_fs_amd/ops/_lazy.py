"""numpy on first use.

beekern must import without numpy: scripts that use only beekern and the
standard library run in sandboxes forked from a zygote that never loaded
numpy (runtime/zygote.py, executor kind "nano"), and numpy's ~90 mappings and
~7 MB of private memory are then neither copied at each fork nor torn down at
each exit.  The array code keeps writing ``np.<name>``; the first such access
imports numpy.  Reductions hand back ``numpy.float64`` when numpy is loaded
(as before) and a Python ``float`` -- same value, same ``str`` -- otherwise.
"""

from __future__ import annotations

import sys


class _LazyNumpy:
    __slots__ = ()

    def __getattr__(self, name: str):
        import numpy

        return getattr(numpy, name)

    def __repr__(self) -> str:
        return "<numpy, imported on first use>"


np = _LazyNumpy()


def numpy_loaded():
    """The numpy module if something in this process imported it, else None."""
    return sys.modules.get("numpy")


def scalar(v: float):
    """A reduction's result: numpy.float64 when numpy is loaded, else float."""
    m = sys.modules.get("numpy")
    return m.float64(v) if m is not None else v


def is_number(x) -> bool:
    """int / float, or a numpy scalar (only possible once numpy is loaded)."""
    if isinstance(x, (int, float)):
        return True
    m = sys.modules.get("numpy")
    return m is not None and isinstance(x, (m.floating, m.integer))


def is_integer(x) -> bool:
    if isinstance(x, int):
        return True
    m = sys.modules.get("numpy")
    return m is not None and isinstance(x, m.integer)
