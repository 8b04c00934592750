"""``import beekern`` inside a sandbox: the MI355X kernel library
(`bee_code_interpreter_fs_amd.ops`) under a short name for user code."""
import sys as _sys

from bee_code_interpreter_fs_amd import ops as _ops

_sys.modules[__name__] = _ops
