"""Ad-hoc dependency installation for sandboxed scripts.

Reference behaviour (`executor/server.rs:174-195`): ``upm guess`` lists the
script's imports, names already provided by the image (``requirements.txt`` +
``requirements-skip.txt``, `server.rs:43-66`) are dropped, and the rest are
``pip install``-ed before the run, ignoring failures.

Here the guess is an ``ast`` import scan in the sandbox itself; a module is
"missing" when ``importlib.util.find_spec`` cannot find it.  Installs go into
the sandbox's own runtime-packages directory (already on ``sys.path``) so one
execution never changes another's environment.  The target machines have no
package index, so installs only happen from a local wheelhouse
(``APP_WHEELHOUSE`` -> ``BEE_WHEELHOUSE``); without one the scan is a no-op
and the script fails with its natural ``ModuleNotFoundError``.
"""

from __future__ import annotations

import ast
import importlib.util
import os
import subprocess
import sys
from typing import Iterable, List, Set

# import name -> distribution name, for the common mismatches
IMPORT_TO_DIST = {
    "cv2": "opencv-python",
    "PIL": "pillow",
    "sklearn": "scikit-learn",
    "yaml": "pyyaml",
    "bs4": "beautifulsoup4",
    "fitz": "pymupdf",
    "docx": "python-docx",
    "pptx": "python-pptx",
    "dateutil": "python-dateutil",
    "ffmpeg": "ffmpeg-python",
    "Crypto": "pycryptodome",
    "magic": "python-magic",
    "attr": "attrs",
    "skimage": "scikit-image",
}

# provided by the runtime image / stdlib-like names never worth installing
SKIP = {"beekern", "bee_code_interpreter_fs_amd", "__future__", "torch", "numpy", "pandas", "scipy", "matplotlib"}


def imported_modules(source: str) -> List[str]:
    try:
        tree = ast.parse(source)
    except SyntaxError:
        return []
    names: List[str] = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            names.extend(alias.name.split(".")[0] for alias in node.names)
        elif isinstance(node, ast.ImportFrom) and node.level == 0 and node.module:
            names.append(node.module.split(".")[0])
    seen: Set[str] = set()
    return [n for n in names if not (n in seen or seen.add(n))]


def missing_modules(names: Iterable[str]) -> List[str]:
    out = []
    stdlib = getattr(sys, "stdlib_module_names", frozenset())
    for name in names:
        if name in SKIP or name in stdlib or name in sys.modules:
            continue
        try:
            if importlib.util.find_spec(name) is None:
                out.append(name)
        except (ImportError, ValueError):
            out.append(name)
    return out


def install_missing(source: str, target_dir: str, wheelhouse: str = "", timeout: float = 120.0) -> List[str]:
    """Install missing imports from ``wheelhouse`` into ``target_dir``; returns
    the distributions attempted.  Failures are ignored, as in the reference."""
    wheelhouse = wheelhouse or os.environ.get("BEE_WHEELHOUSE", "")
    if not wheelhouse or not os.path.isdir(wheelhouse):
        return []  # nothing to install from: skip the parse and the path scans
    missing = missing_modules(imported_modules(source))
    if not missing:
        return []
    dists = [IMPORT_TO_DIST.get(m, m) for m in missing]
    cmd = [
        sys.executable, "-m", "pip", "install", "--no-index", "--find-links", wheelhouse,
        "--target", target_dir, "--no-cache-dir", "--quiet", "--disable-pip-version-check", *dists,
    ]
    try:
        subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout, check=False)
    except Exception:
        pass
    importlib.invalidate_caches()
    return dists
