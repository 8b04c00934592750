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

# import name -> distribution name where they differ.  The reference resolves
# imports with upm's pypi_map.sqlite (executor/Dockerfile:30-37,122-124); this
# table covers the mismatches that code written by LLMs actually hits.
IMPORT_TO_DIST = {
    "cv2": "opencv-python-headless", "PIL": "pillow", "sklearn": "scikit-learn", "skimage": "scikit-image",
    "yaml": "pyyaml", "bs4": "beautifulsoup4", "fitz": "pymupdf", "docx": "python-docx", "pptx": "python-pptx",
    "dateutil": "python-dateutil", "ffmpeg": "ffmpeg-python", "Crypto": "pycryptodome", "Cryptodome": "pycryptodomex",
    "magic": "python-magic", "attr": "attrs", "dotenv": "python-dotenv", "jwt": "pyjwt", "serial": "pyserial",
    "usb": "pyusb", "OpenSSL": "pyopenssl", "git": "gitpython", "github": "pygithub", "telegram": "python-telegram-bot",
    "discord": "discord.py", "slugify": "python-slugify", "Levenshtein": "python-levenshtein", "pylab": "matplotlib",
    "mpl_toolkits": "matplotlib", "google": "protobuf", "grpc": "grpcio", "zmq": "pyzmq", "nacl": "pynacl",
    "jose": "python-jose", "multipart": "python-multipart", "socks": "pysocks", "wx": "wxpython", "gi": "pygobject",
    "sqlalchemy": "sqlalchemy", "psycopg2": "psycopg2-binary", "MySQLdb": "mysqlclient", "pymysql": "pymysql",
    "ldap": "python-ldap", "Image": "pillow", "pdfminer": "pdfminer.six",
    "pdfplumber": "pdfplumber", "PyPDF2": "PyPDF2", "pypdf": "pypdf", "reportlab": "reportlab",
    "openpyxl": "openpyxl", "xlrd": "xlrd", "xlsxwriter": "xlsxwriter", "odf": "odfpy", "tabulate": "tabulate",
    "markdown": "markdown", "mistune": "mistune", "lxml": "lxml", "html5lib": "html5lib", "pyquery": "pyquery",
    "nltk": "nltk", "spacy": "spacy", "gensim": "gensim", "textblob": "textblob", "wordcloud": "wordcloud",
    "networkx": "networkx", "igraph": "python-igraph", "graphviz": "graphviz", "pydot": "pydot", "shapely": "shapely",
    "geopandas": "geopandas", "pyproj": "pyproj", "folium": "folium", "plotly": "plotly", "bokeh": "bokeh",
    "seaborn": "seaborn", "altair": "altair", "statsmodels": "statsmodels", "sympy": "sympy", "xarray": "xarray",
    "netCDF4": "netcdf4", "h5py": "h5py", "tables": "tables", "pyarrow": "pyarrow", "polars": "polars",
    "duckdb": "duckdb", "numba": "numba", "llvmlite": "llvmlite", "cython": "cython", "Cython": "cython",
    "xgboost": "xgboost", "lightgbm": "lightgbm", "catboost": "catboost", "tensorflow": "tensorflow",
    "keras": "keras", "transformers": "transformers", "tokenizers": "tokenizers", "datasets": "datasets",
    "sentencepiece": "sentencepiece", "tiktoken": "tiktoken", "imageio": "imageio", "moviepy": "moviepy",
    "pydub": "pydub", "librosa": "librosa", "soundfile": "soundfile", "sounddevice": "sounddevice",
    "qrcode": "qrcode", "barcode": "python-barcode", "pyzbar": "pyzbar", "pytesseract": "pytesseract",
    "pdf2image": "pdf2image", "pikepdf": "pikepdf", "weasyprint": "weasyprint", "pypandoc": "pypandoc",
    "yt_dlp": "yt-dlp", "youtube_dl": "youtube-dl", "emoji": "emoji", "faker": "faker", "requests": "requests",
    "httpx": "httpx", "aiohttp": "aiohttp", "websocket": "websocket-client", "websockets": "websockets",
    "toml": "toml", "tomli": "tomli", "ujson": "ujson", "orjson": "orjson", "simplejson": "simplejson",
    "jsonschema": "jsonschema", "pydantic": "pydantic", "tqdm": "tqdm", "rich": "rich", "colorama": "colorama",
    "termcolor": "termcolor", "click": "click", "typer": "typer", "jinja2": "jinja2", "cowsay": "cowsay",
    "pytz": "pytz", "tzdata": "tzdata", "arrow": "arrow", "pendulum": "pendulum", "babel": "babel",
    "unidecode": "unidecode", "chardet": "chardet", "cchardet": "cchardet", "regex": "regex",
}

# distributions the image provides (the reference's requirements.txt:1-4 and
# requirements-skip.txt:1-24, mapped onto this image) -- never installed ad
# hoc, so a guess can not shadow the image's build of them
PREINSTALLED = {
    # OS-packaged in the reference image
    "ffmpeg-python", "jinja2", "matplotlib", "moviepy", "numpy", "opencv-python", "opencv-python-headless",
    "pandas", "pdf2image", "pikepdf", "pillow", "pypandoc", "scipy", "sympy", "tabulate", "xarray", "xonsh",
    # installed manually there
    "pymupdf",
    # requirements.txt
    "PyPDF2", "pydantic", "pydantic_core",
    # this image
    "torch", "beekern", "bee_code_interpreter_fs_amd",
}

# import names never worth a lookup
SKIP = {"beekern", "bee_code_interpreter_fs_amd", "__future__", "torch", "numpy", "pandas", "scipy", "matplotlib"}


def distribution_for(module: str) -> str:
    return IMPORT_TO_DIST.get(module, module)


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
    dists = [d for d in (distribution_for(m) for m in missing) if d not in PREINSTALLED]
    if not dists:
        return []
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
