"""xonsh-style shell lines in Python payloads.

The reference renames every payload to ``.xsh`` and runs it with ``xonsh``
(`executor/server.rs:197-206`), so a payload may mix Python with shell
commands.  Sandboxes here run Python directly (a zygote-forked interpreter;
starting xonsh costs ~80 ms, the reference's own TODO at `server.rs:204`),
and this module lowers the xonsh subset that code-interpreter payloads use
to ordinary Python before the script is compiled:

* **subprocess-mode lines** -- a statement line whose first word is not
  Python (``ls -la``, ``pip install x``, ``echo $HOME | wc -c``,
  ``./run.sh``, ``cd /tmp``) runs as a shell command line.  As in xonsh, a
  line that parses as Python is still a command when its leading name is
  not bound anywhere in the script and is not a builtin (``ls -l`` is
  ``ls - l`` to Python);
* **Python-mode operators** -- ``$NAME`` / ``${expr}`` (environment
  variables, assignable), ``$(cmd)`` (captured stdout, a str), ``!(cmd)``
  (a captured :class:`CommandResult`), ``$[cmd]`` (run, output not
  captured, ``None``) and ``![cmd]`` (run uncaptured, a result object);
* inside a command, ``@(expr)`` interpolates a Python value (lists become
  several arguments) and ``@$(cmd)`` splices a command's output as words;
* literals: path strings ``p"dir/f"`` / ``pf"{d}/f"`` (``pathlib.Path``)
  and glob literals ``g`*.csv``` (the sorted list of matching paths).

Command lines run under ``bash -c`` with the script's environment, so pipes,
redirections, globs, ``&&``/``||`` and ``$VAR`` expansion behave as a shell's
do; ``cd`` (alone on its line) changes the script's own working directory
and ``exit [n]`` ends the script, as xonsh's aliases do.  A failing command
does not stop the script (xonsh's default ``$RAISE_SUBPROC_ERROR = False``).

Plain Python pays ~10-35 us (40 lines - 1.6 KB): :func:`maybe_shell` is a
line regex pass plus a walk over the quote characters, and only a payload
it flags is analysed; a payload with no shell construct compiles
from its original text, so its SyntaxErrors read exactly as Python's.
Line numbers are preserved by the lowering (tracebacks point at the user's
lines).
"""

from __future__ import annotations

import ast
import builtins
import keyword
import os
import re
import shlex
import subprocess
import sys
from collections.abc import MutableMapping
from typing import List, Optional, Tuple

RUNTIME_NAME = "__bee_xsh__"

# a line that starts like a command: a path, or a non-keyword word followed
# by nothing or by something other than an operator.  The pattern starts with
# a literal newline, so the engine skips from line start to line start.
_LINE = re.compile(
    r"\n[ \t]*(?:[/~]|\.[/.A-Za-z_]|([A-Za-z_][A-Za-z0-9_]*)"
    r"(?:[ \t]*(?:#[^\n]*)?(?=\n)|[ \t]+[^ \t\n=#(\[.,:;+*/%&|^<>!\-]|[ \t]+-[A-Za-z\-]))"
)
_SOFT = {"match", "case", "_", "type"}


def maybe_shell(source: str) -> bool:
    """Cheap screen (~15 us for a 40-line payload, ~35 us for the 1.6 KB
    headline payload on the build host): False means the payload certainly
    has no xonsh construct."""
    if "$" in source or "!(" in source or "![" in source or _has_xsh_literal(source):
        return True
    for m in _LINE.finditer("\n" + source + "\n"):
        head = m.group(1)
        if head is None or not keyword.iskeyword(head):
            return True
    return False


# ---------------------------------------------------------------- scanning

# string prefixes, xonsh's path strings (p, pr, rp, pf, fp) included
_STR_PREFIX = re.compile(r"(?i)(?:rb|br|fr|rf|pr|rp|pf|fp|r|b|f|u|p)?(?:'''|\"\"\"|'|\")")
# a path string (p"..."), or a glob literal (g`...`): not Python, so only a
# payload with one of them (or another xonsh construct) is ever lowered
_XSH_LITERAL = re.compile(r"(?<![\w.'\"])(?:[pP][rRfF]?|[rRfF][pP])['\"]|(?<![\w.])g`")
_QUOTE = re.compile(r"['\"`]")
_P_FORMS = frozenset(("p", "pr", "pf", "rp", "fp"))


def _word_char(c: str) -> bool:
    return c.isalnum() or c == "_"


def _has_xsh_literal(src: str) -> bool:
    """``_XSH_LITERAL.search(src) is not None``, by visiting only the quote
    characters: the regex's leading lookbehind runs at every position (~160
    us on a 1.6 KB payload, every Execute without a precompiled payload);
    this is ~15 us."""
    for m in _QUOTE.finditer(src):
        i = m.start()
        if src[i] == "`":
            if i >= 1 and src[i - 1] == "g" and (i < 2 or not (_word_char(src[i - 2]) or src[i - 2] == ".")):
                return True
            continue
        j = i
        while j > 0 and i - j < 2 and src[j - 1] in "pPrRfF":
            j -= 1
        # the longest prefix first, then the one-letter one (as the regex's alternation does)
        for k in range(j, i):
            pre = src[k:i].lower()
            if pre in _P_FORMS and (k == 0 or not (_word_char(src[k - 1]) or src[k - 1] in ".'\"")):
                return True
    return False
_OPENERS = {"(": ")", "[": "]", "{": "}"}


def _skip_string(src: str, i: int) -> int:
    """i at a string prefix/quote; returns the index after the literal (or
    the end of the line for an unterminated one-quote string)."""
    m = _STR_PREFIX.match(src, i)
    assert m is not None
    q = m.group(0).lstrip("rRbBfFuUpP")
    j = m.end()
    n = len(src)
    while j < n:
        c = src[j]
        if c == "\\":
            j += 2
            continue
        if len(q) == 1 and c == "\n":
            return j
        if src.startswith(q, j):
            return j + len(q)
        j += 1
    return n


def _string_start(src: str, i: int) -> bool:
    c = src[i]
    if c in "'\"":
        return True
    if c.isalpha() and (i == 0 or not (src[i - 1].isalnum() or src[i - 1] == "_")):
        m = _STR_PREFIX.match(src, i)
        return m is not None
    return False


def _match_close(src: str, i: int) -> int:
    """i at an opening bracket; index of its matching closer (quotes
    respected), or -1."""
    stack = [_OPENERS[src[i]]]
    j = i + 1
    n = len(src)
    while j < n:
        c = src[j]
        if c in "'\"":
            j = _skip_string(src, j)
            continue
        if c == "\\":
            j += 2
            continue
        if c in _OPENERS:
            stack.append(_OPENERS[c])
        elif c in ")]}":
            if c != stack[-1]:
                return -1
            stack.pop()
            if not stack:
                return j
        j += 1
    return -1


def _logical_lines(src: str) -> List[Tuple[int, int]]:
    """(start, end) offsets of each logical line (end excludes the newline):
    newlines inside brackets, strings or after a backslash do not end one.
    ``$(``/``$[``/``!(``/``![`` open brackets like any other."""
    out = []
    start = 0
    depth = 0
    i = 0
    n = len(src)
    while i < n:
        c = src[i]
        if c == "#":
            while i < n and src[i] != "\n":
                i += 1
            continue
        if _string_start(src, i):
            i = _skip_string(src, i)
            continue
        if c == "\\" and i + 1 < n and src[i + 1] == "\n":
            i += 2
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth = max(0, depth - 1)
        elif c == "\n" and depth == 0:
            out.append((start, i))
            start = i + 1
        i += 1
    if start < n:
        out.append((start, n))
    return out


# ------------------------------------------------------- operator lowering

def _lower_ops(text: str) -> str:
    """Python-mode xonsh operators -> calls on the runtime object.  Newlines
    a lowered construct spanned are kept inside its call's parentheses."""
    out = []
    i = 0
    n = len(text)
    while i < n:
        c = text[i]
        if c == "#":
            j = text.find("\n", i)
            j = n if j < 0 else j
            out.append(text[i:j])
            i = j
            continue
        if _string_start(text, i):
            j = _skip_string(text, i)
            lit = text[i:j]
            prefix = _STR_PREFIX.match(text, i).group(0).rstrip("'\"")
            if "p" in prefix.lower():
                # xonsh path string: p"~/x" is pathlib.Path("~/x") (an f-string
                # path formats first: pf"{d}/x")
                rest = prefix.replace("p", "").replace("P", "") + lit[len(prefix):]
                lit = f'__import__("pathlib").Path({rest})'
            out.append(lit)
            i = j
            continue
        if text.startswith("g`", i) and (i == 0 or not (text[i - 1].isalnum() or text[i - 1] in "_.")):
            j = text.find("`", i + 2)
            if j > 0 and "\n" not in text[i + 2:j]:
                # xonsh glob literal: g`*.py` is the sorted list of matching paths
                out.append(f"sorted(__import__('glob').glob({text[i + 2:j]!r}, recursive=True))")
                i = j + 1
                continue
        two = text[i:i + 2]
        if two in ("$(", "$[", "!(", "![", "${"):
            j = _match_close(text, i + 1)
            if j < 0:
                out.append(c)
                i += 1
                continue
            inner = text[i + 2:j]
            pad = "\n" * inner.count("\n")
            if two == "${":
                out.append(f"{RUNTIME_NAME}.env[{_lower_ops(inner)}]")
            else:
                fn = {"$(": "out", "$[": "run", "!(": "pipe", "![": "run_obj"}[two]
                out.append(f"{RUNTIME_NAME}.{fn}({inner.strip()!r}{pad})")
            i = j + 1
            continue
        if c == "$":
            m = re.match(r"[A-Za-z_][A-Za-z0-9_]*", text[i + 1:])
            if m:
                out.append(f"{RUNTIME_NAME}.env[{m.group(0)!r}]")
                i += 1 + m.end()
                continue
        out.append(c)
        i += 1
    return "".join(out)


def _has_ops(text: str) -> bool:
    return _lower_ops(text) != text


# ----------------------------------------------------- line classification

_HEAD = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")


def _leftmost_name(node: ast.AST) -> Optional[str]:
    """`ls -la` -> 'ls' (BinOp/UnaryOp/Compare chains down their left
    operand); anything that is not such a chain -> None."""
    while True:
        if isinstance(node, ast.Name):
            return node.id
        if isinstance(node, ast.BinOp):
            node = node.left
        elif isinstance(node, ast.Compare):
            node = node.left
        elif isinstance(node, ast.BoolOp):
            node = node.values[0]
        else:
            return None


def _bound_names(tree: ast.AST) -> set:
    names = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name) and isinstance(node.ctx, (ast.Store, ast.Del)):
            names.add(node.id)
        elif isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            names.add(node.name)
        elif isinstance(node, ast.alias):
            names.add((node.asname or node.name).split(".")[0])
        elif isinstance(node, ast.arg):
            names.add(node.arg)
        elif isinstance(node, (ast.Global, ast.Nonlocal)):
            names.update(node.names)
        elif isinstance(node, ast.ExceptHandler) and node.name:
            names.add(node.name)
        elif isinstance(node, (ast.MatchAs, ast.MatchStar)) and node.name:
            names.add(node.name)
        elif isinstance(node, ast.MatchMapping) and node.rest:
            names.add(node.rest)
    return names


_PY_NAMES = set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__builtins__", "__spec__", "__loader__",
                                  "__package__", "__cached__", "__annotations__"}

# kinds of logical line
_PY, _SHELL, _MAYBE = 0, 1, 2


def _classify(text: str) -> Tuple[int, Optional[str]]:
    """(_PY | _SHELL | _MAYBE, leading name) of one dedented logical line."""
    body = text.strip()
    if not body or body.startswith("#"):
        return _PY, None
    if body.startswith("..."):
        return _PY, None
    if body[0] in "/~" or (body[0] == "." and len(body) > 1 and body[1] in "/."):
        return _SHELL, None
    m = _HEAD.match(body)
    if m is None:
        return _PY, None
    head = m.group(0)
    if keyword.iskeyword(head):
        return _PY, None
    rest = body[m.end():]
    if rest[:1] in ("(", "[", "=", ",", ":") or re.match(r"\.[A-Za-z_]", rest):
        return _PY, None
    lowered = _lower_ops(body)
    try:
        mod = ast.parse(lowered)
    except SyntaxError:
        code_part = body.split("#", 1)[0].rstrip()
        if code_part.endswith(":") and head in _SOFT:
            return _PY, None
        return _SHELL, head
    if len(mod.body) == 1 and isinstance(mod.body[0], ast.Expr):
        name = _leftmost_name(mod.body[0].value)
        if name is not None and name == head:
            return _MAYBE, head
    return _PY, None


def translate(source: str) -> Optional[str]:
    """The payload with its xonsh constructs lowered to Python, or None when
    it has none (run the original text)."""
    lines = _logical_lines(source)
    kinds = []
    for start, end in lines:
        text = source[start:end]
        kinds.append(_classify(text))
    if not any(k != _PY for k, _ in kinds) and not _has_ops(source):
        return None

    def assemble(shell_of) -> str:
        parts = []
        prev = 0
        for idx, (start, end) in enumerate(lines):
            parts.append(source[prev:start])
            text = source[start:end]
            if shell_of(idx):
                indent = text[: len(text) - len(text.lstrip(" \t"))]
                cmd = text.strip()
                parts.append(f"{indent}{RUNTIME_NAME}.run({cmd!r})" + "\n" * text.count("\n"))
            else:
                parts.append(_lower_ops(text))
            prev = end
        parts.append(source[prev:])
        return "".join(parts)

    # bindings of the script with every candidate line taken as a command
    draft = assemble(lambda i: kinds[i][0] != _PY)
    star_import = False
    try:
        tree = ast.parse(draft)
        bound = _bound_names(tree)
        # `from m import *` binds names no scan can see: a bare-name line
        # stays Python then
        star_import = any(isinstance(n, ast.alias) and n.name == "*" for n in ast.walk(tree))
    except SyntaxError:
        bound = set()

    def is_shell(i: int) -> bool:
        kind, head = kinds[i]
        if kind == _SHELL:
            # a line that is not Python but starts with a name the script
            # binds (or a builtin, `print "x"`) stays Python: its
            # SyntaxError is the useful report
            if head in ("exit", "quit") and head not in bound:
                return True  # xonsh's `exit 3` alias
            return head is None or not (head in bound or head in _PY_NAMES)
        if kind == _MAYBE:
            return not star_import and head not in bound and head not in _PY_NAMES
        return False

    if not any(is_shell(i) for i in range(len(lines))) and not _has_ops(source):
        return None
    return assemble(is_shell)


def _valid_python_needs_lowering(source: str) -> bool:
    """The screen passed (a `$` in a string, a docstring line that reads like
    a command, ...): one parse of the whole payload settles most cases.  A
    payload that is valid Python has no xonsh operator outside its strings
    (`$`, `!(`, `![` are syntax errors there), so only a bare-name
    expression statement (`pwd`, `ls -la`) whose leading name the script
    never binds can still be a command; the per-line analysis runs only
    then, or when the payload is not Python at all."""
    try:
        tree = ast.parse(source)
    except (SyntaxError, ValueError, RecursionError, MemoryError):
        return True
    candidates = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Expr):
            name = _leftmost_name(node.value)
            if name is not None and name not in _PY_NAMES:
                candidates.append(name)
        elif isinstance(node, ast.alias) and node.name == "*":
            return False  # names no scan can see: bare names stay Python
    if not candidates:
        return False
    bound = _bound_names(tree)
    return any(n not in bound for n in candidates)


def lower_payload(source: str) -> Optional[str]:
    """The payload's lowering, or None when it is plain Python (or its
    lowering would not compile either: the original text's SyntaxError is
    then the report)."""
    if not maybe_shell(source):
        return None
    if not _valid_python_needs_lowering(source):
        return None
    try:
        lowered = translate(source)
    except (RecursionError, ValueError):
        return None
    if lowered is None:
        return None
    try:
        ast.parse(lowered)
    except SyntaxError:
        return None
    return lowered


# ------------------------------------------------------------------ runtime

class CommandResult:
    """What ``!(cmd)`` / ``![cmd]`` return (xonsh's CommandPipeline subset):
    ``.out`` / ``.err`` (None when not captured), ``.returncode`` (``.rtn``),
    truthy when the command succeeded, ``str()`` = stdout, iterable over
    stdout lines."""

    __slots__ = ("args", "out", "err", "returncode")

    def __init__(self, args: str, out: Optional[str], err: Optional[str], returncode: int) -> None:
        self.args, self.out, self.err, self.returncode = args, out, err, returncode

    @property
    def rtn(self) -> int:
        return self.returncode

    @property
    def output(self) -> Optional[str]:
        return self.out

    @property
    def lines(self) -> List[str]:
        return (self.out or "").splitlines(keepends=True)

    def __bool__(self) -> bool:
        return self.returncode == 0

    def __str__(self) -> str:
        return self.out or ""

    def __iter__(self):
        return iter(self.lines)

    def __repr__(self) -> str:
        return f"CommandResult(args={self.args!r}, returncode={self.returncode})"


class _Env(MutableMapping):
    """``$NAME``: the script's environment (os.environ); values are str."""

    def __getitem__(self, key):
        return os.environ[key]

    def __setitem__(self, key, value):
        if isinstance(value, (list, tuple)):
            value = os.pathsep.join(str(v) for v in value)
        os.environ[key] = str(value)

    def __delitem__(self, key):
        del os.environ[key]

    def __iter__(self):
        return iter(os.environ)

    def __len__(self):
        return len(os.environ)

    def __repr__(self):
        return f"Env({dict(os.environ)!r})"


class Runtime:
    """The object lowered payloads call (bound as ``__bee_xsh__``)."""

    def __init__(self) -> None:
        self.env = _Env()
        self.last_returncode = 0
        self.shell = "/bin/bash" if os.path.exists("/bin/bash") else "/bin/sh"

    # -- expansion of @(...) / @$(...) in the caller's scope
    def _expand(self, cmd: str, frame) -> str:
        if "@" not in cmd:
            return cmd
        out = []
        i = 0
        n = len(cmd)
        while i < n:
            if cmd.startswith("@(", i) or cmd.startswith("@$(", i):
                sub = cmd.startswith("@$(", i)
                open_at = i + (2 if sub else 1)
                j = _match_close(cmd, open_at)
                if j > 0:
                    inner = cmd[open_at + 1:j]
                    if sub:
                        words = self._capture(self._expand(inner, frame))[0].split()
                    else:
                        val = eval(inner, frame.f_globals, frame.f_locals)  # noqa: S307 - the user's own expression
                        words = [str(v) for v in val] if isinstance(val, (list, tuple)) else [str(val)]
                    out.append(" ".join(shlex.quote(w) for w in words))
                    i = j + 1
                    continue
            if cmd[i] in "'\"":
                j = _skip_string(cmd, i)
                out.append(cmd[i:j])
                i = j
                continue
            out.append(cmd[i])
            i += 1
        return "".join(out)

    @staticmethod
    def _flush() -> None:
        for stream in (sys.stdout, sys.stderr):
            try:
                stream.flush()
            except Exception:
                pass

    def _builtin(self, cmd: str) -> Optional[int]:
        """xonsh's `cd` / `exit` aliases when they are the whole line."""
        try:
            words = shlex.split(cmd)
        except ValueError:
            return None
        if not words or any(w in ("|", "&&", "||", ";", ">", "<", "&") for w in words):
            return None
        if words[0] == "cd" and len(words) <= 2:
            target = words[1] if len(words) == 2 else os.environ.get("HOME", "/")
            if target == "-":
                target = os.environ.get("OLDPWD", os.getcwd())
            target = os.path.expanduser(os.path.expandvars(target))
            old = os.getcwd()
            try:
                os.chdir(target)
            except OSError as e:
                self._flush()
                sys.stderr.write(f"cd: {e.strerror}: {target}\n")
                return 1
            os.environ["OLDPWD"] = old
            os.environ["PWD"] = os.getcwd()
            return 0
        if words[0] == "exit" and len(words) <= 2:
            raise SystemExit(int(words[1]) if len(words) == 2 and words[1].lstrip("-").isdigit() else 0)
        return None

    def _spawn(self, cmd: str, capture_out: bool, capture_err: bool):
        self._flush()
        r = subprocess.run(
            [self.shell, "-c", cmd],
            stdout=subprocess.PIPE if capture_out else None,
            stderr=subprocess.PIPE if capture_err else None,
        )
        self.last_returncode = r.returncode
        dec = lambda b: b.decode("utf-8", errors="replace") if b is not None else None  # noqa: E731
        return dec(r.stdout), dec(r.stderr), r.returncode

    def _capture(self, cmd: str):
        return self._spawn(cmd, True, False)

    # -- the lowered forms
    def run(self, cmd: str) -> None:
        """A subprocess-mode line / ``$[cmd]``: output goes where the
        script's goes."""
        cmd = self._expand(cmd, sys._getframe(1))
        rc = self._builtin(cmd)
        if rc is None:
            self._spawn(cmd, False, False)
        else:
            self.last_returncode = rc
        return None

    def run_obj(self, cmd: str) -> CommandResult:
        cmd = self._expand(cmd, sys._getframe(1))
        rc = self._builtin(cmd)
        if rc is None:
            _, _, rc = self._spawn(cmd, False, False)
        self.last_returncode = rc
        return CommandResult(cmd, None, None, rc)

    def out(self, cmd: str) -> str:
        """``$(cmd)``: the command's stdout."""
        return self._capture(self._expand(cmd, sys._getframe(1)))[0]

    def pipe(self, cmd: str) -> CommandResult:
        """``!(cmd)``: stdout, stderr and status, all captured."""
        cmd = self._expand(cmd, sys._getframe(1))
        out, err, rc = self._spawn(cmd, True, True)
        return CommandResult(cmd, out, err, rc)
