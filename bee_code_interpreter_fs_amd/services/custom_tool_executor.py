"""Custom tools: turn a Python function's source into an LLM tool definition
(name, description, JSON-Schema draft-07 input schema) and run it in a sandbox.

Behavioural parity with `src/code_interpreter/services/custom_tool_executor.py`
(rules pinned by `test/e2e/test_grpc.py:109-261`):

* source = ``[import ...]* + def`` after ``textwrap.dedent``; syntax errors
  become ``"Syntax error: {msg} on line {lineno}"`` (`:59-62`);
* argument-shape errors are *collected* (`:73-96`) with the exact messages
  below;
* docstring directives ``:param <name>:`` / ``:return:`` start at the
  beginning of a line and may span several lines (`:242-264`);
* ``required`` = positional args without defaults + keyword-only args with no
  default (`:114-125`);
* description = function description + ``"\\n\\nReturns: <ann> -- <doc>"``
  (`:132-148`);
* execution wraps the tool in a script that silences the tool's own stdout,
  calls it with the JSON input and prints ``json.dumps(result)``; a non-zero
  exit raises :class:`CustomToolExecuteError` with the sandbox stderr.

Documented divergences (supersets / bug fixes):

* ``Any`` maps to ``{}`` ("any JSON value") instead of ``{"type": "array"}``;
* an unsupported annotation is reported as a parse error instead of
  escaping as an uncaught ``ValueError``;
* ``List``/``Dict``/``tuple``/``X | Y``/``None`` annotations and parameter
  names with digits/capitals are accepted.
"""

from __future__ import annotations

import ast
import inspect
import json
import re
import textwrap
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

JSON_SCHEMA_DRAFT7 = "http://json-schema.org/draft-07/schema#"

ERR_SHAPE = "The tool source code must only define a single function, optionally preceded by imports."
ERR_POSONLY = "The tool function must not have positional-only arguments"
ERR_VARARGS = "The tool function must not have *args"
ERR_KWARGS = "The tool function must not have **kwargs"
ERR_ANNOTATIONS = "The tool function arguments must have type annotations"


@dataclass
class CustomTool:
    name: str
    description: str
    input_schema: Dict[str, Any]


class CustomToolParseError(Exception):
    def __init__(self, errors: List[str]) -> None:
        super().__init__("; ".join(errors))
        self.errors = list(errors)


class CustomToolExecuteError(Exception):
    def __init__(self, stderr: str) -> None:
        super().__init__(stderr)
        self.stderr = stderr


class UnsupportedAnnotation(Exception):
    pass


# --------------------------------------------------------------------------
# parsing
# --------------------------------------------------------------------------


def _split_source(tool_source_code: str) -> Tuple[List[ast.stmt], ast.FunctionDef]:
    source = textwrap.dedent(tool_source_code)
    try:
        body = ast.parse(source).body
    except SyntaxError as e:
        raise CustomToolParseError([f"Syntax error: {e.msg} on line {e.lineno}"])
    if not body:
        raise CustomToolParseError([ERR_SHAPE])
    *prelude, fn = body
    if not isinstance(fn, ast.FunctionDef) or any(
        not isinstance(node, (ast.Import, ast.ImportFrom)) for node in prelude
    ):
        raise CustomToolParseError([ERR_SHAPE])
    return prelude, fn


def _shape_errors(fn: ast.FunctionDef) -> List[str]:
    a = fn.args
    checks = [
        (bool(a.posonlyargs), ERR_POSONLY),
        (a.vararg is not None, ERR_VARARGS),
        (a.kwarg is not None, ERR_KWARGS),
        (any(arg.annotation is None for arg in a.args + a.kwonlyargs), ERR_ANNOTATIONS),
    ]
    return [msg for failed, msg in checks if failed]


_DIRECTIVE = re.compile(r"^\s*:")
_PARAM = re.compile(r"^params?\s+([A-Za-z_][A-Za-z0-9_]*)\s*:\s?(.*)\Z", re.DOTALL)
_RETURN = re.compile(r"^returns?\s*:\s?(.*)\Z", re.DOTALL)


def parse_docstring(docstring: str) -> Tuple[str, str, Dict[str, str]]:
    """ReST-ish docstring → (description, return description, {param: text}).

    A line whose first non-blank character is ``:`` opens a directive; every
    following line up to the next directive continues it.
    """
    sections: List[List[str]] = [[]]
    for line in inspect.cleandoc(docstring or "").split("\n"):
        if _DIRECTIVE.match(line):
            sections.append([line.lstrip()[1:]])
        else:
            sections[-1].append(line)
    texts = ["\n".join(s).strip() for s in sections]
    params: Dict[str, str] = {}
    returns = ""
    for text in texts[1:]:
        m = _PARAM.match(text)
        if m:
            params[m.group(1)] = m.group(2).strip()
            continue
        m = _RETURN.match(text)
        if m:
            returns = m.group(1).strip()
    return texts[0], returns, params


_SCALARS = {
    "int": {"type": "integer"},
    "float": {"type": "number"},
    "str": {"type": "string"},
    "bool": {"type": "boolean"},
    "None": {"type": "null"},
    "Any": {},
    "typing.Any": {},
}


def _strip_typing(name: str) -> str:
    return name[len("typing.") :] if name.startswith("typing.") else name


def annotation_to_schema(node: ast.AST) -> Dict[str, Any]:
    """Map a type annotation AST to a JSON schema fragment."""
    if isinstance(node, ast.Constant) and node.value is None:
        return {"type": "null"}
    if isinstance(node, ast.BinOp) and isinstance(node.op, ast.BitOr):
        return {"anyOf": [annotation_to_schema(node.left), annotation_to_schema(node.right)]}
    if isinstance(node, ast.Subscript):
        head = _strip_typing(ast.unparse(node.value))
        params = node.slice.elts if isinstance(node.slice, ast.Tuple) else [node.slice]
        if head in ("list", "List") and len(params) == 1:
            return {"type": "array", "items": annotation_to_schema(params[0])}
        if head in ("dict", "Dict") and len(params) == 2:
            if ast.unparse(params[0]) != "str":
                raise UnsupportedAnnotation(f"Unsupported type: {ast.unparse(node)} (object keys must be str)")
            return {"type": "object", "additionalProperties": annotation_to_schema(params[1])}
        if head == "Optional" and len(params) == 1:
            return {"anyOf": [{"type": "null"}, annotation_to_schema(params[0])]}
        if head == "Union":
            return {"anyOf": [annotation_to_schema(p) for p in params]}
        if head in ("Tuple", "tuple") and isinstance(node.slice, ast.Tuple):
            return {
                "type": "array",
                "minItems": len(params),
                "items": [annotation_to_schema(p) for p in params],
                "additionalItems": False,
            }
        raise UnsupportedAnnotation(f"Unsupported type: {ast.unparse(node)}")
    name = ast.unparse(node)
    if name in _SCALARS:
        return dict(_SCALARS[name])
    raise UnsupportedAnnotation(f"Unsupported type: {name}")


def parse_tool(tool_source_code: str) -> CustomTool:
    _, fn = _split_source(tool_source_code)
    errors = _shape_errors(fn)
    if errors:
        raise CustomToolParseError(errors)

    description, return_doc, param_docs = parse_docstring(ast.get_docstring(fn) or "")
    properties: Dict[str, Any] = {}
    type_errors: List[str] = []
    for arg in fn.args.args + fn.args.kwonlyargs:
        try:
            schema = annotation_to_schema(arg.annotation)
        except UnsupportedAnnotation as e:
            type_errors.append(f"{e} (argument {arg.arg!r})")
            continue
        if param_docs.get(arg.arg):
            schema["description"] = param_docs[arg.arg]
        properties[arg.arg] = schema
    if type_errors:
        raise CustomToolParseError(type_errors)

    n_positional_required = len(fn.args.args) - len(fn.args.defaults)
    required = [a.arg for a in fn.args.args[:n_positional_required]]
    required += [a.arg for a, d in zip(fn.args.kwonlyargs, fn.args.kw_defaults) if d is None]

    returns = " -- ".join(p for p in (ast.unparse(fn.returns) if fn.returns else "", return_doc) if p)
    full_description = "\n\n".join(p for p in (description, f"Returns: {returns}" if returns else "") if p)

    return CustomTool(
        name=fn.name,
        description=full_description,
        input_schema={
            "$schema": JSON_SCHEMA_DRAFT7,
            "type": "object",
            "title": fn.name,
            "properties": properties,
            "required": required,
            "additionalProperties": False,
        },
    )


# --------------------------------------------------------------------------
# execution
# --------------------------------------------------------------------------

_RUNNER = """\
import contextlib as _bee_ctx
import json as _bee_json
{imports}

_bee_ns = {{}}
with _bee_ctx.redirect_stdout(None):
    exec(compile({source!r}, "<tool>", "exec"), _bee_ns)
    _bee_result = _bee_ns[{name!r}](**_bee_json.loads({payload!r}))
print(_bee_json.dumps(_bee_result))
"""


def build_tool_script(tool_source_code: str, tool_input: Dict[str, Any]) -> str:
    """Script that runs the tool once; imports are hoisted so the sandbox's
    dependency scan sees them."""
    prelude, fn = _split_source(tool_source_code)
    return _RUNNER.format(
        imports="\n".join(ast.unparse(node) for node in prelude),
        source=textwrap.dedent(tool_source_code),
        name=fn.name,
        payload=json.dumps(tool_input),
    )


class CustomToolExecutor:
    def __init__(self, code_executor) -> None:
        self.code_executor = code_executor

    def parse(self, tool_source_code: str) -> CustomTool:
        return parse_tool(tool_source_code)

    async def execute(self, tool_source_code: str, tool_input: Dict[str, Any], timeout: Optional[float] = None) -> Any:
        if not isinstance(tool_input, dict):
            raise CustomToolExecuteError("tool input must be a JSON object")
        script = build_tool_script(tool_source_code, tool_input)
        result = await self.code_executor.execute(source_code=script, timeout=timeout)
        if result.exit_code != 0:
            raise CustomToolExecuteError(result.stderr)
        try:
            return json.loads(result.stdout)
        except json.JSONDecodeError as e:
            raise CustomToolExecuteError(f"tool output is not JSON ({e}): {result.stdout[-2000:]}")
