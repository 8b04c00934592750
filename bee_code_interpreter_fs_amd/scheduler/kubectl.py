"""Async ``kubectl`` CLI wrapper (Kubernetes backend only).

Same contract as the reference (`services/kubectl.py:24-193`): a method per
sub-command (``kubectl.get("pod", name)``), kwargs become ``--key=value``
flags (``True`` -> bare ``--key``; falsy dropped; a leading ``_`` is stripped
so ``_for=`` can spell ``--for=``), flags go before a ``--`` separator,
commands that support it get ``--output=json`` and return parsed JSON, and a
non-zero exit raises ``RuntimeError`` with stderr.  Constructor kwargs are
default flags for every command (namespace, context).
"""

from __future__ import annotations

import asyncio
import json
import logging
import shlex
from typing import Any, Dict, List, Optional, Union

logger = logging.getLogger("kubectl")

JSON_VERBS = frozenset(
    "annotate apply autoscale create edit events expose get label patch replace run scale taint version wait".split()
)
TEXT_VERBS = frozenset(
    (
        "api_resources api_versions attach auth certificate cluster_info completion config cordon cp ctx debug "
        "delete describe diff drain exec explain help kustomize logs ns options plugin port_forward proxy rollout "
        "set top uncordon"
    ).split()
)

Input = Union[bytes, str, list, dict, None]


def _flags(kwargs: Dict[str, Any]) -> Dict[str, Any]:
    # None/False/"" drop the flag; 0 is a real value (--grace-period=0), which
    # the reference's truthiness filter silently dropped
    return {k.lstrip("_").replace("_", "-"): v for k, v in kwargs.items() if v is not None and v is not False and v != ""}


class Kubectl:
    def __init__(self, binary: str = "kubectl", **defaults: Any) -> None:
        self.binary = binary
        self.defaults = _flags(defaults)

    def build_args(self, verb: str, *args: str, **kwargs: Any) -> List[str]:
        flags = {**self.defaults, **_flags(kwargs)}
        rendered = [f"--{k}" if v is True else f"--{k}={v}" for k, v in flags.items()]
        args_l = list(args)
        cut = args_l.index("--") if "--" in args_l else len(args_l)
        return [verb.replace("_", "-"), *args_l[:cut], *rendered, *args_l[cut:]]

    async def _exec(self, argv: List[str], stdin: Optional[bytes]) -> tuple:
        proc = await asyncio.create_subprocess_exec(
            self.binary, *argv,
            stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE,
        )
        out, err = await proc.communicate(stdin)
        return proc.returncode, out, err

    async def command(self, verb: str, *args: str, input: Input = None, **kwargs: Any) -> Union[str, dict]:
        as_json = verb in JSON_VERBS
        if as_json:
            kwargs.setdefault("output", "json")
        argv = self.build_args(verb, *args, **kwargs)
        logger.info("kubectl %s", shlex.join(argv))
        if isinstance(input, (list, dict)):
            input = json.dumps(input)
        if isinstance(input, str):
            input = input.encode()
        code, out, err = await self._exec(argv, input or None)
        if code != 0:
            raise RuntimeError(f"Error ({code}) running kubectl command: {err.decode(errors='replace')}")
        text = out.decode()
        return json.loads(text) if as_json and text.strip() else text

    def __getattr__(self, name: str):
        if name.startswith("__") or (name not in JSON_VERBS and name not in TEXT_VERBS):
            raise AttributeError(f"Command {name} not found")

        async def call(*args: str, input: Input = None, **kwargs: Any):
            return await self.command(name, *args, input=input, **kwargs)

        call.__name__ = name
        return call

    async def exec_raw(self, *args: str, **kwargs: Any) -> asyncio.subprocess.Process:
        argv = self.build_args("exec", *args, **kwargs)
        return await asyncio.create_subprocess_exec(
            self.binary, *argv,
            stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE,
        )
