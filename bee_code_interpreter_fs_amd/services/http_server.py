"""REST API (FastAPI).

Routes and shapes follow `services/http_server.py:36-213` of the reference:

  PUT    /v1/files                   multipart field ``file`` -> {"hash": id}
  GET    /v1/files/{hash}?delete=    raw bytes (attachment), optional delete
  DELETE /v1/files/{hash}            {"message": "File deleted"}
  POST   /v1/execute                 {source_file | source_code, files, timeout}
  POST   /v1/parse-custom-tool       400 {"error_messages": [...]} on bad tools
  POST   /v1/execute-custom-tool     400 {"stderr": ...} when the tool fails

Differences: ``/v1/execute`` accepts ``source_code`` as well as this fork's
``source_file`` (the reference's own e2e tests send ``source_code``,
`test/e2e/test_http.py:24-28`) plus ``gpus`` / ``hbm_bytes`` / ``nprocs``;
downloads stream from disk instead of buffering; deleting a missing object
is a 404 instead of an unhandled 500; uploads also accept a raw
``application/octet-stream`` body.  Added: ``GET /health``, ``GET /metrics``,
``GET /v1/status``.
"""

from __future__ import annotations

import json
import logging
import socket
import time
from typing import Annotated, Dict, List, Optional

from fastapi import Depends, FastAPI, HTTPException, Request
from fastapi.responses import FileResponse, JSONResponse, PlainTextResponse
from pydantic import BaseModel, Field, StringConstraints
from starlette.background import BackgroundTask

from ..utils.logging import new_request_id
from ..utils.validation import ABSOLUTE_PATH_PATTERN, HASH_PATTERN, ValidationError
from .custom_tool_executor import CustomToolExecuteError, CustomToolExecutor, CustomToolParseError
from .metrics import METRICS
from .multipart import MultipartError, boundary_of, parse_multipart
from .storage import Storage

logger = logging.getLogger("code_interpreter_service")

AbsolutePath = Annotated[str, StringConstraints(pattern=ABSOLUTE_PATH_PATTERN)]
Hash = Annotated[str, StringConstraints(pattern=HASH_PATTERN)]


class ExecuteRequest(BaseModel):
    source_file: Optional[AbsolutePath] = None
    source_code: Optional[str] = None
    files: Dict[AbsolutePath, Hash] = Field(default_factory=dict)
    timeout: float = Field(default=60, gt=0, le=86400)
    gpus: Optional[int] = Field(default=None, ge=0, le=64)
    hbm_bytes: Optional[int] = Field(default=None, ge=0)
    nprocs: int = Field(default=1, ge=1, le=64)
    numpy_offload: Optional[bool] = None  # None = APP_NUMPY_OFFLOAD (ops/numpy_offload.py)


class ExecuteResponse(BaseModel):
    stdout: str
    stderr: str
    exit_code: int
    files: Dict[str, str]
    timings_ms: Dict[str, float] = Field(default_factory=dict)
    gpu_ids: List[int] = Field(default_factory=list)


class ParseCustomToolRequest(BaseModel):
    tool_source_code: str


class ParseCustomToolResponse(BaseModel):
    tool_name: str
    tool_input_schema_json: str
    tool_description: str


class ExecuteCustomToolRequest(BaseModel):
    tool_source_code: str
    tool_input_json: str


class ExecuteCustomToolResponse(BaseModel):
    tool_output_json: str


def create_http_server(code_executor, custom_tool_executor: CustomToolExecutor, file_storage: Storage,
                       peer_guard=None) -> FastAPI:
    """``peer_guard`` (services/peer_guard.py): every route but /health
    refuses callers that are sandboxes of this node with 403."""
    app = FastAPI(title="bee-code-interpreter (MI355X)")

    def set_request_id() -> str:
        return new_request_id()

    @app.middleware("http")
    async def _metrics(request: Request, call_next):
        t0 = time.perf_counter()
        if peer_guard is not None and request.client is not None and request.url.path != "/health":
            server = request.scope.get("server")
            fam = socket.AF_INET6 if ":" in request.client.host else socket.AF_INET
            why = await peer_guard.check(fam, request.client.host, request.client.port,
                                         tuple(server) if server and server[1] is not None else None)
            if why:
                logger.warning("%s %s refused: %s", request.method, request.url.path, why)
                METRICS.inc("bee_http_requests_total", route="refused", method=request.method, status=403)
                return JSONResponse(status_code=403, content={"detail": why})
        response = await call_next(request)
        route = request.scope.get("route")
        path = getattr(route, "path", "unmatched")
        METRICS.inc("bee_http_requests_total", route=path, method=request.method, status=response.status_code)
        METRICS.observe_ms("bee_http_latency_ms", (time.perf_counter() - t0) * 1e3, route=path)
        return response

    @app.put("/v1/files")
    async def write_file(request: Request, request_id: str = Depends(set_request_id)):
        ctype = request.headers.get("content-type", "")
        try:
            async with file_storage.writer() as w:
                if ctype.startswith("multipart/form-data"):
                    found = []

                    async def on_part(name, filename, headers):
                        if name == "file" and not found:
                            found.append(name)
                            return w.write
                        return None

                    await parse_multipart(request.stream(), boundary_of(ctype), on_part)
                    if not found:
                        raise HTTPException(status_code=422, detail="multipart field 'file' is required")
                else:
                    async for chunk in request.stream():
                        await w.write(chunk)
        except HTTPException:
            raise
        except MultipartError as e:
            raise HTTPException(status_code=422, detail=str(e))
        except Exception as e:
            logger.exception("Error writing file")
            raise HTTPException(status_code=500, detail=str(e))
        logger.info("Wrote file with hash %s", w.hash)
        return {"hash": w.hash}

    @app.get("/v1/files/{file_hash}")
    async def get_file(file_hash: str, delete: bool = False, request_id: str = Depends(set_request_id)):
        try:
            path = file_storage.path_of(file_hash)
        except ValueError:
            raise HTTPException(status_code=404, detail=f"File with hash {file_hash} not found")
        if not await file_storage.exists(file_hash):
            raise HTTPException(status_code=404, detail=f"File with hash {file_hash} not found")
        background = None
        if delete:

            async def _delete():
                try:
                    await file_storage.delete(file_hash)
                    logger.info("Deleted file with hash %s", file_hash)
                except FileNotFoundError:
                    pass

            background = BackgroundTask(_delete)
        return FileResponse(
            path,
            media_type="application/octet-stream",
            headers={"Content-Disposition": f"attachment; filename={file_hash}"},
            background=background,
        )

    @app.delete("/v1/files/{file_hash}")
    async def delete_file(file_hash: str, request_id: str = Depends(set_request_id)):
        try:
            await file_storage.delete(file_hash)
        except FileNotFoundError:
            raise HTTPException(status_code=404, detail=f"File with hash {file_hash} not found")
        logger.info("Deleted file with hash %s", file_hash)
        return {"message": "File deleted"}

    @app.post("/v1/execute", response_model=ExecuteResponse)
    async def execute(request: ExecuteRequest, request_id: str = Depends(set_request_id)):
        if (request.source_code is None) == (request.source_file is None):
            raise HTTPException(status_code=422, detail="exactly one of source_code / source_file is required")
        kwargs = dict(files=request.files, timeout=request.timeout, hbm_bytes=request.hbm_bytes)
        if request.gpus is not None:
            kwargs["gpus"] = request.gpus
            kwargs["nprocs"] = request.nprocs
        if request.numpy_offload is not None:
            kwargs["numpy_offload"] = request.numpy_offload
        if request.source_file is not None:
            kwargs["source_file"] = request.source_file
        else:
            kwargs["source_code"] = request.source_code
        logger.info("Executing code with files %s", request.files)
        try:
            result = await code_executor.execute(**kwargs)
        except FileNotFoundError as e:
            raise HTTPException(status_code=404, detail=str(e))
        except ValidationError as e:
            raise HTTPException(status_code=422, detail=e.errors)
        except ValueError as e:  # a request no GPU of the node can take (gpus, hbm_bytes)
            raise HTTPException(status_code=400, detail=str(e))
        except Exception as e:
            logger.exception("Error executing code")
            raise HTTPException(status_code=500, detail=str(e))
        METRICS.observe_phases("bee_execute_phase_ms", result.timings_ms)
        return ExecuteResponse(
            stdout=result.stdout,
            stderr=result.stderr,
            exit_code=result.exit_code,
            files=result.files,
            timings_ms=result.timings_ms,
            gpu_ids=result.gpu_ids,
        )

    @app.post("/v1/parse-custom-tool", response_model=ParseCustomToolResponse)
    async def parse_custom_tool(request: ParseCustomToolRequest, request_id: str = Depends(set_request_id)):
        tool = custom_tool_executor.parse(tool_source_code=request.tool_source_code)
        return ParseCustomToolResponse(
            tool_name=tool.name,
            tool_input_schema_json=json.dumps(tool.input_schema),
            tool_description=tool.description,
        )

    @app.exception_handler(CustomToolParseError)
    async def _parse_error(request, e: CustomToolParseError):
        logger.warning("Invalid custom tool: %s", e.errors)
        return JSONResponse(status_code=400, content={"error_messages": e.errors})

    @app.post("/v1/execute-custom-tool", response_model=ExecuteCustomToolResponse)
    async def execute_custom_tool(request: ExecuteCustomToolRequest, request_id: str = Depends(set_request_id)):
        try:
            tool_input = json.loads(request.tool_input_json)
        except json.JSONDecodeError as e:
            raise HTTPException(status_code=422, detail=f"tool_input_json: {e}")
        result = await custom_tool_executor.execute(tool_source_code=request.tool_source_code, tool_input=tool_input)
        return ExecuteCustomToolResponse(tool_output_json=json.dumps(result))

    @app.exception_handler(CustomToolExecuteError)
    async def _exec_error(request, e: CustomToolExecuteError):
        logger.warning("Error executing custom tool: %s", e.stderr[-500:])
        return JSONResponse(status_code=400, content={"stderr": e.stderr})

    @app.get("/health")
    async def health():
        ok = code_executor.healthy()
        return JSONResponse(status_code=200 if ok else 503, content={"status": "SERVING" if ok else "NOT_SERVING"})

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(METRICS.render(), media_type="text/plain; version=0.0.4")

    @app.get("/v1/status")
    async def status():
        if hasattr(code_executor, "status"):
            return await code_executor.status()
        return code_executor.stats()

    return app
