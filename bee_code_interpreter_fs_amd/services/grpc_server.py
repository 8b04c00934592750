"""gRPC host: CodeInterpreterService + grpc.health.v1 + server reflection.

Parity: `services/grpc_server.py:22-71` — ``grpc.aio`` server, insecure or TLS
port, reflection enabled (the README's grpcurl example relies on it,
`README.md:46`), ``stop(grace=5)``.  The reference left health checking as a
TODO (`:71`); the standard ``grpc.health.v1.Health`` service is implemented
here, reporting NOT_SERVING when no executor slot is healthy.

There are no generated stubs on this image, so handlers are registered with
``grpc.method_handlers_generic_handler`` and message classes built from the
descriptors in ``models/proto.py``; reflection serves those same descriptors.
"""

from __future__ import annotations

import asyncio
import logging
from typing import Callable, Dict, List, Optional

import grpc

from ..models import proto as pb

logger = logging.getLogger("grpc_server")


def _unary(fn, req_cls, resp_cls):
    return grpc.unary_unary_rpc_method_handler(
        fn, request_deserializer=req_cls.FromString, response_serializer=resp_cls.SerializeToString
    )


class HealthServicer:
    SERVING, NOT_SERVING, SERVICE_UNKNOWN = 1, 2, 3

    def __init__(self, services: List[str], probe: Callable[[], bool]) -> None:
        self.services = set(services)
        self.probe = probe

    def _status(self, service: str) -> int:
        if service and service not in self.services:
            return self.SERVICE_UNKNOWN
        return self.SERVING if self.probe() else self.NOT_SERVING

    async def Check(self, request, context):
        status = self._status(request.service)
        if status == self.SERVICE_UNKNOWN:
            await context.abort(grpc.StatusCode.NOT_FOUND, f"unknown service {request.service!r}")
        return pb.HealthCheckResponse(status=status)

    async def Watch(self, request, context):
        last = None
        while True:
            status = self._status(request.service)
            if status != last:
                yield pb.HealthCheckResponse(status=status)
                last = status
            await asyncio.sleep(2.0)


class ReflectionServicer:
    """grpc.reflection.v1alpha / v1 ServerReflectionInfo over our descriptors."""

    def __init__(self, package: str, service_names: List[str]) -> None:
        self.msgs = pb.reflection[package]
        self.service_names = service_names
        self.by_name: Dict[str, bytes] = {f.proto.name: f.serialized for f in pb.ALL_FILES}

    def _file_response(self, names: List[str]):
        seen, out = set(), []

        def add(name: str) -> None:
            if name in seen or name not in self.by_name:
                return
            seen.add(name)
            out.append(self.by_name[name])
            for dep in pb.POOL.FindFileByName(name).dependencies:
                add(dep.name)

        for n in names:
            add(n)
        return self.msgs.FileDescriptorResponse(file_descriptor_proto=out)

    def _symbol_file(self, symbol: str) -> Optional[str]:
        try:
            return pb.POOL.FindFileContainingSymbol(symbol).name
        except KeyError:
            pass
        # "pkg.Service.Method" -> look the service up
        head = symbol.rsplit(".", 1)[0]
        try:
            return pb.POOL.FindFileContainingSymbol(head).name
        except KeyError:
            return None

    def _answer(self, req):
        M = self.msgs
        resp = M.ServerReflectionResponse(valid_host=req.host, original_request=req)
        kind = req.WhichOneof("message_request")
        if kind == "list_services":
            resp.list_services_response.CopyFrom(
                M.ListServiceResponse(service=[M.ServiceResponse(name=n) for n in self.service_names])
            )
        elif kind == "file_by_filename":
            if req.file_by_filename in self.by_name:
                resp.file_descriptor_response.CopyFrom(self._file_response([req.file_by_filename]))
            else:
                resp.error_response.CopyFrom(M.ErrorResponse(error_code=5, error_message="file not found"))
        elif kind == "file_containing_symbol":
            name = self._symbol_file(req.file_containing_symbol)
            if name:
                resp.file_descriptor_response.CopyFrom(self._file_response([name]))
            else:
                resp.error_response.CopyFrom(M.ErrorResponse(error_code=5, error_message="symbol not found"))
        elif kind == "all_extension_numbers_of_type":
            resp.all_extension_numbers_response.CopyFrom(
                M.ExtensionNumberResponse(base_type_name=req.all_extension_numbers_of_type)
            )
        else:
            resp.error_response.CopyFrom(M.ErrorResponse(error_code=12, error_message="unimplemented"))
        return resp

    async def ServerReflectionInfo(self, request_iterator, context):
        async for req in request_iterator:
            yield self._answer(req)


class GrpcServer:
    def __init__(self, servicer, health_probe: Callable[[], bool], server_credentials=None) -> None:
        self.server = grpc.aio.server(
            options=[("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)]
        )
        self.server_credentials = server_credentials
        self.bound_port: Optional[int] = None
        self.peer_guard = getattr(servicer, "peer_guard", None)  # learns the ports bound below
        services = [pb.CI_SERVICE, pb.HEALTH_SERVICE] + [f"{p}.ServerReflection" for p in pb.REFLECTION_FILES]
        ci = {
            "Execute": _unary(servicer.Execute, pb.ExecuteRequest, pb.ExecuteResponse),
            "ParseCustomTool": _unary(servicer.ParseCustomTool, pb.ParseCustomToolRequest, pb.ParseCustomToolResponse),
            "ExecuteCustomTool": _unary(
                servicer.ExecuteCustomTool, pb.ExecuteCustomToolRequest, pb.ExecuteCustomToolResponse
            ),
        }
        health = HealthServicer([pb.CI_SERVICE], health_probe)
        hh = {
            "Check": _unary(health.Check, pb.HealthCheckRequest, pb.HealthCheckResponse),
            "Watch": grpc.unary_stream_rpc_method_handler(
                health.Watch,
                request_deserializer=pb.HealthCheckRequest.FromString,
                response_serializer=pb.HealthCheckResponse.SerializeToString,
            ),
        }
        handlers = [
            grpc.method_handlers_generic_handler(pb.CI_SERVICE, ci),
            grpc.method_handlers_generic_handler(pb.HEALTH_SERVICE, hh),
        ]
        for pkg in pb.REFLECTION_FILES:
            r = ReflectionServicer(pkg, services)
            m = pb.reflection[pkg]
            handlers.append(
                grpc.method_handlers_generic_handler(
                    f"{pkg}.ServerReflection",
                    {
                        "ServerReflectionInfo": grpc.stream_stream_rpc_method_handler(
                            r.ServerReflectionInfo,
                            request_deserializer=m.ServerReflectionRequest.FromString,
                            response_serializer=m.ServerReflectionResponse.SerializeToString,
                        )
                    },
                )
            )
        self.server.add_generic_rpc_handlers(handlers)
        for s in services:
            logger.info("Registered service %s", s)

    def bind(self, listen_addr: str) -> int:
        if self.server_credentials is None:
            logger.info("Starting server on insecure port %s", listen_addr)
            self.bound_port = self.server.add_insecure_port(listen_addr)
        else:
            logger.info("Starting server on secure port %s", listen_addr)
            self.bound_port = self.server.add_secure_port(listen_addr, self.server_credentials)
        if self.peer_guard is not None and self.bound_port:
            self.peer_guard.ports.add(self.bound_port)
        return self.bound_port

    async def start(self, listen_addr: Optional[str] = None) -> None:
        if listen_addr is not None:
            self.bind(listen_addr)
        await self.server.start()

    async def serve(self, listen_addr: str) -> None:
        await self.start(listen_addr)
        try:
            await self.server.wait_for_termination()
        finally:
            await self.server.stop(grace=5)

    async def stop(self, grace: float = 5) -> None:
        await self.server.stop(grace=grace)
