"""Wire schemas: ``code_interpreter.v1`` (bee-proto), ``grpc.health.v1`` and
``grpc.reflection.v1alpha`` / ``grpc.reflection.v1``.

The reference imports generated classes from the ``bee-proto`` submodule,
which is empty in the reference snapshot (`.gitmodules:1-4`).  Message and
field *names* below are confirmed by the reference's usage (servicer
`code_interpreter_servicer.py:55-135`, `health_check.py:48`, e2e tests);
field *numbers* and the names of the oneof arm message types are
reconstructed and UNVERIFIED — they all live in :data:`CODE_INTERPRETER_FIELDS`
so they can be corrected in one place.  JSON / grpcurl clients depend only
on names; binary clients depend on the numbers.

Fields numbered >= 100 are MI355X-native extensions (timeout, GPU gang size,
HBM quota, path-based execute, timings); old clients never set them.
"""

from __future__ import annotations

from google.protobuf import descriptor_pool

from .protobuf_builder import (
    BOOL,
    BYTES,
    DOUBLE,
    INT32,
    INT64,
    STRING,
    CompiledFile,
    Field,
    Map,
    Message,
    Method,
    Service,
    build_file,
)

CI_PACKAGE = "code_interpreter.v1"
CI_FILE = "code_interpreter/v1/code_interpreter_service.proto"
CI_SERVICE = f"{CI_PACKAGE}.CodeInterpreterService"

_P = "." + CI_PACKAGE

# ---- the single table of reconstructed field numbers ------------------------
CODE_INTERPRETER_FIELDS = {
    "ExecuteRequest": [
        Field("source_code", 1, STRING),
        Field("executor_id", 2, STRING),
        Field("files", 3, Map(STRING, STRING)),
        # extensions
        Field("timeout", 100, DOUBLE),
        Field("gpus", 101, INT32),
        Field("hbm_bytes", 102, INT64),
        Field("source_file", 103, STRING),
        # unset = the service default (APP_NUMPY_OFFLOAD); ops/numpy_offload.py
        Field("numpy_offload", 104, BOOL, proto3_optional=True),
    ],
    "ExecuteResponse": [
        Field("stdout", 1, STRING),
        Field("stderr", 2, STRING),
        Field("exit_code", 3, INT32),
        Field("files", 4, Map(STRING, STRING)),
        # extensions
        Field("timings_ms", 100, Map(STRING, DOUBLE)),
        Field("gpu_ids", 101, INT32, repeated=True),
    ],
    "ParseCustomToolRequest": [
        Field("tool_source_code", 1, STRING),
    ],
    "ParseCustomToolResponseSuccess": [
        Field("tool_name", 1, STRING),
        Field("tool_input_schema_json", 2, STRING),
        Field("tool_description", 3, STRING),
    ],
    "ParseCustomToolResponseError": [
        Field("error_messages", 1, STRING, repeated=True),
    ],
    "ParseCustomToolResponse": [
        Field("success", 1, _P + ".ParseCustomToolResponseSuccess", oneof="response"),
        Field("error", 2, _P + ".ParseCustomToolResponseError", oneof="response"),
    ],
    "ExecuteCustomToolRequest": [
        Field("tool_source_code", 1, STRING),
        Field("tool_input_json", 2, STRING),
        Field("executor_id", 3, STRING),
    ],
    "ExecuteCustomToolResponseSuccess": [
        Field("tool_output_json", 1, STRING),
    ],
    "ExecuteCustomToolResponseError": [
        Field("stderr", 1, STRING),
    ],
    "ExecuteCustomToolResponse": [
        Field("success", 1, _P + ".ExecuteCustomToolResponseSuccess", oneof="response"),
        Field("error", 2, _P + ".ExecuteCustomToolResponseError", oneof="response"),
    ],
}

CI_METHODS = [
    Method("Execute", _P + ".ExecuteRequest", _P + ".ExecuteResponse"),
    Method("ParseCustomTool", _P + ".ParseCustomToolRequest", _P + ".ParseCustomToolResponse"),
    Method("ExecuteCustomTool", _P + ".ExecuteCustomToolRequest", _P + ".ExecuteCustomToolResponse"),
]

# ---- grpc.health.v1 (standard schema) ---------------------------------------
HEALTH_PACKAGE = "grpc.health.v1"
HEALTH_FILE = "grpc/health/v1/health.proto"
HEALTH_SERVICE = f"{HEALTH_PACKAGE}.Health"
HEALTH_STATUS = (("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2), ("SERVICE_UNKNOWN", 3))

# ---- grpc.reflection (standard schema, v1alpha and v1 are identical) ---------
REFLECTION_FILES = {
    "grpc.reflection.v1alpha": "grpc_reflection/v1alpha/reflection.proto",
    "grpc.reflection.v1": "grpc/reflection/v1/reflection.proto",
}


def _reflection_messages(p: str):
    return [
        Message(
            "ServerReflectionRequest",
            [
                Field("host", 1, STRING),
                Field("file_by_filename", 3, STRING, oneof="message_request"),
                Field("file_containing_symbol", 4, STRING, oneof="message_request"),
                Field("file_containing_extension", 5, f".{p}.ExtensionRequest", oneof="message_request"),
                Field("all_extension_numbers_of_type", 6, STRING, oneof="message_request"),
                Field("list_services", 7, STRING, oneof="message_request"),
            ],
        ),
        Message("ExtensionRequest", [Field("containing_type", 1, STRING), Field("extension_number", 2, INT32)]),
        Message(
            "ServerReflectionResponse",
            [
                Field("valid_host", 1, STRING),
                Field("original_request", 2, f".{p}.ServerReflectionRequest"),
                Field("file_descriptor_response", 4, f".{p}.FileDescriptorResponse", oneof="message_response"),
                Field("all_extension_numbers_response", 5, f".{p}.ExtensionNumberResponse", oneof="message_response"),
                Field("list_services_response", 6, f".{p}.ListServiceResponse", oneof="message_response"),
                Field("error_response", 7, f".{p}.ErrorResponse", oneof="message_response"),
            ],
        ),
        Message("FileDescriptorResponse", [Field("file_descriptor_proto", 1, BYTES, repeated=True)]),
        Message(
            "ExtensionNumberResponse",
            [Field("base_type_name", 1, STRING), Field("extension_number", 2, INT32, repeated=True)],
        ),
        Message("ListServiceResponse", [Field("service", 1, f".{p}.ServiceResponse", repeated=True)]),
        Message("ServiceResponse", [Field("name", 1, STRING)]),
        Message("ErrorResponse", [Field("error_code", 1, INT32), Field("error_message", 2, STRING)]),
    ]


POOL = descriptor_pool.DescriptorPool()

code_interpreter = CompiledFile(
    build_file(
        CI_FILE,
        CI_PACKAGE,
        [Message(name, fields) for name, fields in CODE_INTERPRETER_FIELDS.items()],
        [Service("CodeInterpreterService", CI_METHODS)],
    ),
    POOL,
)

health = CompiledFile(
    build_file(
        HEALTH_FILE,
        HEALTH_PACKAGE,
        [
            Message("HealthCheckRequest", [Field("service", 1, STRING)]),
            Message(
                "HealthCheckResponse",
                [Field("status", 1, f"enum:.{HEALTH_PACKAGE}.HealthCheckResponse.ServingStatus")],
                enums={"ServingStatus": HEALTH_STATUS},
            ),
        ],
        [
            Service(
                "Health",
                [
                    Method("Check", f".{HEALTH_PACKAGE}.HealthCheckRequest", f".{HEALTH_PACKAGE}.HealthCheckResponse"),
                    Method(
                        "Watch",
                        f".{HEALTH_PACKAGE}.HealthCheckRequest",
                        f".{HEALTH_PACKAGE}.HealthCheckResponse",
                        server_streaming=True,
                    ),
                ],
            )
        ],
    ),
    POOL,
)

reflection = {
    pkg: CompiledFile(
        build_file(
            fname,
            pkg,
            _reflection_messages(pkg),
            [
                Service(
                    "ServerReflection",
                    [
                        Method(
                            "ServerReflectionInfo",
                            f".{pkg}.ServerReflectionRequest",
                            f".{pkg}.ServerReflectionResponse",
                            client_streaming=True,
                            server_streaming=True,
                        )
                    ],
                )
            ],
        ),
        POOL,
    )
    for pkg, fname in REFLECTION_FILES.items()
}

# convenient aliases mirroring generated-module names
ExecuteRequest = code_interpreter.ExecuteRequest
ExecuteResponse = code_interpreter.ExecuteResponse
ParseCustomToolRequest = code_interpreter.ParseCustomToolRequest
ParseCustomToolResponse = code_interpreter.ParseCustomToolResponse
ExecuteCustomToolRequest = code_interpreter.ExecuteCustomToolRequest
ExecuteCustomToolResponse = code_interpreter.ExecuteCustomToolResponse
HealthCheckRequest = health.HealthCheckRequest
HealthCheckResponse = health.HealthCheckResponse

ALL_FILES = [code_interpreter, health, *reflection.values()]


def method_path(service: str, method: str) -> str:
    return f"/{service}/{method}"


class CodeInterpreterServiceStub:
    """Client stub (sync or aio channel), equivalent of the generated stub."""

    def __init__(self, channel) -> None:
        for m in CI_METHODS:
            req = code_interpreter.messages[m.input.rsplit(".", 1)[1]]
            resp = code_interpreter.messages[m.output.rsplit(".", 1)[1]]
            setattr(
                self,
                m.name,
                channel.unary_unary(
                    method_path(CI_SERVICE, m.name),
                    request_serializer=req.SerializeToString,
                    response_deserializer=resp.FromString,
                ),
            )


class HealthStub:
    def __init__(self, channel) -> None:
        self.Check = channel.unary_unary(
            method_path(HEALTH_SERVICE, "Check"),
            request_serializer=HealthCheckRequest.SerializeToString,
            response_deserializer=HealthCheckResponse.FromString,
        )
        self.Watch = channel.unary_stream(
            method_path(HEALTH_SERVICE, "Watch"),
            request_serializer=HealthCheckRequest.SerializeToString,
            response_deserializer=HealthCheckResponse.FromString,
        )
