"""Health check CLI: one real ``Execute`` round trip.

Parity with `src/code_interpreter/health_check.py:25-53`: sends
``Execute(executor_id="health-check", source_code="print(21 * 2)")`` to
``APP_GRPC_LISTEN_ADDR`` and asserts stdout ``"42\\n"``.  The reference's TLS
branch hands *server* credentials to a client channel (`:35-43`); this uses
``grpc.ssl_channel_credentials`` (CA + client cert/key).
"""

from __future__ import annotations

import sys

import grpc

from .config import Config
from .models import proto as pb


def make_channel(config: Config, target: str = None):
    target = target or config.grpc_listen_addr.replace("0.0.0.0", "127.0.0.1")
    if not (config.grpc_tls_cert and config.grpc_tls_cert_key and config.grpc_tls_ca_cert):
        return grpc.insecure_channel(target)
    creds = grpc.ssl_channel_credentials(
        root_certificates=config.grpc_tls_ca_cert,
        private_key=config.grpc_tls_cert_key,
        certificate_chain=config.grpc_tls_cert,
    )
    return grpc.secure_channel(target, creds)


def health_check(config: Config = None, target: str = None, timeout: float = 9999) -> None:
    config = config or Config()
    with make_channel(config, target) as channel:
        response = pb.CodeInterpreterServiceStub(channel).Execute(
            pb.ExecuteRequest(executor_id="health-check", source_code="print(21 * 2)"),
            timeout=timeout,  # k8s probes carry their own timeouts
        )
    assert response.stdout == "42\n", f"unexpected health-check output: {response.stdout!r} / {response.stderr!r}"


def main() -> None:
    try:
        health_check()
    except Exception as e:  # noqa: BLE001
        print(f"health check failed: {e}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
