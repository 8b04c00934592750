#!/usr/bin/env bash
# One Execute round trip against APP_GRPC_LISTEN_ADDR (default 0.0.0.0:50051).
cd "$(dirname "$0")/.." && exec python3 -m bee_code_interpreter_fs_amd.health_check
