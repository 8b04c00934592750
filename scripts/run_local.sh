#!/usr/bin/env bash
# Build the native pieces and run the service on this node's GPUs.
#   scripts/run_local.sh            # all visible MI355X, one front-end per GPU
#   APP_GPU_IDS='[]' scripts/run_local.sh   # CPU-only sandboxes
set -euo pipefail
cd "$(dirname "$0")/.."
python3 -c "import __graft_entry__ as g; g.build()"
export APP_FILE_STORAGE_PATH="${APP_FILE_STORAGE_PATH:-./.tmp/files}"
export APP_SANDBOX_ROOT="${APP_SANDBOX_ROOT:-/dev/shm/bee-sandboxes}"
export APP_FRONTEND_PROCESSES="${APP_FRONTEND_PROCESSES:-0}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
exec python3 -m bee_code_interpreter_fs_amd
