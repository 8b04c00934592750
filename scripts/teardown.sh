#!/usr/bin/env bash
# Remove sandboxes left behind by a killed service (the daemons clean up on
# normal shutdown; executors die with their service via PDEATHSIG).
set -euo pipefail
rm -rf "${APP_SANDBOX_ROOT:-/dev/shm/bee-sandboxes}" /tmp/bee-run-* 2>/dev/null || true
