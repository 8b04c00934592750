"""``python -m code_interpreter.health_check`` -> the MI355X service's check."""
import sys

from bee_code_interpreter_fs_amd.health_check import health_check

if __name__ == "__main__":
    try:
        health_check()
    except Exception as e:  # noqa: BLE001
        print(f"health check failed: {e}", file=sys.stderr)
        sys.exit(1)
