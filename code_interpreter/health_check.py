"""``python -m code_interpreter.health_check`` -> the MI355X service's check."""
from bee_code_interpreter_fs_amd.health_check import health_check, main  # noqa: F401

if __name__ == "__main__":
    main()
