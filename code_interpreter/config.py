"""Re-export: the ``APP_*`` configuration of the MI355X service."""
from bee_code_interpreter_fs_amd.config import Config  # noqa: F401
