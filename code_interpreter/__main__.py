from bee_code_interpreter_fs_amd.__main__ import run

run()
