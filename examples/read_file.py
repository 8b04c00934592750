# Run with files={"/workspace/greeting.txt": <id returned by write_file.py>}.
# Reading an unchanged input does not re-report it.
with open("/workspace/greeting.txt") as fh:
    print(fh.read())
