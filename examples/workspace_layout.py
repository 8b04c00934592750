# The sandbox's working directory and what was staged into it.
import os

print("cwd:", os.getcwd())
for root, dirs, names in os.walk("."):
    for n in sorted(names):
        print(os.path.join(root, n))
