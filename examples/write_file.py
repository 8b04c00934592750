# Creates a workspace file; the Execute response reports it in `files`.
with open("greeting.txt", "w") as fh:
    fh.write("Hello, World!")
print("wrote greeting.txt")
