# Smallest possible payload: CPU plumbing benchmark (BASELINE config 1).
print("hello world")
