# Non-zero exit code with the Python traceback in stderr.
numerator, denominator = 1, 0
print(numerator / denominator)
