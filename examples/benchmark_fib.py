# CPU big-integer workload (BASELINE config 2 runs it in a GPU-pinned sandbox):
# 1000 iterative Fibonacci(10000) evaluations, self-timed.
import time


def fib_iter(n):
    a, b = 0, 1
    for _ in range(n):
        a, b = b, a + b
    return a


t0 = time.time()
for _ in range(1000):
    value = fib_iter(10000)
print("digits:", len(str(value)))
print(f"Execution Time: {time.time() - t0:.4f} seconds")
