# Long-running CPU work (exponential recursion); useful as a timeout probe.
def fib(n):
    return n if n < 2 else fib(n - 1) + fib(n - 2)


for i in range(40):
    print(i, fib(i))
