# The reference's benchmark-numpy payload (examples/benchmark-numpy.py of
# bee-code-interpreter-fs, minus its license header), unmodified on purpose:
# bench.py --workload numpy_offload sends exactly this source with
# numpy_offload=True, so the numpy.random.rand draw lives on the sandbox's
# MI355X and numpy.sum(numpy.square(...)) dispatches to the beekern kernels
# (ops/numpy_offload.py); without the offload it is plain CPU numpy.

import numpy
import time

def cpu_intensive_computation():
    array_size = 10**8
    large_array = numpy.random.rand(array_size)
    result = numpy.sum(numpy.square(large_array))
    return result

start_time = time.time()
result = cpu_intensive_computation()
end_time = time.time()
print("Result:", result)
print("Execution Time:", end_time - start_time, "seconds")
