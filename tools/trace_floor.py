"""k_trace2's duration against its queue length (the drain passes' floor):
izpi_gpu_trace over n random rays from inside the C3 box, several n, under
`rocprofv3 --kernel-trace --stats`; the kernel trace gives each launch's duration.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/floor -o run -- python tools/trace_floor.py
"""
import ctypes as C
import sys
import numpy as np
sys.path.insert(0, ".")
from izpi_amd import _native as N
from izpi_amd import configs
from izpi_amd.renderer import GPURenderer

cfg = configs.configs()["C3"]
r = GPURenderer(cfg.build(), 16, 16, 1, bvh="gpu")
rng = np.random.default_rng(1)
for n in [1, 64, 1024, 16384, 65536, 262144, 1048576]:
    rays = np.zeros((n, 8))
    rays[:, 0:3] = rng.uniform([5, 5, 5], [95, 95, 95], (n, 3))
    rays[:, 3:6] = rng.normal(size=(n, 3))
    rays[:, 6], rays[:, 7] = 0.001, 1.7976931348623157e308
    out = (N.Hit * n)()
    for rep in range(3):
        assert N.lib().izpi_gpu_trace(r.ctx, rays.ctypes.data_as(C.POINTER(C.c_double)), n, out) == 0
    print("n=%d done" % n, flush=True)
r.close()
