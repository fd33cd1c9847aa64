"""izpi_amd — MI355X-native path-tracing inner loop for izpi (flynn-nrg/izpi).

Product pieces: izpi_amd/csrc (gfx950 HIP kernels + the C ABI of include/izpi_gpu.h,
C++ host scene producer of include/izpi_host.h), and this thin Python host mirror
(scene description, GPURenderer = render.Renderer drop-in, multi-GPU sharding).
"""
from . import _native  # noqa: F401

__all__ = ["_native", "scene", "configs", "renderer", "build"]
