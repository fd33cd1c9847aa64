import sys, time
sys.path.insert(0, '.')
from izpi_amd import configs, _native as N
from izpi_amd.renderer import GPURenderer
cfg = configs.configs()["C4"]
scene = cfg.build()
for bvh in ("reference", "gpu", "reference", "gpu"):
    r = GPURenderer(scene, cfg.width, cfg.height, 64, sampler=cfg.sampler, bvh=bvh)
    t = time.perf_counter(); r.render(); dt = time.perf_counter() - t
    s = r.stats
    print(bvh, "%.3f s" % dt, {k: round(s[k], 2) for k in ("kernel_ms", "shade_ms", "tail_ms", "total_ms", "launches", "node_visits", "tri_tests", "sph_tests")}, "stack", r.host.stack_bound, "nodes", r.host.desc.num_nodes)
    r.close()
