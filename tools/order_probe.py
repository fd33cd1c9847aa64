"""Shade/trace time of consecutive renderers in one process (run-order effects)."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    cfg = configs.configs()["C3"]
    scene = cfg.build()
    import os
    for spec in sys.argv[1].split(","):
        bvh, _, method = spec.partition(":")  # e.g. gpu:lbvh
        os.environ["IZPI_BVH_METHOD"] = method
        r = GPURenderer(scene, cfg.width, cfg.height, cfg.spp, bvh=bvh)
        for i in range(3):
            t = time.perf_counter()
            r.render()
            st = r.stats
            print(spec, i, "%.1f ms wall, trace %.1f shade %.1f total %.1f" % ((time.perf_counter() - t) * 1e3, st["kernel_ms"],
                                                                          st["shade_ms"], st["total_ms"]), flush=True)
        r.close()


if __name__ == "__main__":
    main()
