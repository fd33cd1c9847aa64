"""Per-step traversal cost vs. dragon mesh size (L2-locality probe), one GPU.

python tools/step_cost.py --spp 64 --n 261,120,40
Prints trace/shade ms, node/prim wave-steps and ns per wave-step for each mesh size.
With a -DIZPI_TRACE_CLOCKS library the per-phase wave cycles are printed on stderr."""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--n", default="261,120,40")
    ap.add_argument("--size", type=int, default=1024)
    a = ap.parse_args()
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    for n in [int(x) for x in a.n.split(",")]:
        scene = configs.cornell_dragon(1.0, n=n)
        r = GPURenderer(scene, a.size, a.size, a.spp)
        r.render()
        r.render()
        st = r.stats
        steps = st["node_steps"] + st["prim_steps"]
        print("n=%d tris=%d trace %.1f ms shade %.1f ms rays %.3g nodes/ray %.1f tris/ray %.1f node_steps %.3g prim_steps %.3g "
              "ns/step(chip) %.3f" % (n, 12 * n * n + 12, st["kernel_ms"], st["shade_ms"], st["rays"],
                                      st["node_visits"] / st["rays"], st["tri_tests"] / st["rays"], st["node_steps"],
                                      st["prim_steps"], st["kernel_ms"] * 1e6 / max(steps, 1)), flush=True)
        r.close()


if __name__ == "__main__":
    main()
