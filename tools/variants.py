"""A/B experiments on compile-time variants of the library.

    python tools/variants.py build NAME [-DFOO ...]      # here (CPU): izpi_amd/_lib/variants/NAME/libizpi_gpu.so
    python tools/variants.py run --config C4 --spp 64 --frames 3 [--tune slots=N ...] base NAME ...   # on the GPU box

`base` is the product library. Each variant renders in a fresh child process (same scene,
same request) and prints one JSON line per frame: device time, trace / shade / tail ms and
an image digest, so a variant that must be bit-exact can be checked against `base`.
Timing-only variants (results deliberately wrong) are told apart by their digest.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
VDIR = ROOT / "izpi_amd" / "_lib" / "variants"


def build(name, defines, src=None):
    """Compile the library with extra -D flags (or from another checkout's csrc, e.g. a
    `git worktree` of an older commit) into izpi_amd/_lib/variants/NAME/."""
    from izpi_amd import build as B
    from concurrent.futures import ThreadPoolExecutor
    out = VDIR / name
    out.mkdir(parents=True, exist_ok=True)
    sources = [Path(src) / s.name for s in B.SOURCES] if src else B.SOURCES
    objs = [out / (s.name + ".o") for s in sources]
    cmds = [[B.HIPCC, "--offload-arch=%s" % B.ARCH, *B.COMMON_FLAGS, *defines, "-c", "-o", str(o), str(s)]
            for s, o in zip(sources, objs)]
    with ThreadPoolExecutor(len(cmds)) as ex:
        list(ex.map(lambda c: subprocess.run(c, check=True), cmds))
    subprocess.run([B.HIPCC, "--offload-arch=%s" % B.ARCH, "-shared", "-fPIC", "-o", str(out / "libizpi_gpu.so"),
                    *map(str, objs), *B.LINK], check=True)
    for o in objs:
        o.unlink()
    (out / "defines.txt").write_text(" ".join(defines) + "\n")
    print("built", out / "libizpi_gpu.so", " ".join(defines))


def child(a):
    from izpi_amd import _native as N
    if a.variant != "base":
        N.LIB_PATH = VDIR / a.variant / "libizpi_gpu.so"

        class OlderLib(N.C.CDLL):  # a variant built from an older checkout may lack newer entry points
            def __getattr__(self, name):
                try:
                    return super().__getattr__(name)
                except AttributeError:
                    return N.C.CFUNCTYPE(N.C.c_int)(lambda *args: -1)
        N.C.CDLL = OlderLib
    from izpi_amd import configs
    from izpi_amd.renderer import GPURenderer
    cfg = configs.configs()[a.config]
    spp = a.spp or cfg.spp
    tune = {}
    for kv in a.tune or []:
        k, v = kv.split("=")
        tune[k] = int(v)
    r = GPURenderer(cfg.build(), cfg.width, cfg.height, spp, max_depth=cfg.max_depth, sampler=cfg.sampler, device=0,
                    bvh="gpu", bvh_leaf_max=a.leaf_max, tuning=N.tuning(**tune) if tune else None,
                    accumulation=N.ACC_FORWARD if a.acc == "forward" else N.ACC_RECURSIVE)
    post = N.POST_SPECTRAL if cfg.sampler == N.SAMPLER_SPECTRAL else N.POST_NONE
    for i in range(a.frames):
        img = r.render(post=post)
        st = r.stats
        print(json.dumps({"variant": a.variant, "acc": a.acc, "tune": tune, "leaf_max": a.leaf_max, "config": a.config, "spp": spp, "frame": i,
                          "slots": st["slots"], "chunk_spp": st["chunk_spp"], "workspace_gb": round(st["workspace_bytes"] / 1e9, 1),
                          "device_ms": round(st["total_ms"], 3), "trace_ms": round(st["kernel_ms"], 3),
                          "shade_ms": round(st["shade_ms"], 3), "tail_ms": round(st["tail_ms"], 3),
                          "launches": st["launches"], "rays": st["rays"],
                          "nodes_per_ray": round(st["node_visits"] / max(st["rays"], 1), 3),
                          "tri_per_ray": round(st["tri_tests"] / max(st["rays"], 1), 3),
                          "digest": hashlib.sha1(img.tobytes()).hexdigest()[:16]}), flush=True)
    r.close()


def run(a):
    for v in a.variants:
        cmd = [sys.executable, __file__, "child", "--config", a.config, "--frames", str(a.frames), "--variant", v, "--acc", a.acc]
        if a.spp:
            cmd += ["--spp", str(a.spp)]
        for kv in a.tune or []:
            cmd += ["--tune", kv]
        if a.leaf_max:
            cmd += ["--leaf-max", str(a.leaf_max)]
        rc = subprocess.run(cmd, timeout=a.timeout).returncode
        if rc != 0:
            sys.exit("variant %s: exit %d" % (v, rc))


def main():
    p = argparse.ArgumentParser()
    sub = p.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("build")
    b.add_argument("name")
    b.add_argument("--src", default=None, help="csrc directory of another checkout")
    b.add_argument("defines", nargs="*")
    r = sub.add_parser("run")
    r.add_argument("--config", default="C3")
    r.add_argument("--spp", type=int, default=None)
    r.add_argument("--frames", type=int, default=3)
    r.add_argument("--timeout", type=int, default=300)
    r.add_argument("--tune", action="append", help="izpi_render_tuning field=value (repeatable)")
    r.add_argument("--leaf-max", type=int, default=None, help="primitives per leaf of the GPU-built BVH4")
    r.add_argument("--acc", default="forward", choices=["forward", "recursive"], help="accumulation (the bench's default: forward)")
    r.add_argument("variants", nargs="+")
    c = sub.add_parser("child")
    c.add_argument("--config", default="C3")
    c.add_argument("--spp", type=int, default=None)
    c.add_argument("--frames", type=int, default=3)
    c.add_argument("--variant", default="base")
    c.add_argument("--tune", action="append")
    c.add_argument("--leaf-max", type=int, default=None)
    c.add_argument("--acc", default="forward")
    a, rest = p.parse_known_args()
    if a.cmd == "build":
        build(a.name, a.defines + rest, a.src)
    elif a.cmd == "run":
        run(a)
    else:
        child(a)


if __name__ == "__main__":
    main()
