"""Build the native pieces in-tree.

* ``izpi_amd/_lib/libizpi_gpu.so`` — the product: gfx950 HIP kernels + C ABI
  (include/izpi_gpu.h) + the C++ host scene producer (include/izpi_host.h).
(The CPU oracle is test infrastructure and builds from oracle/Makefile.)

It is compiled with ``-ffp-contract=off`` and without fast-math so that every
``a*b+c`` rounds twice on host and device alike (Go on amd64 emits no FMA).
"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "izpi_amd" / "csrc"
LIBDIR = ROOT / "izpi_amd" / "_lib"
LIB = LIBDIR / "libizpi_gpu.so"

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function"]
SOURCES = [CSRC / "trace.hip", CSRC / "shade_colour.hip", CSRC / "shade_colour_fwd.hip", CSRC / "shade_spectral.hip",
           CSRC / "shade_spectral_fwd.hip", CSRC / "izpi_gpu.hip", CSRC / "bvh_build.hip", CSRC / "host_scene.cpp",
           CSRC / "scene_io.cpp"]
DEPS = SOURCES + [CSRC / "izpi_kern.h", CSRC / "shade.h", CSRC / "izpi_dev.h", CSRC / "gomath.h", CSRC / "cie_tables.h", CSRC / "lightsources.h",
                  ROOT / "include" / "izpi_gpu.h", ROOT / "include" / "izpi_host.h", ROOT / "include" / "izpi_types.h", ROOT / "include" / "izpi_gpu_debug.h"]


def _tmp_name(target):
    """A per-process name next to `target`: two processes building at once (pytest beside
    bench.py, ranks of a launcher without torchrun) never write one file; os.replace then
    swaps the finished file in, so readers never see a partial one."""
    return target.with_name("%s.tmp%d" % (target.name, os.getpid()))


def _stale(target, deps):
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


CLI = LIBDIR / "izpi-render"
CLI_SRC = CSRC / "izpi_render.cpp"


def build_cli(force=False, verbose=True):
    """izpi-render: the C++ host (izpi_amd/csrc/izpi_render.cpp) linked to the library."""
    if not force and not _stale(CLI, [CLI_SRC, LIB, ROOT / "include" / "izpi_gpu.h", ROOT / "include" / "izpi_host.h"]):
        return CLI
    tmp = _tmp_name(CLI)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-o", str(tmp), str(CLI_SRC), "-L" + str(LIBDIR),
           "-lizpi_gpu", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, CLI)
    return CLI


LINK = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]  # RCCL: multi-process framebuffer gather


REPLAY = LIBDIR / "go_shim_replay"
REPLAY_SRC = ROOT / "integration" / "c" / "go_shim_replay.c"


def build_replay(force=False, verbose=True):
    """go_shim_replay: the Go shim's C call sequence in C (integration/c), for the tests."""
    if not force and not _stale(REPLAY, [REPLAY_SRC, LIB, ROOT / "include" / "izpi_gpu.h", ROOT / "include" / "izpi_host.h"]):
        return REPLAY
    tmp = _tmp_name(REPLAY)
    cmd = [os.environ.get("CC", "gcc"), "-O2", "-std=c99", "-Wall", "-I" + str(ROOT / "include"), "-o", str(tmp),
           str(REPLAY_SRC), "-L" + str(LIBDIR), "-lizpi_gpu", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, REPLAY)
    return REPLAY


def build_gpu(force=False, verbose=True):
    if not force and not _stale(LIB, DEPS):
        build_cli(force, verbose)
        build_replay(force, verbose)
        return LIB
    LIBDIR.mkdir(parents=True, exist_ok=True)
    objdir = LIBDIR / ("obj.%d" % os.getpid())  # per process: concurrent builds never share an object file
    objdir.mkdir(exist_ok=True)
    # one hipcc per source, in parallel (izpi_gpu.hip dominates), then one link
    from concurrent.futures import ThreadPoolExecutor
    objs = [objdir / (src.name + ".o") for src in SOURCES]
    cmds = [[HIPCC, "--offload-arch=%s" % ARCH, *COMMON_FLAGS, "-c", "-o", str(o), str(src)] for src, o in zip(SOURCES, objs)]
    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    with ThreadPoolExecutor(len(cmds)) as ex:
        list(ex.map(run, cmds))
    tmp = _tmp_name(LIB)
    run([HIPCC, "--offload-arch=%s" % ARCH, "-shared", "-fPIC", "-o", str(tmp), *map(str, objs), *LINK])
    os.replace(tmp, LIB)
    shutil.rmtree(objdir, ignore_errors=True)
    build_cli(True, verbose)
    build_replay(True, verbose)
    return LIB


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    force = "--force" in argv
    build_gpu(force=force)


if __name__ == "__main__":
    main()
