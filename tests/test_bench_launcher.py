"""bench.py's launcher plumbing on CPU (no GPU work, --dry-run): `--gpus N` without
torchrun is one process driving N GPUs (mode "threads"), torchrun is one rank per GPU
(mode "ranks", gloo for the launcher's barrier and max of times). Both must report
n_gpus = N and deal every tile of the frame to exactly one share, with the library's
own share rule (izpi_host_share_tiles)."""
import json
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("n", [1, 3, 8])
def test_gpus_flag_without_torchrun(n):
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--dry-run"], capture_output=True,
                         text=True, timeout=300, cwd="/tmp")
    assert out.returncode == 0, out.stderr
    line = _last_json(out.stdout)
    assert line["n_gpus"] == n and line["mode"] == ("threads" if n > 1 else "single")
    assert line["tiles_covered"] == line["tiles"] == 1024
    assert line["max_share_tiles"] == -(-1024 // n)


def test_torchrun_two_ranks():
    port = _free_port()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                          "--gpus", "2", "--dry-run"], capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-2000:]
    line = _last_json(out.stdout)
    assert line["n_gpus"] == 2 and line["mode"] == "ranks"
    assert line["tiles_covered"] == 1024


def test_torchrun_world_must_match_gpus():
    port = _free_port()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                          "--gpus", "4", "--dry-run"], capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert out.returncode != 0


def test_share_rule_partitions_frame():
    """izpi_host_share_tiles: shares are disjoint, cover the frame, keep spiral order."""
    from izpi_amd import sharding
    from izpi_amd.renderer import common_tiles
    tiles = common_tiles(1920, 1080)
    for n in (1, 2, 3, 7, 8):
        parts = [sharding.shard_tiles(tiles, r, n) for r in range(n)]
        assert sum(len(p) for p in parts) == len(tiles)
        for r, p in enumerate(parts):
            assert np.array_equal(p, tiles[r::n])
