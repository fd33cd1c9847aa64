"""Multi-rank path on CPU (gloo, world_size 2 and 3): the library's own share rule
(izpi_host_share_tiles), padded block size (izpi_host_share_block) and root assembly
(izpi_host_assemble_shares, the host twin of the device's k_unpack step in
izpi_gpu_render_rank), with the blocks moved by a gloo gather and fed by oracle renders of
each rank's tiles. The assembled canvas must be bit-identical to a single-rank render:
per pixel-sample RNG streams make the image partition-independent; a
Python restatement of the unpack rule cross-checks the library's."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

W = H = 64
SPP = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_render(tiles):
    import ctypes as C
    from izpi_amd import _native as N
    from izpi_amd import configs
    from oracle import oracle as O
    o = O.OracleScene(configs.cornell_rgb(1.0), aspect_override=1.0)
    req = N.RenderReq(width=W, height=H, spp=SPP, max_depth=50, sampler=N.SAMPLER_COLOUR, seed=12345)
    t = np.ascontiguousarray(tiles, np.uint32)
    req.num_tiles = len(t)
    req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
    canvas, _ = o.render(req, threads=2)
    return canvas.reshape(H, W, 4)


def _worker(rank, world, port, outdir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from izpi_amd import sharding
    from oracle import oracle as O
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    all_tiles = O.tiles(W, H)
    mine = sharding.shard_tiles(all_tiles, rank, world)
    packed = np.zeros(sharding.packed_len(all_tiles, world))
    if len(mine):
        part = sharding.pack_from_canvas(_oracle_render(mine), mine, H)
        packed[:part.size] = part
    got = sharding.gather_packed(torch.from_numpy(packed), rank, world)
    if rank == 0:
        blocks = np.concatenate([g.numpy() for g in got])
        canvas = sharding.assemble(all_tiles, world, blocks, W, H)
        check = np.zeros((H, W, 4))
        for r in range(world):
            rt = sharding.shard_tiles(all_tiles, r, world)
            if len(rt):
                sharding.unpack_into(check, rt, got[r].numpy()[:sharding.tile_pixels(rt) * 4], W, H)
        assert canvas.tobytes() == check.tobytes()
        np.save(os.path.join(outdir, "canvas_%d.npy" % world), canvas)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_is_partition_independent(tmp_path, world):
    from oracle import oracle as O
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / ("canvas_%d.npy" % world))
    full = _oracle_render(O.tiles(W, H))
    assert got.tobytes() == full.tobytes()
    assert np.all(full[0] == 0) and np.all(full[1:, :, 3] == 1.0)
