"""Tile sharding across GPUs (one process per GPU) and the framebuffer gather.

renderer.go:172-188 feeds tiles to workers dynamically; here the partition is static
and interleaved — tile i goes to rank i % world — so centre tiles (dragon, glass) are
spread over all ranks. Per pixel-sample RNG streams make every pixel independent of
the partition, so the gathered canvas is bit-identical for any world size.

Each rank packs its tiles contiguously (IZPI_OUT_PACKED: tile after tile, rows of
sample y, 4 doubles per pixel). One collective moves them to rank 0: ``dist.gather``
of equal-sized (padded) packed buffers — over RCCL/xGMI with the "nccl" backend, or
gloo in the CPU tests. Rank 0 scatters them into the canvas (k_unpack on the GPU;
:func:`assemble` = izpi_host_assemble_shares, the library's host twin of it).
"""
import numpy as np


def shard_tiles(all_tiles, rank, world):
    """Tiles of share `rank` of `world`: the library's own rule (izpi_host_share_tiles),
    the one izpi_gpu_multi_render and izpi_gpu_render_rank deal the frame with."""
    import ctypes as C
    from . import _native as N
    t = np.ascontiguousarray(np.asarray(all_tiles, np.uint32).reshape(-1, 4))
    out = np.zeros_like(t)
    n = N.lib().izpi_host_share_tiles(t.ctypes.data_as(N.c_uint32_p), len(t), rank, world,
                                      out.ctypes.data_as(N.c_uint32_p))
    assert n == len(range(rank, len(t), world))
    return np.ascontiguousarray(out[:n])


def tile_pixels(tiles):
    t = np.asarray(tiles, np.int64)
    return int(((t[:, 2] - t[:, 0] + 1) * (t[:, 3] - t[:, 1] + 1)).sum())


def packed_len(all_tiles, world):
    """Doubles per rank's (padded) packed buffer: the library's share block
    (izpi_host_share_block: max tiles per rank * tile pixels * 4)."""
    from . import _native as N
    t = np.asarray(all_tiles, np.int64)
    return int(N.lib().izpi_host_share_block(len(t), int(t[0, 2] - t[0, 0] + 1), int(t[0, 3] - t[0, 1] + 1), world))


def assemble(all_tiles, world, gathered, width, height, canvas=None):
    """Rank 0's assembly of the gathered share blocks (`world` blocks of packed_len
    doubles, in rank order) into the canvas: the library's izpi_host_assemble_shares, the
    host twin of what izpi_gpu_render_rank's root runs on the device (k_unpack)."""
    from . import _native as N
    t = np.ascontiguousarray(np.asarray(all_tiles, np.uint32).reshape(-1, 4))
    g = np.ascontiguousarray(np.asarray(gathered, np.float64).reshape(-1))
    if g.size != world * packed_len(t, world):
        raise ValueError("gathered holds %d doubles, expected %d blocks of %d" % (g.size, world, packed_len(t, world)))
    if canvas is None:
        canvas = np.zeros((height, width, 4), np.float64)
    assert canvas.flags.c_contiguous and canvas.dtype == np.float64 and canvas.size == width * height * 4
    rc = N.lib().izpi_host_assemble_shares(width, height, t.ctypes.data_as(N.c_uint32_p), len(t), world,
                                           g.ctypes.data_as(N.c_double_p), canvas.ctypes.data_as(N.c_double_p))
    if rc != 0:
        raise RuntimeError("izpi_host_assemble_shares: status %d" % rc)
    return canvas


def gather_packed(packed, rank, world, group=None):
    """Gather every rank's packed tensor to rank 0 (list of tensors there, None elsewhere)."""
    import torch.distributed as dist
    if world == 1:
        return [packed]
    out = [packed.new_empty(packed.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, gather_list=out, dst=0, group=group)
    return out


def unpack_into(canvas, tiles, packed, width, height):
    """A Python restatement of k_unpack (packed tile pixels -> canvas rows H - y,
    rgb.go:41), kept as the independent check of izpi_host_assemble_shares."""
    p = 0
    flat = np.asarray(packed).reshape(-1, 4)
    for x0, y0, x1, y1 in np.asarray(tiles, np.int64):
        for y in range(y0, y1 + 1):
            n = x1 - x0 + 1
            row = height - y
            if row < height:
                canvas[row, x0:x1 + 1] = flat[p:p + n]
            p += n
    return canvas


def pack_from_canvas(canvas, tiles, height):
    """Inverse of unpack_into for pixels that have a canvas row (y >= 1); rows dropped
    by the reference (y == 0) are packed as zeros. Used by the CPU tests to turn oracle
    canvases into the packed layout."""
    out = []
    for x0, y0, x1, y1 in np.asarray(tiles, np.int64):
        for y in range(y0, y1 + 1):
            row = height - y
            if row < height:
                out.append(canvas[row, x0:x1 + 1])
            else:
                out.append(np.zeros((x1 - x0 + 1, 4)))
    return np.concatenate(out).reshape(-1)
