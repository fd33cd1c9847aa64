"""GPURenderer — the drop-in for izpi's render.Renderer (internal/render/renderer.go:26-28).

``GPURenderer(scene, W, H, spp, max_depth, ...)`` mirrors ``render.New`` (renderer.go:73-104)
and ``.render()`` mirrors ``Render(ctx) image.Image`` (renderer.go:108-222): it returns the
float64 NRGBA canvas (H, W, 4) the Go renderer fills — RGB for the Colour sampler, CIE XYZ
before post-processing for the Spectral sampler (``.render_spectral_rgb()`` applies
FireflyRejection + XYZToRGB on the GPU like renderer.go:216-219).

Multi-GPU (one process per GPU, torch.distributed over RCCL): tiles are dealt
round-robin (tile_id % world == rank), each rank renders its tiles into a packed
device buffer, and one ``gather`` moves them to rank 0, which scatters them into the
canvas on its GPU (izpi_gpu_unpack_tiles). Per pixel-sample RNG streams make the image
independent of the partition.
"""
import ctypes as C
import os

import numpy as np

from . import _native as N
from .scene import HostScene


# primitives per leaf of the GPU-built tree (the reference allows up to 4, bvh4.go:638)
GPU_BVH_METHOD = N.BVH_PLOC
GPU_BVH_LEAF_MAX = 3  # measured on C3: 3 -> 1146, 2 -> 1137, 4 -> 1065 Msamples/s


def _check(rc, ctx, what):
    if rc != 0:
        msg = N.lib().izpi_gpu_last_error(ctx).decode() if ctx else ""
        raise RuntimeError("%s failed (status %d): %s" % (what, rc, msg))


def common_tiles(width, height):
    """common.Tiles + grid.WalkGrid spiral order, as an (n, 4) uint32 array."""
    buf = (C.c_uint32 * (4 * (width * height // 16 + 16)))()
    n = N.lib().izpi_host_tiles(width, height, buf, len(buf) // 4)
    if n == 0:
        raise ValueError("%dx%d is not divisible by any common.Tiles step" % (width, height))
    return np.frombuffer(buf, np.uint32, count=4 * n).reshape(n, 4).copy()


class GPURenderer:
    def __init__(self, scene, width, height, spp, max_depth=50, sampler=N.SAMPLER_COLOUR, background=(0.0, 0.0, 0.0),
                 spectral_background=None, device=0, seed=12345, bvh_seed=12345, host_scene=None, bvh="reference",
                 bvh_leaf_max=None):
        """bvh="reference": hitable.NewBVH4's tree, rebuilt bit for bit on the host (the
        parity default); bvh="gpu": the GPU linear BVH4 builder (izpi_gpu_build_bvh4),
        same node format, different topology."""
        if bvh not in ("reference", "gpu"):
            raise ValueError("bvh must be 'reference' or 'gpu'")
        self.width, self.height, self.spp, self.max_depth = int(width), int(height), int(spp), int(max_depth)
        self.sampler = int(sampler)
        self.background = tuple(float(b) for b in background)
        self.seed = int(seed)
        self.device = int(device)
        # leader mode: aspect = W/H overrides the scene camera (transport.go aspectOverride)
        self.host = host_scene or HostScene(scene, aspect_override=float(width) / float(height), bvh_seed=bvh_seed,
                                            skip_bvh=bvh == "gpu")
        if spectral_background is None:
            self._bg_wl = np.zeros(0)
            self._bg_val = np.zeros(0)
        else:
            wl, val = spectral_background
            self._bg_wl = np.ascontiguousarray(wl, np.float64)
            self._bg_val = np.ascontiguousarray(val, np.float64)
        L = N.lib()
        ctx = C.c_void_p()
        rc = L.izpi_gpu_open(self.device, C.byref(ctx))
        if rc != 0:
            raise RuntimeError("izpi_gpu_open(%d) failed: no HIP device?" % self.device)
        self.ctx = ctx
        self.bvh_build_ms = None
        if bvh == "gpu" and host_scene is None:
            nodes, order, self.bvh_build_ms = self.build_bvh4(self.host.prim_boxes(),
                                                              bvh_leaf_max or GPU_BVH_LEAF_MAX)
            self.host.set_bvh(nodes, order)
        _check(L.izpi_gpu_upload_scene(ctx, C.byref(self.host.desc)), ctx, "izpi_gpu_upload_scene")
        self.stats = None

    def build_bvh4(self, boxes, leaf_max=4, method=None):
        """izpi_gpu_build_bvh4 over [n][6] f64 boxes: (nodes (m, 128) uint8, order, ms)."""
        if method is None:  # IZPI_BVH_METHOD=lbvh|ploc overrides the default (experiments)
            method = {"lbvh": N.BVH_LBVH, "ploc": N.BVH_PLOC}.get(os.environ.get("IZPI_BVH_METHOD", ""), GPU_BVH_METHOD)
        boxes = np.ascontiguousarray(boxes, np.float64).reshape(-1, 6)
        n = len(boxes)
        nodes = np.zeros((max(1, 2 * n), 128), np.uint8)
        order = np.zeros(max(1, n), np.uint32)
        m = C.c_uint32()
        ms = C.c_double()
        _check(N.lib().izpi_gpu_build_bvh4(self.ctx, boxes.ctypes.data_as(N.c_double_p), n, leaf_max, method,
                                            nodes.ctypes.data_as(C.POINTER(N.BVH4Node)), len(nodes), C.byref(m),
                                            order.ctypes.data_as(N.c_uint32_p), C.byref(ms)),
               self.ctx, "izpi_gpu_build_bvh4")
        return nodes[:m.value].copy(), order[:n].copy(), ms.value

    # -------------------------------------------------------------- request
    def request(self, tiles=None, layout=N.OUT_CANVAS, spp=None, post=N.POST_NONE):
        req = N.RenderReq()
        req.post = post
        req.exposure = self.exposure
        req.width, req.height = self.width, self.height
        req.spp = self.spp if spp is None else int(spp)
        req.max_depth = self.max_depth
        req.sampler = self.sampler
        req.out_layout = layout
        req.background[:] = self.background
        req.seed = self.seed
        keep = []
        if tiles is not None:
            t = np.ascontiguousarray(tiles, np.uint32).reshape(-1, 4)
            keep.append(t)
            req.num_tiles = len(t)
            req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
        if self._bg_wl.size:
            req.num_bg_spd = self._bg_wl.size
            req.bg_spd_wavelengths = self._bg_wl.ctypes.data_as(C.POINTER(C.c_double))
            req.bg_spd_values = self._bg_val.ctypes.data_as(C.POINTER(C.c_double))
        req._keep = keep
        return req

    # --------------------------------------------------------------- render
    @property
    def exposure(self):
        return float(self.host.desc.camera.exposure)  # Scene.Exposure = camera exposure (scene.go:30)

    def render(self, tiles=None, canvas=None, spp=None, post=N.POST_NONE):
        """Render.Render(): returns the (H, W, 4) float64 canvas (host memory). With
        post=POST_SPECTRAL (whole frame only) the XYZ canvas goes through
        FireflyRejection + XYZToRGB on the GPU, as Render does for the Spectral sampler;
        with POST_GAMMA_CLAMP the leader's png pipeline (Gamma, Clamp(1.0)) follows."""
        if canvas is None:
            canvas = np.zeros((self.height, self.width, 4), np.float64)
        req = self.request(tiles, N.OUT_CANVAS, spp, post)
        st = N.RenderStats()
        rc = N.lib().izpi_gpu_render(self.ctx, C.byref(req), canvas.ctypes.data_as(C.POINTER(C.c_double)), C.byref(st))
        _check(rc, self.ctx, "izpi_gpu_render")
        self.stats = st.as_dict()
        return canvas

    def render_spectral_rgb(self):
        """The full reference Render() for the Spectral sampler: XYZ render, then
        FireflyRejection + XYZToRGB (renderer.go:215-219), all on the GPU."""
        return self.render(post=N.POST_SPECTRAL)

    def spectral_post(self, xyz_ptr, rgba_ptr):
        """FireflyRejection + XYZToRGB of a device XYZ canvas into another device canvas."""
        _check(N.lib().izpi_gpu_spectral_post(self.ctx, C.c_void_p(xyz_ptr), C.c_void_p(rgba_ptr), self.width,
                                              self.height, C.c_double(self.exposure)), self.ctx,
               "izpi_gpu_spectral_post")

    def postprocess(self, canvas_ptr, filters):
        """postprocess.Pipeline.Apply on a device canvas, in place: filters is a list of
        (N.FILTER_GAMMA | N.FILTER_CLAMP, param) applied in order (pipeline.go:20-31)."""
        k = np.array([f[0] for f in filters], np.uint32)
        p = np.array([f[1] for f in filters], np.float64)
        _check(N.lib().izpi_gpu_postprocess(self.ctx, C.c_void_p(canvas_ptr), self.width, self.height,
                                            k.ctypes.data_as(N.c_uint32_p), p.ctypes.data_as(N.c_double_p), len(k)),
               self.ctx, "izpi_gpu_postprocess")

    def render_device(self, out_ptr, tiles=None, layout=N.OUT_CANVAS, spp=None):
        """Render into device memory at `out_ptr` (e.g. torch tensor .data_ptr())."""
        req = self.request(tiles, layout, spp)
        st = N.RenderStats()
        rc = N.lib().izpi_gpu_render_device(self.ctx, C.byref(req), C.c_void_p(out_ptr), C.byref(st))
        _check(rc, self.ctx, "izpi_gpu_render_device")
        self.stats = st.as_dict()
        return self.stats

    def output_doubles(self, tiles=None, layout=N.OUT_CANVAS):
        req = self.request(tiles, layout)
        return N.lib().izpi_gpu_output_bytes(C.byref(req)) // 8

    def unpack(self, tiles, packed_ptr, canvas_ptr):
        req = self.request(tiles, N.OUT_PACKED)
        _check(N.lib().izpi_gpu_unpack_tiles(self.ctx, C.byref(req), C.c_void_p(packed_ptr), C.c_void_p(canvas_ptr)),
               self.ctx, "izpi_gpu_unpack_tiles")

    # ------------------------------------------------------------ multi-GPU
    def render_distributed(self, rank, world, group=None, tiles=None, post=N.POST_NONE):
        """Tile-sharded render over `world` ranks; returns the canvas as a torch tensor
        on rank 0 (None elsewhere) and this rank's stats. One RCCL gather. With
        post=POST_SPECTRAL rank 0 applies FireflyRejection + XYZToRGB after the gather."""
        import torch
        from . import sharding
        all_tiles = common_tiles(self.width, self.height) if tiles is None else np.asarray(tiles, np.uint32)
        mine = sharding.shard_tiles(all_tiles, rank, world)
        dev = torch.device("cuda", self.device)
        packed = torch.zeros(sharding.packed_len(all_tiles, world), dtype=torch.float64, device=dev)
        self.stats = None
        if len(mine):
            self.render_device(packed.data_ptr(), tiles=mine, layout=N.OUT_PACKED)
        torch.cuda.synchronize(dev)
        gathered = sharding.gather_packed(packed, rank, world, group)
        if rank != 0:
            return None, self.stats
        canvas = torch.zeros((self.height, self.width, 4), dtype=torch.float64, device=dev)
        for r in range(world):
            rt = sharding.shard_tiles(all_tiles, r, world)
            if len(rt):
                self.unpack(rt, gathered[r].data_ptr(), canvas.data_ptr())
        if post & N.POST_SPECTRAL:
            rgb = torch.empty_like(canvas)
            self.spectral_post(canvas.data_ptr(), rgb.data_ptr())
            canvas = rgb
        if post & N.POST_GAMMA_CLAMP:  # leader.go:179-182
            self.postprocess(canvas.data_ptr(), [(N.FILTER_GAMMA, 0.0), (N.FILTER_CLAMP, 1.0)])
        torch.cuda.synchronize(dev)
        return canvas, self.stats

    def close(self):
        if getattr(self, "ctx", None):
            N.lib().izpi_gpu_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
