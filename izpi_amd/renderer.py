"""GPURenderer — the drop-in for izpi's render.Renderer (internal/render/renderer.go:26-28).

``GPURenderer(scene, W, H, spp, max_depth, ...)`` mirrors ``render.New`` (renderer.go:73-104)
and ``.render()`` mirrors ``Render(ctx) image.Image`` (renderer.go:108-222): it returns the
float64 NRGBA canvas (H, W, 4) the Go renderer fills — RGB for the Colour sampler, CIE XYZ
before post-processing for the Spectral sampler (``.render_spectral_rgb()`` applies
FireflyRejection + XYZToRGB on the GPU like renderer.go:216-219).

Multi-GPU goes through the library (include/izpi_gpu.h): tiles are dealt round-robin
(tile_id % G == i), each device renders its tiles into a packed buffer, and the shares
are gathered to device 0, which scatters them into the canvas. Two forms:

* ``MultiGPURenderer`` — one process drives every GPU (izpi_gpu_multi_*): one host
  thread and stream per device, xGMI peer copies to device 0;
* ``GPURenderer.render_rank`` — one process per GPU (torchrun): the library's own RCCL
  communicator (izpi_gpu_comm_init) and one ncclGather to rank 0.

Per pixel-sample RNG streams make the image independent of the partition.
"""
import ctypes as C

import numpy as np

from . import _native as N
from .scene import HostScene


GPU_BVH_METHOD = N.BVH_PLOC_SAH


def gpu_leaf_max(desc):
    """Primitives per leaf of the GPU-built tree for a scene (izpi_scene_desc), by the
    library's rule (izpi_host_bvh_leaf_max, shared with the Go shim): 3, or 2 when
    spheres are at least a quarter of the primitives. A sphere test (square root and two
    f64 divisions) costs more than a node visit, so sphere-heavy scenes want smaller leaves:
    C5 (10 spheres of 22 primitives) at 32 spp 876.7 -> 851.6 ms per frame with 2 (1: 931),
    C4 (2 of 16) 194.9 -> 196.8 ms, C3 (no spheres) best at 3 (profiles/r3c/c5_leaf.log)."""
    return int(N.lib().izpi_host_bvh_leaf_max(C.byref(desc)))


def _check(rc, ctx, what):
    if rc != 0:
        msg = N.lib().izpi_gpu_last_error(ctx).decode() if ctx else ""
        raise RuntimeError("%s failed (status %d): %s" % (what, rc, msg))


def build_bvh4(ctx, boxes, leaf_max=4, method=None):
    """izpi_gpu_build_bvh4 on context `ctx` over [n][6] f64 boxes: (nodes (m, 128) uint8, order, ms)."""
    if method is None:
        method = GPU_BVH_METHOD
    boxes = np.ascontiguousarray(boxes, np.float64).reshape(-1, 6)
    n = len(boxes)
    nodes = np.zeros((max(1, 2 * n), 128), np.uint8)
    order = np.zeros(max(1, n), np.uint32)
    m = C.c_uint32()
    ms = C.c_double()
    _check(N.lib().izpi_gpu_build_bvh4(ctx, boxes.ctypes.data_as(N.c_double_p), n, leaf_max, method,
                                        nodes.ctypes.data_as(C.POINTER(N.BVH4Node)), len(nodes), C.byref(m),
                                        order.ctypes.data_as(N.c_uint32_p), C.byref(ms)),
           ctx, "izpi_gpu_build_bvh4")
    return nodes[:m.value].copy(), order[:n].copy(), ms.value


def make_request(width, height, spp, max_depth, sampler, background, seed, exposure, bg_spd=None, tiles=None,
                 layout=N.OUT_CANVAS, post=N.POST_NONE, tuning=None, accumulation=N.ACC_RECURSIVE):
    """izpi_render_req for Render (the arrays it points to are kept alive on `req._keep`).
    tuning: an N.RenderTuning (launch settings; None = the library's defaults).
    accumulation: N.ACC_RECURSIVE (bitwise against the oracle's recursion) or N.ACC_FORWARD."""
    req = N.RenderReq()
    req.abi_version = N.IZPI_ABI_VERSION
    req.accumulation = accumulation
    req.post = post
    req.exposure = exposure
    req.width, req.height = width, height
    req.spp = spp
    req.max_depth = max_depth
    req.sampler = sampler
    req.out_layout = layout
    req.background[:] = background
    req.seed = seed
    keep = []
    if tiles is not None:
        t = np.ascontiguousarray(tiles, np.uint32).reshape(-1, 4)
        keep.append(t)
        req.num_tiles = len(t)
        req.tiles = t.ctypes.data_as(C.POINTER(C.c_uint32))
    if bg_spd is not None and len(bg_spd[0]):
        wl, val = bg_spd
        keep += [wl, val]
        req.num_bg_spd = wl.size
        req.bg_spd_wavelengths = wl.ctypes.data_as(C.POINTER(C.c_double))
        req.bg_spd_values = val.ctypes.data_as(C.POINTER(C.c_double))
    if tuning is not None:
        keep.append(tuning)
        req.tuning = C.pointer(tuning)
    req._keep = keep
    return req


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
                 bvh_leaf_max=None, tuning=None, accumulation=N.ACC_RECURSIVE, bvh_quantized=False):
        """bvh="reference": hitable.NewBVH4's tree, rebuilt bit for bit on the host (the
        parity default); bvh="gpu": the GPU linear BVH4 builder (izpi_gpu_build_bvh4),
        same node format, different topology. tuning: an
        N.RenderTuning for every request (None = library defaults). accumulation: how a
        path's radiance is summed (N.ACC_*; the attribute may be changed between frames).
        bvh_quantized: upload the tree with IZPI_SCENE_QUANTIZED_BVH (64-B nodes whose
        decoded boxes contain the exact ones: half the node memory, C3's traversal 5% slower,
        DESIGN.md 3.6); default off."""
        self.tuning = tuning
        self.bvh_quantized = bool(bvh_quantized)
        self.accumulation = int(accumulation)
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
        self.bvh_leaf_max = (bvh_leaf_max or gpu_leaf_max(self.host.desc)) if bvh == "gpu" else None
        if bvh == "gpu" and host_scene is None:
            nodes, order, self.bvh_build_ms = self.build_bvh4(self.host.prim_boxes(),
                                                              self.bvh_leaf_max)
            self.host.set_bvh(nodes, order)
        self.host.set_flags(N.SCENE_QUANTIZED_BVH if self.bvh_quantized else 0)
        _check(L.izpi_gpu_upload_scene(ctx, C.byref(self.host.desc)), ctx, "izpi_gpu_upload_scene")
        self.stats = None

    def use_tree(self, scene, bvh, bvh_seed=12345, bvh_leaf_max=None, bvh_quantized=False):
        """Re-upload `scene` with another BVH (`bvh`, `bvh_quantized` as in __init__) into this
        context. Its render buffers stay and are reused by the next frame of the same request:
        a second renderer would allocate, and leave for the driver to clear, a second workspace."""
        self.bvh_quantized = bool(bvh_quantized)
        if bvh not in ("reference", "gpu"):
            raise ValueError("bvh must be 'reference' or 'gpu'")
        self.host = HostScene(scene, aspect_override=float(self.width) / float(self.height), bvh_seed=bvh_seed,
                              skip_bvh=bvh == "gpu")
        self.bvh_build_ms = None
        self.bvh_leaf_max = (bvh_leaf_max or gpu_leaf_max(self.host.desc)) if bvh == "gpu" else None
        if bvh == "gpu":
            nodes, order, self.bvh_build_ms = self.build_bvh4(self.host.prim_boxes(), self.bvh_leaf_max)
            self.host.set_bvh(nodes, order)
        self.host.set_flags(N.SCENE_QUANTIZED_BVH if self.bvh_quantized else 0)
        _check(N.lib().izpi_gpu_upload_scene(self.ctx, C.byref(self.host.desc)), self.ctx, "izpi_gpu_upload_scene")

    def build_bvh4(self, boxes, leaf_max=4, method=None):
        """izpi_gpu_build_bvh4 over [n][6] f64 boxes: (nodes (m, 128) uint8, order, ms)."""
        return build_bvh4(self.ctx, boxes, leaf_max, method)

    # -------------------------------------------------------------- request
    def request(self, tiles=None, layout=N.OUT_CANVAS, spp=None, post=N.POST_NONE):
        return make_request(self.width, self.height, self.spp if spp is None else int(spp), self.max_depth,
                            self.sampler, self.background, self.seed, self.exposure, (self._bg_wl, self._bg_val),
                            tiles, layout, post, self.tuning, self.accumulation)

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

    def prepare(self, tiles=None, layout=N.OUT_CANVAS, post=N.POST_NONE):
        """izpi_gpu_prepare: allocate the workspace of this renderer's requests ahead of the
        first frame (render.New's canvas allocation, renderer.go:73-104); after comm_init,
        this rank's share of render_rank."""
        req = self.request(tiles, layout, None, post)
        _check(N.lib().izpi_gpu_prepare(self.ctx, C.byref(req)), self.ctx, "izpi_gpu_prepare")

    def progress(self):
        """(samples finished, samples of the request) of the render running on this context,
        readable from another thread while render() runs (izpi_gpu_progress)."""
        d, t = C.c_uint64(), C.c_uint64()
        _check(N.lib().izpi_gpu_progress(self.ctx, C.byref(d), C.byref(t)), self.ctx, "izpi_gpu_progress")
        return d.value, t.value

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

    def render_device(self, out_ptr, tiles=None, layout=N.OUT_CANVAS, spp=None, post=N.POST_NONE):
        """Render into device memory at `out_ptr` (e.g. torch tensor .data_ptr())."""
        req = self.request(tiles, layout, spp, post)
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
    def comm_init(self, world, rank, comm_id):
        """Join the library's RCCL communicator (one process per GPU); comm_id is rank 0's
        izpi_gpu_comm_id bytes, broadcast by the launcher."""
        cid = (C.c_uint8 * N.COMM_ID_BYTES).from_buffer_copy(bytes(comm_id))
        _check(N.lib().izpi_gpu_comm_init(self.ctx, world, rank, cid), self.ctx, "izpi_gpu_comm_init")

    def render_rank(self, out_ptr=None, post=N.POST_NONE, tiles=None):
        """Collective Render over the communicator: this rank's share of the frame, one
        ncclGather, and on rank 0 the assembled canvas written to device memory at
        `out_ptr` (post-processed). Returns this rank's stats."""
        req = self.request(tiles, N.OUT_CANVAS, None, post)
        st = N.RenderStats()
        rc = N.lib().izpi_gpu_render_rank(self.ctx, C.byref(req), C.c_void_p(out_ptr or 0), C.byref(st))
        _check(rc, self.ctx, "izpi_gpu_render_rank")
        self.stats = st.as_dict()
        return self.stats

    def render_distributed(self, rank, world, post=N.POST_NONE):
        """render_rank into a torch canvas on rank 0 (None elsewhere); the communicator
        must be set up (comm_init) when world > 1. Returns (canvas, stats)."""
        import torch
        dev = torch.device("cuda", self.device)
        canvas = torch.zeros((self.height, self.width, 4), dtype=torch.float64, device=dev) if rank == 0 else None
        if world == 1:
            st = self.render_device(canvas.data_ptr(), post=post)
        else:
            st = self.render_rank(canvas.data_ptr() if canvas is not None else None, post)
        return canvas, st

    def bvh_nodes(self):
        """The uploaded tree's BVH4Node records, (n, 128) uint8, with their exact boxes (a
        quantised upload tests the decoded boxes that oracle.quantize_bvh4 restates)."""
        d = self.host.desc
        nodes = np.frombuffer(bytes(C.string_at(C.addressof(d.nodes.contents), 128 * d.num_nodes)), np.uint8).reshape(-1, 128)
        return nodes.copy()

    def close(self):
        if getattr(self, "ctx", None):
            N.lib().izpi_gpu_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiGPURenderer:
    """Render over several GPUs from one process (izpi_gpu_multi_*): the scene is
    replicated on every device, the frame's tiles are dealt tile % G, device 0 gathers
    and assembles the canvas. Same arguments as GPURenderer plus ``devices``."""

    def __init__(self, scene, width, height, spp, devices, max_depth=50, sampler=N.SAMPLER_COLOUR,
                 background=(0.0, 0.0, 0.0), spectral_background=None, seed=12345, bvh_seed=12345, bvh="gpu",
                 bvh_leaf_max=None, tuning=None, accumulation=N.ACC_RECURSIVE, bvh_quantized=False):
        self.tuning = tuning
        self.accumulation = int(accumulation)
        self.bvh_quantized = bool(bvh_quantized)
        if bvh not in ("reference", "gpu"):
            raise ValueError("bvh must be 'reference' or 'gpu'")
        self.width, self.height, self.spp, self.max_depth = int(width), int(height), int(spp), int(max_depth)
        self.sampler = int(sampler)
        self.background = tuple(float(b) for b in background)
        self.seed = int(seed)
        self.devices = [int(d) for d in devices]
        if spectral_background is None:
            self._bg = (np.zeros(0), np.zeros(0))
        else:
            self._bg = tuple(np.ascontiguousarray(x, np.float64) for x in spectral_background)
        self.host = HostScene(scene, aspect_override=float(width) / float(height), bvh_seed=bvh_seed,
                              skip_bvh=bvh == "gpu")
        L = N.lib()
        m = C.c_void_p()
        devs = (C.c_int * len(self.devices))(*self.devices)
        rc = L.izpi_gpu_multi_open(devs, len(self.devices), C.byref(m))
        if rc != 0:
            raise RuntimeError("izpi_gpu_multi_open(%s) failed (status %d)" % (self.devices, rc))
        self.m = m
        self.bvh_build_ms = None
        self.bvh_leaf_max = (bvh_leaf_max or gpu_leaf_max(self.host.desc)) if bvh == "gpu" else None
        if bvh == "gpu":
            nodes, order, self.bvh_build_ms = build_bvh4(L.izpi_gpu_multi_context(m, 0), self.host.prim_boxes(),
                                                         self.bvh_leaf_max)
            self.host.set_bvh(nodes, order)
        self.host.set_flags(N.SCENE_QUANTIZED_BVH if self.bvh_quantized else 0)
        self._check(L.izpi_gpu_multi_upload_scene(m, C.byref(self.host.desc)), "izpi_gpu_multi_upload_scene")
        self.stats = None

    def _check(self, rc, what):
        if rc != 0:
            msg = N.lib().izpi_gpu_multi_last_error(self.m).decode()
            raise RuntimeError("%s failed (status %d): %s" % (what, rc, msg))

    @property
    def exposure(self):
        return float(self.host.desc.camera.exposure)

    def render(self, canvas=None, post=N.POST_NONE, to_host=True):
        """Render.Render over all devices. Returns the (H, W, 4) canvas (host), or None with
        to_host=False (the canvas stays on device 0: the timing form). self.stats is the
        list of per-device stats."""
        req = make_request(self.width, self.height, self.spp, self.max_depth, self.sampler, self.background,
                           self.seed, self.exposure, self._bg, None, N.OUT_CANVAS, post, self.tuning,
                           self.accumulation)
        G = len(self.devices)
        st = (N.RenderStats * G)()
        if to_host and canvas is None:
            canvas = np.zeros((self.height, self.width, 4), np.float64)
        ptr = canvas.ctypes.data_as(C.c_void_p) if to_host else None
        self._check(N.lib().izpi_gpu_multi_render(self.m, C.byref(req), ptr, st), "izpi_gpu_multi_render")
        self.stats = [st[i].as_dict() for i in range(G)]
        return canvas if to_host else None

    def prepare(self, post=N.POST_NONE):
        """izpi_gpu_multi_prepare: every device's workspace for its share, ahead of the first frame."""
        req = make_request(self.width, self.height, self.spp, self.max_depth, self.sampler, self.background,
                           self.seed, self.exposure, self._bg, None, N.OUT_CANVAS, post, self.tuning,
                           self.accumulation)
        self._check(N.lib().izpi_gpu_multi_prepare(self.m, C.byref(req)), "izpi_gpu_multi_prepare")

    def close(self):
        if getattr(self, "m", None):
            N.lib().izpi_gpu_multi_close(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
