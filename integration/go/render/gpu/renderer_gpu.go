//go:build izpi_gpu

// Package gpu is the drop-in MI355X renderer for izpi (SURVEY.md §8(f) row 1).
//
// It implements render.Renderer (internal/render/renderer.go:26-28) on top of the C ABI
// of libizpi_gpu.so (include/izpi_gpu.h, include/izpi_host.h). Copy this directory to
// internal/render/gpu/ in the izpi tree, put the library and headers under
// third_party/izpi_amd/{lib,include}, and build with -tags izpi_gpu.
//
// The scene crosses the boundary as the transport.Scene protobuf the leader already
// holds (leader.go:43-112): proto.Marshal on the Go side, izpi_scene_parse_binary and
// izpi_scene_to_input (transport.ToScene's rules restated in C++) on the other. Image
// textures are decoded by Go (texture.NewFromFile, leader.go:84-98) and handed over as
// float64 texels; streamed triangles are appended to the marshalled scene. Nothing here
// is compiled in this repository (no Go toolchain); it is written against the
// reference's exported API and the C headers.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../third_party/izpi_amd/include
#cgo LDFLAGS: -L${SRCDIR}/../../../third_party/izpi_amd/lib -lizpi_gpu -Wl,-rpath,${SRCDIR}/../../../third_party/izpi_amd/lib
#include <stdlib.h>
#include "izpi_gpu.h"
#include "izpi_host.h"
*/
import "C"

import (
	"context"
	"errors"
	"fmt"
	"image"
	"image/color"
	"time"
	"unsafe"

	"github.com/flynn-nrg/floatimage/floatimage"
	pb_transport "github.com/flynn-nrg/izpi/internal/proto/transport"
	"github.com/flynn-nrg/izpi/internal/render"
	"github.com/flynn-nrg/izpi/internal/sampler"
	"github.com/flynn-nrg/izpi/internal/texture"
	"google.golang.org/protobuf/proto"

	pb "github.com/cheggaaa/pb/v3"
	log "github.com/sirupsen/logrus"
)

// Ensure interface compliance (renderer.go:26-28).
var _ render.Renderer = (*Renderer)(nil)

// BVH selects the acceleration structure.
type BVH int

const (
	// BVHGPU (the default) builds a PLOC BVH4 with a surface-area collapse on the GPU (≈20 ms).
	// C3 traverses 8.5 nodes per ray on it against 34 on the reference tree. The image equals
	// the reference tree's except where two primitives are hit at exactly the same distance
	// (equal-t tie-breaks, A11) or a box is culled at tMax by float rounding: bitwise equal on
	// C1-C5 (INTEGRATION.md).
	BVHGPU BVH = iota
	// BVHReference rebuilds hitable.NewBVH4's tree bit for bit on the host (≈0.6 s for 800k
	// triangles): the traversal order, and so every tie-break, of izpi's own tree.
	BVHReference
)

// Accumulation selects how a sample's radiance is summed (izpi_render_req.accumulation).
type Accumulation int

const (
	// AccumulationForward (the default) carries each path's throughput forward: the same
	// paths and random draws, the recursion's result within the north star's pixel RMSE
	// < 1e-6 (rounding only), no per-bounce records (a smaller, faster workspace).
	AccumulationForward Accumulation = iota
	// AccumulationRecursive unwinds colour.go:44-57 / sampler/spectral.go:60-72 in its own
	// operation order: bit-identical to the CPU restatement.
	AccumulationRecursive
)

// Options are the render.New parameters (renderer.go:73-104) the GPU path uses, plus the device.
type Options struct {
	SizeX, SizeY, NumSamples, MaxDepth int
	Background                         [3]float64    // colours.Black in leader mode (leader.go:140)
	SpectralBackground                 []float64     // 75 values at the CIE wavelengths, nil = black
	SamplerType                        sampler.SamplerType
	Device                             int
	Devices                            []int         // >1 entries: one Render fans out over these GPUs (izpi_gpu_multi_*)
	Seed                               uint64        // master seed of the per-sample LCG streams
	BVH                                BVH
	Accumulation                       Accumulation
	PNGPipeline                        bool          // Gamma + Clamp(1.0) on the GPU (leader.go:179-182)
	Verbose                            bool          // progress bar while a frame renders (renderer.go:119-121)
}

// Renderer renders one frame per Render call on one MI355X (or several, Options.Devices).
//
// cgo pointer rules: every request passed to C is a Go value that holds C pointers only.
// The spectral background and tile lists live in C.malloc memory, because Go memory
// passed to C (the request) may not hold Go pointers.
type Renderer struct {
	ctx   *C.izpi_ctx   // single device, or device 0's context of m
	m     *C.izpi_multi // multi-GPU form (Options.Devices), nil otherwise
	ps    *C.izpi_proto_scene
	host  *C.izpi_host_scene
	req   C.izpi_render_req
	bg    *C.double // C.malloc: [75] wavelengths then [75] values of the spectral background, or nil
	sizeX   int
	sizeY   int
	ndev    int    // contexts of the render (1, or len(Options.Devices))
	verbose bool   // progress bar (Options.Verbose)
	numRays uint64 // rays of the last Render (RendererImpl.numRays, renderer.go:213)
}

// Tile is one workUnit rectangle with inclusive bounds (renderer.go:56-70), as a
// RenderTileRequest carries it (worker/render.go:18-21).
type Tile struct{ X0, Y0, X1, Y1 int }

func lastHostError() error { return errors.New(C.GoString(C.izpi_host_last_error())) }

func (r *Renderer) deviceError(what string, rc C.int) error {
	if r.m != nil && what != "izpi_gpu_build_bvh4" {
		return fmt.Errorf("%s: status %d: %s", what, int(rc), C.GoString(C.izpi_gpu_multi_last_error(r.m)))
	}
	return fmt.Errorf("%s: status %d: %s", what, int(rc), C.GoString(C.izpi_gpu_last_error(r.ctx)))
}

// New mirrors render.New for the leader: protoScene as read from the .pbtxt/.izpi file,
// textures as loaded by the leader (filename -> ImageTxt), streamed triangles if any.
func New(protoScene *pb_transport.Scene, textures map[string]*texture.ImageTxt,
	streamed []*pb_transport.Triangle, opt Options) (*Renderer, error) {
	r := &Renderer{sizeX: opt.SizeX, sizeY: opt.SizeY, ndev: 1, verbose: opt.Verbose}
	ok := false
	defer func() {
		if !ok {
			r.Close()
		}
	}()
	// 1. the scene, in the wire format the C++ ingestion reads
	scene := proto.Clone(protoScene).(*pb_transport.Scene)
	if len(streamed) > 0 {
		if scene.Objects == nil {
			scene.Objects = &pb_transport.SceneObjects{}
		}
		// streamed triangles are embedded after the file's own (transport.go:568-583)
		scene.Objects.Triangles = append(scene.Objects.Triangles, streamed...)
	}
	buf, err := proto.Marshal(scene)
	if err != nil {
		return nil, err
	}
	if len(buf) == 0 {
		return nil, errors.New("empty scene")
	}
	if rc := C.izpi_scene_parse_binary(unsafe.Pointer(&buf[0]), C.uint64_t(len(buf)), &r.ps); rc != 0 {
		return nil, lastHostError()
	}
	// 2. image textures as float64 NRGBA texels, row 0 = image top, with ImageTxt.Value's
	//    conversion for 8-bit images (image.go:91-100)
	for name, it := range textures {
		texels := toFloat64NRGBA(it.GetData())
		b := it.GetData().Bounds()
		cname := C.CString(name)
		rc := C.izpi_scene_set_image(r.ps, cname, C.uint32_t(b.Dx()), C.uint32_t(b.Dy()), (*C.double)(unsafe.Pointer(&texels[0])))
		C.free(unsafe.Pointer(cname))
		if rc != 0 {
			return nil, lastHostError()
		}
	}
	// 3. transport.ToScene up to the BVH, leader mode aspect W/H (transport.go:522-529)
	var in *C.izpi_scene_input
	if rc := C.izpi_scene_to_input(r.ps, C.double(float64(opt.SizeX)/float64(opt.SizeY)), 12345, &in); rc != 0 {
		return nil, lastHostError()
	}
	flags := C.uint32_t(0)
	if opt.BVH == BVHGPU {
		flags = C.IZPI_HOST_SKIP_BVH
	}
	if rc := C.izpi_host_build_scene_ex(in, flags, &r.host); rc != 0 {
		return nil, lastHostError()
	}
	if len(opt.Devices) > 1 {
		// renderer.go:123-147 starts a worker per core; here one host thread per GPU inside the library
		devs := make([]C.int, len(opt.Devices))
		for i, d := range opt.Devices {
			devs[i] = C.int(d)
		}
		if rc := C.izpi_gpu_multi_open(&devs[0], C.uint32_t(len(devs)), &r.m); rc != 0 {
			return nil, fmt.Errorf("izpi_gpu_multi_open(%v): status %d", opt.Devices, int(rc))
		}
		r.ctx = C.izpi_gpu_multi_context(r.m, 0) // owned by r.m
		r.ndev = len(opt.Devices)
	} else if rc := C.izpi_gpu_open(C.int(opt.Device), &r.ctx); rc != 0 {
		return nil, fmt.Errorf("izpi_gpu_open(%d): status %d", opt.Device, int(rc))
	}
	// 4. optional GPU BVH4 build, then the upload
	if opt.BVH == BVHGPU {
		desc := C.izpi_host_scene_desc(r.host)
		n := int(desc.num_tris + desc.num_spheres)
		boxes := make([]float64, 6*n)
		nodes := make([]C.izpi_bvh4_node, 2*n)
		order := make([]uint32, n)
		var numNodes C.uint32_t
		var ms C.double
		if n > 0 {
			C.izpi_host_scene_prim_boxes(r.host, (*C.double)(unsafe.Pointer(&boxes[0])))
			if rc := C.izpi_gpu_build_bvh4(r.ctx, (*C.double)(unsafe.Pointer(&boxes[0])), C.uint32_t(n), C.izpi_host_bvh_leaf_max(desc), C.IZPI_BVH_PLOC|C.IZPI_BVH_SAH,
				&nodes[0], C.uint32_t(len(nodes)), &numNodes, (*C.uint32_t)(unsafe.Pointer(&order[0])), &ms); rc != 0 {
				return nil, r.deviceError("izpi_gpu_build_bvh4", rc)
			}
			if rc := C.izpi_host_scene_set_bvh(r.host, &nodes[0], numNodes, (*C.uint32_t)(unsafe.Pointer(&order[0]))); rc != 0 {
				return nil, lastHostError()
			}
		}
	}
	if r.m != nil {
		if rc := C.izpi_gpu_multi_upload_scene(r.m, C.izpi_host_scene_desc(r.host)); rc != 0 {
			return nil, r.deviceError("izpi_gpu_multi_upload_scene", rc)
		}
	} else if rc := C.izpi_gpu_upload_scene(r.ctx, C.izpi_host_scene_desc(r.host)); rc != 0 {
		return nil, r.deviceError("izpi_gpu_upload_scene", rc)
	}
	// 5. the request: whole frame, Render's post-processing (renderer.go:215-219)
	desc := C.izpi_host_scene_desc(r.host)
	r.req.abi_version = C.IZPI_ABI_VERSION
	r.req.width, r.req.height = C.uint32_t(opt.SizeX), C.uint32_t(opt.SizeY)
	r.req.spp, r.req.max_depth = C.uint32_t(opt.NumSamples), C.uint32_t(opt.MaxDepth)
	r.req.out_layout = C.IZPI_OUT_CANVAS
	r.req.seed = C.uint64_t(opt.Seed)
	r.req.exposure = desc.camera.exposure // Scene.Exposure = camera exposure
	r.req.accumulation = C.IZPI_ACC_FORWARD
	if opt.Accumulation == AccumulationRecursive {
		r.req.accumulation = C.IZPI_ACC_RECURSIVE
	}
	for i := 0; i < 3; i++ {
		r.req.background[i] = C.double(opt.Background[i])
	}
	post := C.uint32_t(C.IZPI_POST_NONE)
	r.req.sampler = C.IZPI_SAMPLER_COLOUR
	if opt.SamplerType == sampler.SpectralSampler {
		r.req.sampler = C.IZPI_SAMPLER_SPECTRAL
		post |= C.IZPI_POST_SPECTRAL // FireflyRejection + XYZToRGB
		if len(opt.SpectralBackground) == 75 { // e.g. colours.SpectralBlack in leader mode (leader.go:142)
			r.bg = (*C.double)(C.malloc(C.size_t(2 * 75 * 8)))
			bg := unsafe.Slice((*float64)(unsafe.Pointer(r.bg)), 2*75)
			for i := 0; i < 75; i++ {
				bg[i] = 380 + 5*float64(i) // the CIE wavelengths of the 75 values
				bg[75+i] = opt.SpectralBackground[i]
			}
			r.req.num_bg_spd = 75
			r.req.bg_spd_wavelengths = r.bg
			r.req.bg_spd_values = (*C.double)(unsafe.Add(unsafe.Pointer(r.bg), 75*8))
		}
	}
	if opt.PNGPipeline {
		post |= C.IZPI_POST_GAMMA_CLAMP
	}
	r.req.post = post
	// 6. render.New's share of the work (renderer.go:73-104): the request's workspace sized,
	// allocated and first touched now, so that the first Render allocates nothing
	prep := r.req // C pointers only
	if r.m != nil {
		if rc := C.izpi_gpu_multi_prepare(r.m, &prep); rc != 0 {
			return nil, r.deviceError("izpi_gpu_multi_prepare", rc)
		}
	} else if rc := C.izpi_gpu_prepare(r.ctx, &prep); rc != 0 {
		return nil, r.deviceError("izpi_gpu_prepare", rc)
	}
	ok = true
	return r, nil
}

// Render mirrors RendererImpl.Render (renderer.go:108-222): the whole frame in one call,
// with the reference's begin / completion log lines (the ray count is the library's
// Sampler-call count, colour.go:38) and, when verbose, a progress bar fed by
// izpi_gpu_progress while the call runs (the reference counts tiles, renderer.go:119-121;
// this one counts samples).
func (r *Renderer) Render(ctx context.Context) image.Image {
	pix := make([]float64, r.sizeX*r.sizeY*4) // floatimage.NewFloat64NRGBA backing store (renderer.go:88)
	req := r.req                              // C pointers only
	st := make([]C.izpi_render_stats, r.ndev) // one per context of the fan-out
	log.Infof("Begin rendering on %v MI355X context(s)", r.ndev)
	startTime := time.Now()
	done := make(chan struct{})
	polled := make(chan struct{})
	go r.progress(done, polled)
	var rc C.int
	if r.m != nil {
		rc = C.izpi_gpu_multi_render(r.m, &req, (*C.double)(unsafe.Pointer(&pix[0])), &st[0])
	} else {
		rc = C.izpi_gpu_render(r.ctx, &req, (*C.double)(unsafe.Pointer(&pix[0])), &st[0])
	}
	close(done)
	<-polled
	if rc != 0 {
		what := "izpi_gpu_render"
		if r.m != nil {
			what = "izpi_gpu_multi_render"
		}
		log.Fatalf("%v", r.deviceError(what, rc)) // the reference log.Fatals on render errors
	}
	r.numRays = 0
	for i := range st {
		r.numRays += uint64(st[i].rays)
	}
	log.Infof("Rendering completed in %v using %v rays", time.Since(startTime), r.numRays)
	return floatimage.NewFloat64NRGBA(image.Rect(0, 0, r.sizeX, r.sizeY), pix)
}

// NumRays is the ray count of the last Render (the figure of its completion log line).
func (r *Renderer) NumRays() uint64 { return r.numRays }

// progress polls the running render's finished samples every 200 ms into a progress bar
// (verbose only) until done is closed, then closes polled.
func (r *Renderer) progress(done <-chan struct{}, polled chan<- struct{}) {
	defer close(polled)
	if !r.verbose {
		<-done
		return
	}
	var d, t C.uint64_t
	poll := func() {
		if r.m != nil {
			C.izpi_gpu_multi_progress(r.m, &d, &t)
		} else {
			C.izpi_gpu_progress(r.ctx, &d, &t)
		}
	}
	bar := pb.Start64(int64(r.sizeX) * int64(r.sizeY) * int64(r.req.spp))
	tick := time.NewTicker(200 * time.Millisecond)
	defer tick.Stop()
	for {
		select {
		case <-done:
			poll()
			bar.SetCurrent(int64(d))
			bar.Finish()
			return
		case <-tick.C:
			poll()
			bar.SetCurrent(int64(d))
		}
	}
}

// RenderTiles is the worker's RenderTile (worker/render.go:17-75) for a batch of
// equal-sized tiles in one device call. Per tile it returns (Y1-Y0+1) rows of (X1-X0+1)*4
// float64 — R,G,B (CIE X,Y,Z for the spectral sampler) and alpha 1 — row Y0 first: the
// Pixels of the RenderTileResponse sequence the worker streams (Width = X1-X0+1,
// Height = 1, PosY = y), with no post-processing, as in the worker. Tiles of different
// sizes go in separate calls.
func (r *Renderer) RenderTiles(tiles []Tile) ([][]float64, error) {
	if len(tiles) == 0 {
		return nil, nil
	}
	ct := (*C.uint32_t)(C.malloc(C.size_t(16 * len(tiles))))
	defer C.free(unsafe.Pointer(ct))
	t := unsafe.Slice((*uint32)(unsafe.Pointer(ct)), 4*len(tiles))
	for i, tl := range tiles {
		if tl.X0 < 0 || tl.Y0 < 0 || tl.X1 < tl.X0 || tl.Y1 < tl.Y0 {
			return nil, fmt.Errorf("bad tile %+v", tl)
		}
		t[4*i], t[4*i+1], t[4*i+2], t[4*i+3] = uint32(tl.X0), uint32(tl.Y0), uint32(tl.X1), uint32(tl.Y1)
	}
	req := r.req // C pointers only
	req.num_tiles = C.uint32_t(len(tiles))
	req.tiles = ct
	req.out_layout = C.IZPI_OUT_PACKED
	req.post = C.IZPI_POST_NONE
	packed := make([]float64, int(C.izpi_gpu_output_bytes(&req))/8)
	var st C.izpi_render_stats
	// on a multi-GPU renderer the batch runs on device 0 (r.ctx)
	if rc := C.izpi_gpu_render(r.ctx, &req, (*C.double)(unsafe.Pointer(&packed[0])), &st); rc != 0 {
		return nil, fmt.Errorf("izpi_gpu_render (tiles): status %d: %s", int(rc), C.GoString(C.izpi_gpu_last_error(r.ctx)))
	}
	out := make([][]float64, len(tiles))
	off := 0
	for i, tl := range tiles {
		n := (tl.X1 - tl.X0 + 1) * (tl.Y1 - tl.Y0 + 1) * 4
		out[i] = packed[off : off+n : off+n]
		off += n
	}
	return out, nil
}

// Close releases the device context and the host-side scene.
func (r *Renderer) Close() {
	if r.m != nil {
		C.izpi_gpu_multi_close(r.m) // closes device 0's context too
		r.m, r.ctx = nil, nil
	}
	if r.ctx != nil {
		C.izpi_gpu_close(r.ctx)
		r.ctx = nil
	}
	if r.host != nil {
		C.izpi_host_scene_free(r.host)
		r.host = nil
	}
	if r.ps != nil {
		C.izpi_scene_free(r.ps)
		r.ps = nil
	}
	if r.bg != nil {
		r.req.num_bg_spd, r.req.bg_spd_wavelengths, r.req.bg_spd_values = 0, nil, nil
		C.free(unsafe.Pointer(r.bg))
		r.bg = nil
	}
}

// toFloat64NRGBA returns W*H*4 float64 texels, row 0 = image top. Float64NRGBA images are
// copied as they are; other images go through color.NRGBAModel and /255, which is what
// ImageTxt.Value does per lookup (image.go:91-100; alpha is not read by the path).
func toFloat64NRGBA(img image.Image) []float64 {
	b := img.Bounds()
	out := make([]float64, 0, b.Dx()*b.Dy()*4)
	if f, ok := img.(*floatimage.Float64NRGBA); ok {
		for y := b.Min.Y; y < b.Max.Y; y++ {
			for x := b.Min.X; x < b.Max.X; x++ {
				p := f.Float64NRGBAAt(x, y)
				out = append(out, p.R, p.G, p.B, p.A)
			}
		}
		return out
	}
	for y := b.Min.Y; y < b.Max.Y; y++ {
		for x := b.Min.X; x < b.Max.X; x++ {
			p := color.NRGBAModel.Convert(img.At(x, y)).(color.NRGBA)
			out = append(out, float64(p.R)/255.0, float64(p.G)/255.0, float64(p.B)/255.0, float64(p.A)/255.0)
		}
	}
	return out
}
