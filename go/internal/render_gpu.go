// render_gpu.go — the Go side of the drop-in boundary: Render on the MI355X path, a cgo binding of
// librtx.so (include/rtx.h) for TwFlem/raytracer-go.
//
// A maintainer copies this file into the reference's package `internal` (next to
// internal/camera.go; the Hittable/Material/Texture fields it flattens are unexported, so it
// must live in that package), adds the three-line hook at the top of Render (INTEGRATION.md:
// `if done, err := c.renderGPU(world, writer); done { return err }`) and points cgo at a build of
// this repository (`make -C raytracer-go_amd`) through the environment, wherever it is checked out:
//   CGO_CFLAGS="-I$RTX/include" CGO_LDFLAGS="-L$RTX/raytracer-go_amd -Wl,-rpath,$RTX/raytracer-go_amd" go build
// ($RTX = this repository's root).  main.go then changes only its camera options:
//   internal.NewCamera(16.0/9.0, 1920, ..., internal.WithGPUs(1), internal.WithSeed(2024))
// (or RTX_GPUS=1 in the environment, with no change at all), and, to build a World of spheres'
// BVH on the GPU instead of NewBVHFromWorld's host recursion (bvh.go:138-185; 100k spheres),
// internal.NewBVHFromWorldGPU(world) in place of internal.NewBVHFromWorld(world).
// Render keeps its CPU path for every scene part, device or option the GPU path does not carry.
//
// Go is not installed in the image this repository is built in, so this file has not been
// compiled; tests/test_go_binding.py checks every C identifier and struct field it names against
// include/rtx.h and drives the exact C-ABI call sequences it issues through ctypes, and the same
// flattening is built and tested in C++ (raytracer-go_amd/host/flatten.cpp).
package internal

/*
#cgo LDFLAGS: -lrtx
#include <stdlib.h>
#include "rtx.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"math"
	"os"
	"runtime"
	"strconv"
	"sync"
	"sync/atomic"
	"unsafe"
)

// gpuConfig holds a Camera's GPU options (WithGPUs, WithSeed).  The Camera struct is camera.go's,
// so they are kept beside it, keyed by the *Camera (a Camera lives as long as its program).
type gpuConfig struct {
	gpus     int
	seed     uint64
	fallback atomic.Bool // RenderGPU is running the CPU Render: the hook stays out of the way
}

var gpuConfigs sync.Map // *Camera -> *gpuConfig

func (c *Camera) gpuConfig() *gpuConfig {
	if v, ok := gpuConfigs.Load(c); ok {
		return v.(*gpuConfig)
	}
	cfg := &gpuConfig{seed: 1}
	if n, err := strconv.Atoi(os.Getenv("RTX_GPUS")); err == nil { // the default without WithGPUs
		cfg.gpus = n
	}
	v, _ := gpuConfigs.LoadOrStore(c, cfg)
	return v.(*gpuConfig)
}

// WithGPUs renders on n MI355X devices of this process: Render runs the megakernel on row-
// interleaved bands of the image, one per device, gathered to device 0 over RCCL (n > 1).  0 keeps
// the reference's CPU path.  Without this option the RTX_GPUS environment variable decides.
func WithGPUs(n int) CameraOpt {
	return func(c *Camera) {
		c.gpuConfig().gpus = n
	}
}

// WithSeed keys the GPU path's counter-based RNG (Philox4x32-10; DESIGN.md §3): the same seed
// gives the same image on any number of devices.  (The CPU path seeds its workers from the clock,
// camera.go:170.)  It also seeds NewBVHFromWorldGPU's axis draws.
func WithSeed(seed uint64) CameraOpt {
	return func(c *Camera) {
		c.gpuConfig().seed = seed
	}
}

// gpuBVH is the tree NewBVHFromWorld would build over a World of spheres, built on the GPU by
// rtx_scene_create_spheres (NewBVH restated, bvh.go:142-185: the same sort and median split per
// node, the axis drawn from the render seed's stream instead of the global rand).  The CPU path
// (Hit, GetBounds) builds the reference's tree on first use.
type gpuBVH struct {
	world *World
	once  sync.Once
	tree  *BVH
}

// NewBVHFromWorldGPU stands in for NewBVHFromWorld (bvh.go:138-140) when the World holds only
// spheres: Render on the GPU path builds the tree on the device (10 ms for 100k spheres, where the
// host recursion takes about 0.5 s), and any CPU use builds the reference's tree.
func NewBVHFromWorldGPU(w *World) Hittable { return &gpuBVH{world: w} }

func (g *gpuBVH) cpu() *BVH {
	g.once.Do(func() { g.tree = NewBVHFromWorld(g.world) })
	return g.tree
}

func (g *gpuBVH) Hit(r *Ray, rayT Interval) (HitInfo, bool) { return g.cpu().Hit(r, rayT) }

func (g *gpuBVH) GetBounds() Aabb { return g.cpu().GetBounds() }

// gpuTables is the flattened Hittable tree (rtx.h).  The slices hold no Go pointers, so
// passing them to C is legal under the cgo rules; librtx copies them and never keeps them.
type gpuTables struct {
	nodes     []C.rtx_bvh_node
	roots     []C.int32_t
	spheres   []C.rtx_sphere
	quads     []C.rtx_quad
	materials []C.rtx_material
	textures  []C.rtx_texture
	texels    []C.uint32_t
	lists     []C.rtx_list  // Worlds nested in the tree (ABI 5)
	listRefs  []C.int32_t
	matIdx    map[Material]C.uint32_t
	texIdx    map[Texture]C.uint32_t
}

// errUnsupported: a scene part the GPU path does not carry (RenderGPU then uses Render).
var errUnsupported = errors.New("rtx: scene type not on the GPU path")

func primRef(typ, idx int) C.int32_t { return C.int32_t(^int32(uint32(typ)<<28 | uint32(idx)&0x0FFFFFFF)) }

func vec(v Vec3) [3]C.float { return [3]C.float{C.float(v.X), C.float(v.Y), C.float(v.Z)} }

// putRGBA16 appends one RTX_TEX_IMAGE texel: Go's 16-bit Color.RGBA() channels, two words.
func (t *gpuTables) putRGBA16(r, g, b, a uint32) {
	t.texels = append(t.texels, C.uint32_t(r&0xFFFF|(g&0xFFFF)<<16), C.uint32_t(b&0xFFFF|(a&0xFFFF)<<16))
}

func (t *gpuTables) texture(tex Texture) (C.uint32_t, error) {
	if i, ok := t.texIdx[tex]; ok {
		return i, nil
	}
	var r C.rtx_texture
	switch v := tex.(type) {
	case SolidColor:
		r._type, r.even = C.RTX_TEX_SOLID, vec(v.albedo.GetColor())
	case *SolidColor:
		r._type, r.even = C.RTX_TEX_SOLID, vec(v.albedo.GetColor())
	case *Checkered:
		r._type, r.scale = C.RTX_TEX_CHECKERED, C.float(v.scale)
		r.even, r.odd = vec(v.even.GetColor()), vec(v.odd.GetColor())
	case *ImageTexture: // materials.go:175-193: At(int(u*Dx), int(v*Dy)).RGBA(), 16 bits per channel
		b := v.img.Bounds()
		r._type = C.RTX_TEX_IMAGE
		if b.Dy() > 0 {
			// GetTexture indexes At from 0; the table (and its border texel) is exact for bounds
			// at the origin, which jpeg.Decode and image.New* return.
			if b.Min.X != 0 || b.Min.Y != 0 {
				return 0, errUnsupported
			}
			r.width, r.height = C.uint32_t(b.Dx()), C.uint32_t(b.Dy())
			if len(t.texels)%2 != 0 { // 8-byte texels at an even word offset
				t.texels = append(t.texels, 0)
			}
			r.texel_offset = C.uint32_t(len(t.texels))
			for y := 0; y < b.Dy(); y++ {
				for x := 0; x < b.Dx(); x++ {
					t.putRGBA16(v.img.At(x, y).RGBA())
				}
			}
			// The border texel: what At returns outside the bounds (u == 1, v == 0, NaN) —
			// color.YCbCr{} = (0, 34678, 0) for jpeg.Decode's *image.YCbCr, 0 for *image.RGBA.
			t.putRGBA16(v.img.At(b.Max.X, b.Min.Y).RGBA())
		} else {
			r.width = C.uint32_t(max(b.Dx(), 0)) // Dy() <= 0: the debug colour (0, 1, 1), no texels
		}
	case *NoiseTexture: // RTX_NOISE_TEXELS: gradients (float32 bits), then permX, permY, permZ
		r._type, r.scale = C.RTX_TEX_NOISE, C.float(v.scale)
		r.texel_offset = C.uint32_t(len(t.texels))
		for _, g := range v.perlin.randVec3 {
			for _, c := range [3]float32{g.X, g.Y, g.Z} {
				t.texels = append(t.texels, C.uint32_t(math.Float32bits(c)))
			}
		}
		for _, perm := range [][]int{v.perlin.permX, v.perlin.permY, v.perlin.permZ} {
			for _, p := range perm {
				t.texels = append(t.texels, C.uint32_t(p))
			}
		}
	default:
		return 0, errUnsupported
	}
	i := C.uint32_t(len(t.textures))
	t.textures = append(t.textures, r)
	t.texIdx[tex] = i
	return i, nil
}

func (t *gpuTables) material(m Material) (C.uint32_t, error) {
	if i, ok := t.matIdx[m]; ok {
		return i, nil
	}
	var r C.rtx_material
	switch v := m.(type) {
	case *Lambertian:
		ti, err := t.texture(v.albedo)
		if err != nil {
			return 0, err
		}
		r._type, r.texture = C.RTX_MAT_LAMBERTIAN, ti
	case *Metal:
		r._type, r.fuzz, r.albedo = C.RTX_MAT_METAL, C.float(v.fuzz), vec(v.albedo.GetColor())
	case *Dielectric:
		r._type, r.ior = C.RTX_MAT_DIELECTRIC, C.float(v.refractiveIndex)
	case DiffuseLight, *DiffuseLight:
		d, ok := v.(DiffuseLight)
		if !ok {
			d = *v.(*DiffuseLight)
		}
		ti, err := t.texture(d.emit)
		if err != nil {
			return 0, err
		}
		r._type, r.texture = C.RTX_MAT_DIFFUSE_LIGHT, ti
	default:
		return 0, errUnsupported
	}
	i := C.uint32_t(len(t.materials))
	t.materials = append(t.materials, r)
	t.matIdx[m] = i
	return i, nil
}

// ref walks the tree in pre-order (a node before its children, left before right), the
// order NewBVH (bvh.go:142-185) creates it in.
func (t *gpuTables) ref(h Hittable) (C.int32_t, error) {
	switch v := h.(type) {
	case *BVH:
		me := len(t.nodes)
		b := v.bBox
		t.nodes = append(t.nodes, C.rtx_bvh_node{
			bmin: [3]C.float{C.float(b.x.min), C.float(b.y.min), C.float(b.z.min)},
			bmax: [3]C.float{C.float(b.x.max), C.float(b.y.max), C.float(b.z.max)},
		})
		l, err := t.ref(v.left)
		if err != nil {
			return 0, err
		}
		r := l
		if v.right != v.left { // one-element split: left == right (bvh.go:162-165)
			if r, err = t.ref(v.right); err != nil {
				return 0, err
			}
		}
		t.nodes[me].left, t.nodes[me].right = l, r
		return C.int32_t(me), nil
	case *Sphere:
		mi, err := t.material(v.Material)
		if err != nil {
			return 0, err
		}
		t.spheres = append(t.spheres, C.rtx_sphere{center: vec(v.Center), radius: C.float(v.Radius), material: mi})
		return primRef(C.RTX_PRIM_SPHERE, len(t.spheres)-1), nil
	case Quad, *Quad: // fields as NewQuad derived them (hittables.go:149-165)
		q, ok := v.(Quad)
		if !ok {
			q = *v.(*Quad)
		}
		mi, err := t.material(q.material)
		if err != nil {
			return 0, err
		}
		t.quads = append(t.quads, C.rtx_quad{
			q: vec(q.Q), material: mi, u: vec(q.u), d: C.float(q.D), v: vec(q.v), w: vec(q.w), normal: vec(q.normal),
		})
		return primRef(C.RTX_PRIM_QUAD, len(t.quads)-1), nil
	case *World: // a World nested in the tree (hittables.go:55-72 as a BVH child): a list ref
		// (an empty one is a miss: a list of no items, ABI 6)
		refs := make([]C.int32_t, len(v.hittables))
		for i, h := range v.hittables {
			r, err := t.ref(h)
			if err != nil {
				return 0, err
			}
			refs[i] = r
		}
		first := len(t.listRefs)
		t.listRefs = append(t.listRefs, refs...)
		t.lists = append(t.lists, C.rtx_list{first: C.uint32_t(first), count: C.uint32_t(len(refs))})
		return primRef(C.RTX_PRIM_LIST, len(t.lists)-1), nil
	default:
		return 0, errUnsupported
	}
}

// rtxError is a library error code with rtx_last_error's message (Render's error return).
type rtxError struct {
	code C.int
	msg  string
}

func (e *rtxError) Error() string { return fmt.Sprintf("rtx error %d: %s", int(e.code), e.msg) }

func rtxErr(rc C.int) error { return &rtxError{code: rc, msg: C.GoString(C.rtx_last_error())} }

// gpuMissing: the library cannot run this render at all (no device, a feature it reports as
// unsupported): RenderGPU then renders on the CPU.  (RCCL trouble is not among them: rtx_render
// assembles the bands with per-band copies when RCCL is unavailable or fails, rtx.h.)
func gpuMissing(rc C.int) bool {
	return rc == C.RTX_ERR_UNSUPPORTED || rc == C.RTX_ERR_NO_DEVICE || rc == C.RTX_ERR_RCCL
}

// flatten: the tree Render receives as rtx.h tables; a plain *World gives one root per item
// (its linear closest-hit scan, hittables.go:55-72).
func flatten(world Hittable) (*gpuTables, error) {
	t := &gpuTables{matIdx: map[Material]C.uint32_t{}, texIdx: map[Texture]C.uint32_t{}}
	items := []Hittable{world}
	if wl, ok := world.(*World); ok {
		items = wl.hittables
	}
	for _, it := range items {
		r, err := t.ref(it)
		if err != nil {
			return nil, err
		}
		t.roots = append(t.roots, r)
	}
	if len(t.roots) == 0 || len(t.materials) == 0 {
		return nil, errUnsupported
	}
	return t, nil
}

// errFallback: the GPU path cannot carry this render (a scene part it does not flatten, no
// device, a feature the library reports unsupported): the CPU path renders it instead.
var errFallback = errors.New("rtx: render on the CPU path")

// renderGPU is the hook at the top of Render (camera.go:180, INTEGRATION.md): with WithGPUs(n > 0)
// (or RTX_GPUS) it renders on the devices and reports done; otherwise, or when the GPU path cannot
// carry the render, Render continues on its CPU path.
func (c *Camera) renderGPU(world Hittable, writer io.Writer) (bool, error) {
	cfg := c.gpuConfig()
	if cfg.gpus <= 0 || cfg.fallback.Load() {
		return false, nil
	}
	err := c.renderOnDevices(world, writer, cfg.seed, cfg.gpus)
	if errors.Is(err, errFallback) {
		return false, nil
	}
	return true, err
}

// RenderGPU is Render (camera.go:180) on the MI355X path with an explicit seed and device count,
// whatever the camera's options: same P3 bytes to writer, same error return; the CPU Render for
// anything the GPU path does not carry.
func (c *Camera) RenderGPU(world Hittable, writer io.Writer, seed uint64, gpus int) error {
	err := c.renderOnDevices(world, writer, seed, max(gpus, 1))
	if errors.Is(err, errFallback) {
		cfg := c.gpuConfig()
		cfg.fallback.Store(true)
		defer cfg.fallback.Store(false)
		return c.Render(world, writer)
	}
	return err
}

// sceneOf uploads the world once (rtx_scene_create, or rtx_scene_create_spheres for a
// NewBVHFromWorldGPU tree): the caller destroys the scene.  Go slices stay pinned only for the
// call; librtx copies them and keeps no pointer into Go memory.
func sceneOf(world Hittable, seed uint64) (*C.rtx_scene, error) {
	var pin runtime.Pinner
	defer pin.Unpin()
	var scene *C.rtx_scene
	if g, ok := world.(*gpuBVH); ok {
		t := &gpuTables{matIdx: map[Material]C.uint32_t{}, texIdx: map[Texture]C.uint32_t{}}
		for _, h := range g.world.hittables { // spheres in Add order: NewBVH's input list
			s, ok := h.(*Sphere)
			if !ok {
				return nil, errFallback
			}
			mi, err := t.material(s.Material)
			if err != nil {
				return nil, err
			}
			t.spheres = append(t.spheres, C.rtx_sphere{center: vec(s.Center), radius: C.float(s.Radius), material: mi})
		}
		if len(t.spheres) == 0 {
			return nil, errFallback
		}
		pin.Pin(&t.spheres[0])
		pin.Pin(&t.materials[0])
		var tex *C.rtx_texture
		var texels *C.uint32_t
		if len(t.textures) > 0 {
			pin.Pin(&t.textures[0])
			tex = &t.textures[0]
		}
		if len(t.texels) > 0 {
			pin.Pin(&t.texels[0])
			texels = &t.texels[0]
		}
		if rc := C.rtx_scene_create_spheres(&t.spheres[0], C.uint32_t(len(t.spheres)), &t.materials[0],
			C.uint32_t(len(t.materials)), tex, C.uint32_t(len(t.textures)), texels, C.uint64_t(len(t.texels)),
			C.uint64_t(seed), 0, &scene, nil); rc != 0 {
			return nil, rtxErr(rc)
		}
		return scene, nil
	}
	t, err := flatten(world)
	if err != nil {
		return nil, err
	}
	var desc C.rtx_scene_desc
	if len(t.nodes) > 0 {
		pin.Pin(&t.nodes[0])
		desc.nodes, desc.n_nodes = &t.nodes[0], C.uint32_t(len(t.nodes))
	}
	pin.Pin(&t.roots[0])
	desc.roots, desc.n_roots = &t.roots[0], C.uint32_t(len(t.roots))
	if len(t.spheres) > 0 {
		pin.Pin(&t.spheres[0])
		desc.spheres, desc.n_spheres = &t.spheres[0], C.uint32_t(len(t.spheres))
	}
	if len(t.quads) > 0 {
		pin.Pin(&t.quads[0])
		desc.quads, desc.n_quads = &t.quads[0], C.uint32_t(len(t.quads))
	}
	pin.Pin(&t.materials[0])
	desc.materials, desc.n_materials = &t.materials[0], C.uint32_t(len(t.materials))
	if len(t.textures) > 0 {
		pin.Pin(&t.textures[0])
		desc.textures, desc.n_textures = &t.textures[0], C.uint32_t(len(t.textures))
	}
	if len(t.texels) > 0 {
		pin.Pin(&t.texels[0])
		desc.texels, desc.n_texels = &t.texels[0], C.uint64_t(len(t.texels))
	}
	if len(t.lists) > 0 {
		pin.Pin(&t.lists[0])
		desc.lists, desc.n_lists = &t.lists[0], C.uint32_t(len(t.lists))
	}
	if len(t.listRefs) > 0 {
		pin.Pin(&t.listRefs[0])
		desc.list_refs, desc.n_list_refs = &t.listRefs[0], C.uint32_t(len(t.listRefs))
	}
	if rc := C.rtx_scene_create(&desc, &scene); rc != 0 {
		return nil, rtxErr(rc)
	}
	return scene, nil
}

// renderOnDevices renders on `gpus` devices and writes Render's P3 bytes; errFallback when the GPU
// path cannot carry the render (nothing has been written then).
func (c *Camera) renderOnDevices(world Hittable, writer io.Writer, seed uint64, gpus int) error {
	c.init() // Camera.init (idempotent, sync.Once): the derived state below (camera.go:128-165)
	scene, err := sceneOf(world, seed)
	var re *rtxError
	if errors.Is(err, errUnsupported) || (errors.As(err, &re) && gpuMissing(re.code)) {
		return errFallback
	}
	if err != nil {
		return err
	}
	// Destroying the last scene on a device also frees the library's sample scratch there, so
	// nothing stays pinned in HBM after Render returns.
	defer C.rtx_scene_destroy(scene)

	w, h := int(c.imageWidth), int(c.imageHeight)
	cam := C.rtx_camera{
		image_width: C.uint32_t(w), image_height: C.uint32_t(h),
		samples_per_pixel: C.uint32_t(c.samplesPerPixel), max_depth: C.uint32_t(max(c.bounceDepth, 0)),
		center: vec(c.center), defocus_angle: C.float(c.defocusAngleRadians),
		pixel00: vec(c.pixel00), pixel_du: vec(c.pixelDu), pixel_dv: vec(c.pixelDv),
		defocus_disk_u: vec(c.defocusDiskU), defocus_disk_v: vec(c.defocusDiskV),
		background: vec(c.background.GetColor()),
	}
	// Render + the P3 text (header included) on the device: rtx_render_ppm on the current device for one
	// GPU; for several, rtx_render_ppm_ex (ABI 9) gathers the row-interleaved bands to device 0 over RCCL
	// and encodes them there, so no per-pixel formatting runs on the host at any device count
	// (camera.go:183-188, 212-215 and vec3.go:141-166 on the GPU, byte-identical).
	text := make([]byte, int(C.rtx_ppm_max_bytes(C.uint32_t(w), C.uint32_t(h))))
	var n C.uint64_t
	var rc C.int
	if gpus <= 1 {
		rc = C.rtx_render_ppm(scene, &cam, C.uint64_t(seed), (*C.char)(unsafe.Pointer(&text[0])),
			C.uint64_t(len(text)), &n, nil)
	} else {
		rc = C.rtx_render_ppm_ex(scene, &cam, C.uint64_t(seed), C.int(gpus), (*C.char)(unsafe.Pointer(&text[0])),
			C.uint64_t(len(text)), &n, nil)
	}
	if rc != 0 {
		if gpuMissing(rc) {
			return errFallback
		}
		return rtxErr(rc)
	}
	_, err = writer.Write(text[:int(n)])
	return err
}
