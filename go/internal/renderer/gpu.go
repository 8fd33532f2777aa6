//go:build rtgo

// gpu.go — the cgo shim that puts the reference's Render path on MI355X GPUs.
//
// Drop this file into raytraceGo's internal/renderer (the package of
// renderer.go) and build with `go build -tags rtgo`; set
//     CGO_CFLAGS="-I<this repo>/include"
//     CGO_LDFLAGS="-L<this repo>/concurrent-raytracer-go_amd/build -Wl,-rpath,<same>"
// so cgo finds rt_api.h and librtgo.so (make -C concurrent-raytracer-go_amd).
// RenderGPU has Render's signature and meaning (renderer.go:67-126): it
// returns a new *image.RGBA whose row y is Go image row y, tone-mapped by
// toneMap + ToRGB (renderer.go:348-367, vector.go:106-109), and fills the
// same benchmarkData fields (renderer.go:103-112).  cmd/raytracer/main.go:49
// calls it in place of Render (INTEGRATION.md §1).
//
// The scene crosses the boundary as the JSON it was loaded from:
// json.Marshal of *scene.Scene (Vec3.MarshalJSON writes [x, y, z],
// vector.go:195-197) parsed by rt_scene_parse_json, which applies
// createMaterial's defaults and GetHittables' type rules (scene.go:59-148)
// exactly as the C++ loader does for a file.  One rt_renderer per
// ParallelRenderer holds the devices' scenes, schedules and buffers between
// calls (NewParallelRenderer once, Render per frame); RT_DEVICES sets how many
// GPUs it shards the tiles over (default 1).
//
// Go cannot run in the image this was written in (no toolchain, SURVEY.md
// §8c): tests/c/shim_sequence.c makes exactly this file's C call sequence
// and is run by the test suite instead.
package renderer

/*
#cgo LDFLAGS: -lrtgo
#include <stdlib.h>
#include "rt_api.h"
*/
import "C"

import (
	"encoding/json"
	"fmt"
	"image"
	"os"
	"strconv"
	"sync"
	"time"
	"unsafe"

	"raytraceGo/internal/scene"
)

var (
	gpuMu        sync.Mutex
	gpuRenderers = map[*ParallelRenderer]*C.rt_renderer{}
)

func cbool(b bool) C.int32_t {
	if b {
		return 1
	}
	return 0
}

func rtError(what string, rc C.int) error {
	return fmt.Errorf("%s failed (%d): %s", what, int(rc), C.GoString(C.rt_last_error()))
}

// gpuRenderer returns r's rt_renderer, made on first use (rt_renderer_create).
func (r *ParallelRenderer) gpuRenderer() (*C.rt_renderer, error) {
	gpuMu.Lock()
	defer gpuMu.Unlock()
	if h, ok := gpuRenderers[r]; ok {
		return h, nil
	}
	n := 1
	if v, err := strconv.Atoi(os.Getenv("RT_DEVICES")); err == nil && v > 0 {
		n = v
	}
	var h *C.rt_renderer
	if rc := C.rt_renderer_create(nil, C.int32_t(n), &h); rc != C.RT_OK {
		return nil, rtError("rt_renderer_create", rc)
	}
	gpuRenderers[r] = h
	return h, nil
}

// StartGPU makes r's rt_renderer now (HIP runtime start-up, contexts, the
// kernels' code objects): the devices' constructor work, so that a caller
// that times Render after NewParallelRenderer (cmd/raytracer/main.go:46-51,
// renderer.go:68,101) keeps it out of the timed call.  RenderGPU makes the
// renderer itself when StartGPU has not run.
func (r *ParallelRenderer) StartGPU() error {
	_, err := r.gpuRenderer()
	return err
}

// CloseGPU frees r's devices' resources (rt_renderer_destroy).
func (r *ParallelRenderer) CloseGPU() {
	gpuMu.Lock()
	defer gpuMu.Unlock()
	if h, ok := gpuRenderers[r]; ok {
		C.rt_renderer_destroy(h)
		delete(gpuRenderers, r)
	}
}

// RenderGPU is Render (renderer.go:67-126) on the GPUs.  Like Render it has
// no error return: a failure of the device path panics with the library's
// message (the reference panics on bad scene input, scene.go:113).
func (r *ParallelRenderer) RenderGPU(s *scene.Scene, width, height int) *image.RGBA {
	start := time.Now()
	data, err := json.Marshal(s)
	if err != nil {
		panic(fmt.Sprintf("RenderGPU: %v", err))
	}
	cdata := C.CBytes(data)
	defer C.free(cdata)
	var sb *C.rt_scene_buf
	// verbose 1: the lines Render prints through GetHittables (scene.go:62-88)
	if rc := C.rt_scene_parse_json((*C.char)(cdata), C.size_t(len(data)), 1, &sb); rc != C.RT_OK {
		panic(rtError("rt_scene_parse_json", rc).Error())
	}
	defer C.rt_scene_free(sb)

	var st C.rt_settings // settings.go:3-25 through the renderer's fields
	C.rt_settings_default(&st)
	st.samples = C.int32_t(r.samples)
	st.max_depth = C.int32_t(r.maxDepth)
	st.anti_aliasing = cbool(r.antiAliasing)
	st.recursive_reflections = cbool(r.recursiveReflections)
	st.soft_shadows = cbool(r.softShadows)
	st.depth_of_field = cbool(r.depthOfField)
	st.num_workers = C.int32_t(r.numWorkers)

	img := image.NewRGBA(image.Rect(0, 0, width, height))
	var stats C.rt_stats
	if width <= 0 || height <= 0 {
		// Render with no tiles (createRenderTasks makes none): an empty image
		stats.objects = C.int32_t(C.rt_scene_view(sb).num_objects)
		stats.lights = C.int32_t(C.rt_scene_view(sb).num_lights)
		return r.finishGPU(s, img, width, height, start, stats)
	}
	h, err := r.gpuRenderer()
	if err != nil {
		panic(err.Error())
	}
	// img.Pix: W*H*4 bytes, row y = Go image row y, the layout rt_renderer_render
	// writes; a Go pointer to pointer-free memory, not retained (cgo rules)
	rc := C.rt_renderer_render(h, C.rt_scene_view(sb), C.int32_t(width), C.int32_t(height), &st, nil,
		(*C.uint8_t)(unsafe.Pointer(&img.Pix[0])), &stats)
	if rc != C.RT_OK {
		panic(rtError("rt_renderer_render", rc).Error())
	}
	return r.finishGPU(s, img, width, height, start, stats)
}

// finishGPU records Render's benchmark data and prints its closing lines
// (renderer.go:101-123).
func (r *ParallelRenderer) finishGPU(s *scene.Scene, img *image.RGBA, width, height int, start time.Time,
	stats C.rt_stats) *image.RGBA {
	renderTime := time.Since(start)
	r.benchmarkData.SceneName = s.GetSceneName() // renderer.go:103-112
	r.benchmarkData.Resolution = fmt.Sprintf("%dx%d", width, height)
	r.benchmarkData.RenderTime = renderTime.Seconds()
	r.benchmarkData.Samples = r.samples
	r.benchmarkData.MaxDepth = r.maxDepth
	r.benchmarkData.NumWorkers = r.numWorkers
	r.benchmarkData.Objects = int(stats.objects)
	r.benchmarkData.Lights = int(stats.lights)
	r.benchmarkData.Timestamp = time.Now()
	r.benchmarkData.Features = []string{
		"Improved metallic reflections with Fresnel effect",
		"Shiny materials with configurable roughness and specular",
		"Enhanced light source reflections",
		"Better specular highlights for metallic surfaces",
	}
	fmt.Printf("Rendering complete!\n")
	fmt.Printf("Enhanced materials features:\n")
	for _, feature := range r.benchmarkData.Features {
		fmt.Printf("- %s\n", feature)
	}
	return img
}
