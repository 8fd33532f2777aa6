/* shim_sequence.c — the exact C call sequence of go/internal/renderer/gpu.go
 * (RenderGPU), for the test suite: Go cannot run in this image, so this
 * program stands in for the cgo side and is checked against the Python
 * mirror's render.
 *
 *   usage: shim_sequence <scene as json.Marshal writes it> <W> <H> <samples> <out.rgba> [devices]
 *   devices: the device of each rank, comma-separated (e.g. 0,0,0: three
 *   ranks on device 0); default 0
 *   exit 0: rendered, raw RGBA (W*H*4) written; exit 2: bad usage / I/O;
 *   exit 3: a library call failed (message on stderr, e.g. no GPU).
 *
 * The calls, in gpu.go's order:
 *   rt_scene_parse_json (the json.Marshal bytes of *scene.Scene; verbose: the
 *     lines GetHittables prints, scene.go:62-88)
 *   rt_settings_default + the ParallelRenderer fields (settings.go:3-25)
 *   rt_renderer_create (first Render of this ParallelRenderer)
 *   rt_renderer_render into the caller's Pix buffer (image.RGBA, W*H*4)
 *   rt_scene_free; rt_renderer_destroy (CloseGPU)
 */
#include <stdio.h>
#include <stdlib.h>

#include "rt_api.h"

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s scene.json W H samples out.rgba [devices]\n", argv[0]);
    return 2;
  }
  const int w = atoi(argv[2]), h = atoi(argv[3]), spp = atoi(argv[4]);
  int devs[64], ndev = 0;
  if (argc > 6) {
    for (const char* p = argv[6]; *p && ndev < 64;) {
      devs[ndev++] = atoi(p);
      while (*p && *p != ',') ++p;
      if (*p == ',') ++p;
    }
  }
  if (ndev == 0) devs[ndev++] = 0;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char* data = (char*)malloc((size_t)n);
  if (!data || fread(data, 1, (size_t)n, f) != (size_t)n) return 2;
  fclose(f);

  rt_scene_buf* sb = NULL;
  int rc = rt_scene_parse_json(data, (size_t)n, 1, &sb);
  free(data);
  if (rc != RT_OK) {
    fprintf(stderr, "rt_scene_parse_json failed (%d): %s\n", rc, rt_last_error());
    return 3;
  }
  rt_settings st;
  rt_settings_default(&st);
  st.samples = spp;  /* r.samples; the other fields keep NewParallelRenderer's defaults */
  st.max_depth = 50;
  st.anti_aliasing = 1;
  st.recursive_reflections = 1;
  st.soft_shadows = 1;
  st.depth_of_field = 0;
  st.num_workers = 8;
  st.num_devices = ndev;

  rt_renderer* r = NULL;
  rc = rt_renderer_create(devs, ndev, &r);
  if (rc != RT_OK) {
    fprintf(stderr, "rt_renderer_create failed (%d): %s\n", rc, rt_last_error());
    rt_scene_free(sb);
    return 3;
  }
  unsigned char* pix = (unsigned char*)calloc((size_t)w * h * 4, 1);
  rt_stats stats;
  rc = rt_renderer_render(r, rt_scene_view(sb), w, h, &st, NULL, pix, &stats);
  rt_scene_free(sb);
  rt_renderer_destroy(r);
  if (rc != RT_OK) {
    fprintf(stderr, "rt_renderer_render failed (%d): %s\n", rc, rt_last_error());
    free(pix);
    return 3;
  }
  FILE* o = fopen(argv[5], "wb");
  if (!o || fwrite(pix, 1, (size_t)w * h * 4, o) != (size_t)w * h * 4) return 2;
  fclose(o);
  free(pix);
  printf("objects %d lights %d render %.6f s\n", stats.objects, stats.lights, stats.render_seconds);
  return 0;
}
