// gi_oracle.h — TEST INFRASTRUCTURE ONLY.
//
// C API of this repo's CPU restatement of the reference per-pixel radiance loop
// (preon7/2019global include/raytracer.h:23-87 and everything it calls), used by tests/ and by
// bench.py's cpu_baseline leg as the checker.  The product (2019global_amd/libgi.so) never links it.
//
// Mode R (mode=0): the reference's semantics bit for bit, pinned against
//   golden vectors produced by the compiled reference (oracle/_ref/ref_harness).
// Mode X (mode=1): the build-defined depth/spp integrator specified in DESIGN.md §"Mode X";
//   nearest hit over all primitives (brute force, or an equivalent padded fp64 BVH for large scenes).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Render the pixel window [x0,x1)x[y0,y1) of a w x h frame of the scene in `scn` (.scn text).
// Outputs are row-major over the window; any output pointer may be NULL.
//   rgb   : fp64 radiance, 3 per pixel (Mode X: the spp mean, clamped at 1)
//   hit   : entity index (push order) of the chosen/primary hit, -1 if none
//   uv    : texture coordinates (int) of that hit
//   ncand : Mode R: length of Octree::intersect's candidate list; Mode X: rays traced per pixel
//   nnode : Mode R: ExpBox node tests made by Octree::intersect
//   q     : Image::setPixel quantisation (RGB888)
// threads <= 0: OpenMP default.  Returns 0 on success, <0 on error (message in gio_last_error).
int gio_render(const char* scn, int w, int h, int mode, int spp, int depth, uint64_t seed,
               int x0, int y0, int x1, int y1, int threads,
               double* rgb, int32_t* hit, int32_t* uv, int32_t* ncand, int32_t* nnode, uint8_t* q);

// bench.py's cpu_baseline: Mode X over full-width rows y = row0 + k*stride (k < n_rows); primary
// samples whose ray misses the scene's bounding box are counted apart and not traced.  out[4]: rays,
// resolved primary samples, pixels, radiance sum.
int gio_time_rows(const char* scn, int w, int h, int spp, int depth, uint64_t seed, int row0, int stride, int n_rows,
                  int threads, double* out, double* rgb, uint8_t* q);

// Octree dump in the same text format as `ref_harness tree` (bbox lines, then DFS node lines).
// Returns the number of bytes needed (excluding NUL); writes at most cap bytes.
long gio_tree(const char* scn, char* buf, long cap);

// Per-(ray, entity) intersect + getTextureCoord, same layout as `ref_harness rays`:
// rays: n x (origin[3], dir[3]); out_hit n*E, out_pn n*E*6, out_uv n*E*2.
int gio_rays(const char* scn, int n, const double* rays, int32_t* out_hit, double* out_pn, int32_t* out_uv);

// ExpBox node test over n x (min[3], max[3], origin[3], dir[3]) records.
int gio_boxes(int n, const double* recs, int32_t* out);

// Mode X closest-hit / shadow queries: -1 (default) = this oracle's BVH above 256 primitives,
// brute force below; 0 = brute force always; 1 = BVH always.  Same results either way (tested).
void gio_set_accel(int mode);
void gio_set_no_shadow(int on);   /* Mode X without shadow rays (GI_FLAG_X_NO_SHADOW; tests) */

const char* gio_last_error(void);

#ifdef __cplusplus
}
#endif
