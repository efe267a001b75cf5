/* gi.h — C-ABI of the MI355X-native (gfx950) per-pixel radiance path for preon7/2019global.
 *
 * This is the drop-in boundary for the reference's render driver.  The reference has no ABI: its
 * path is the header-only class RayTracer (include/raytracer.h:15-101) whose run(w, h)
 * (raytracer.h:23-87) loops over pixels and, per pixel, queries Octree::intersect
 * (octree.h:46-68), calls Entity::intersect / getTextureCoord (entities.h:26, 32) and
 * Material::blinn_phong_texture (material.h:48-62), and stores through Image::setPixel
 * (image.h:14-16).  The entry points below replace, one for one:
 *
 *   gi_scene_create      Octree(min,max) (octree.h:14) + Octree::push_back per entity
 *                        (octree.h:20-43) + the entity constructors (entities.h:45, 138, 581, ...)
 *   gi_camera_init       Camera(pos, lookAt, focal) (camera.h:8-10)
 *   gi_render            RayTracer::run(w, h) (raytracer.h:23-87), host buffers, progressive tiles,
 *                        cancel flag = RayTracer::stop() (raytracer.h:90)
 *   gi_render_device     the same frame into device-resident buffers on a HIP stream (bench,
 *                        multi-GPU tile sharding)
 *   gi_trace_ray         one iteration of raytracer.h:41-84 for an arbitrary ray
 *   gi_unshard_device    reassembles a frame from per-rank packed tiles after the RCCL gather
 *   gi_scene_kernel_ms   HIP-event duration of the last timed render's dominant kernel (bench)
 *   gi_scene_x_form      which Mode X form (persistent kernel / wavefront) a render would run
 *   gi_octree_*          Octree(min,max) + push_back (octree.h:14-43) and the public query
 *                        Octree::intersect(const Ray&) (octree.h:46-68 -> Node::intersect :132-155)
 *                        on the host, for reference-side callers of the candidate list
 *   gi_obj_parse         scene I/O: a Wavefront OBJ mesh as the run of
 *                        ImpTriangle(p1, p2, p3) pushes (entities.h:138) main.cpp:24-48 would write
 *   gi_multi_*           RayTracer::run over several GPUs of one process: a scene replica per
 *                        device, 8x8 tiles dealt round-robin, RCCL send/recv gather over xGMI to
 *                        the first device (the drop-in RayTracer uses it when GI_DEVICES lists
 *                        devices; by default it renders on the current device alone)
 *
 * Conventions: all pointers are plain C pointers; buffers are caller-owned; sizes are in elements;
 * every function returns 0 on success and a negative gi_status on error, with a thread-local
 * message from gi_last_error().  No exception crosses this boundary.  Rendering never falls back
 * to the CPU: without a usable gfx950 device gi_scene_create fails with GI_ERR_DEVICE.
 */
#ifndef GI_H_
#define GI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GI_ABI_VERSION 10

typedef enum gi_status {
    GI_OK = 0,
    GI_ERR_ARG = -1,      /* invalid argument */
    GI_ERR_DEVICE = -2,   /* HIP error / no device */
    GI_ERR_SCENE = -3,    /* unsupported entity or material */
    GI_ERR_CANCELLED = -4,/* *cancel became non-zero; frame partially rendered */
    GI_ERR_NOMEM = -5,    /* host memory exhausted (std::bad_alloc inside the library) */
    GI_ERR_INTERNAL = -6  /* any other exception caught at the boundary */
} gi_status;

/* Entity kinds.  args[] holds the reference constructor's arguments in constructor order. */
typedef enum gi_entity_kind {
    GI_IMP_SPHERE = 1,   /* ImpSphere(pos, float radius, color)              entities.h:45  args: px py pz r cr cg cb            */
    GI_IMP_TRIANGLE = 2, /* ImpTriangle(p1, p2, p3) (material: red)          entities.h:138 args: p1 p2 p3 (9)                   */
    GI_EXP_QUAD = 3,     /* ExpQuad(pos, float w, float l, float alpha, col) entities.h:581 args: px py pz w l alpha cr cg cb    */
    GI_EXP_SPHERE = 4,   /* ExpSphere(pos, float radius, color)              entities.h:461 args: px py pz r cr cg cb            */
    GI_EXP_CUBE = 5,     /* ExpCube(pos, float w, float l, float h, color)   entities.h:652 args: px py pz w l h cr cg cb        */
    GI_EXP_CONE = 6,     /* ExpCone(pos, dir, float h, float r, color)       entities.h:823 args: px py pz dx dy dz h r cr cg cb */
                         /*   (dir is stored but unused: the reference cone always points along (-1,0,-10), :825)           */
    GI_EXP_RECTANGLE = 7,/* ExpRectangle(p1, p2, p3) (material: red)         entities.h:310 args: p1 p2 p3 (9)                   */
    GI_EXP_BOX = 8       /* ExpBox(min, max) (material: red)                 entities.h:381 args: min max (6)                    */
} gi_entity_kind;

typedef struct gi_entity_desc {
    int32_t kind;               /* gi_entity_kind */
    int32_t has_material;       /* 1: entity->material = Material(mat_color, mat_shader); specular_power set */
    double args[11];
    double mat_color[3];
    double mat_shader[3];       /* Material::shader_parameters (material.h:27) */
    double mat_specular_power;  /* Material::specular_power (material.h:29) */
    double mat_reflectivity;    /* Mode X only (the reference has no mirrors): probability in [0, 1] that a
                                   bounce leaves by mirror reflection instead of a diffuse sample (DESIGN.md
                                   "Mode X"); 0 (value-initialised descriptors) = diffuse only.  Mode R
                                   ignores it. */
} gi_entity_desc;

typedef struct gi_scene_desc {
    double octree_min[3];       /* Octree(min, max) */
    double octree_max[3];
    int32_t n_entities;         /* push_back order = candidate order */
    const gi_entity_desc* entities;
} gi_scene_desc;

/* Camera as the reference stores it (camera.h:16-20). */
typedef struct gi_camera {
    double pos[3];
    double up[3];
    double forward[3];          /* normalised */
    double focal;
} gi_camera;

typedef enum gi_mode {
    GI_MODE_R = 0,  /* the reference's semantics bit for bit (depth 1, 1 spp) */
    GI_MODE_X = 1   /* build-defined depth/spp integrator (DESIGN.md "Mode X") */
} gi_mode;

#define GI_FLAG_STATS 1u   /* accumulate work counters into opts->stats (device pointer) */
#define GI_FLAG_R_DFS 2u   /* Mode R: walk the whole reference octree in reverse DFS order instead of
                              reconstructing the candidate list (same result; A/B and tests) */
#define GI_FLAG_TIME 4u    /* record HIP events around the frame's dominant kernel (k_mode_r / k_mode_x; the
                              wavefront form and Mode R's flat phases: their whole sequence) on the render's
                              stream; averaged by gi_scene_kernel_ms */
#define GI_FLAG_X_NO_SHADOW 8u   /* Mode X, test only: no shadow rays (every light is visible).  With
                                    depth 1 and spp 1 this reduces Mode X to the reference's own
                                    shading (raytracer.h:41-84, material.h:48-62), so its stages can
                                    be checked against the reference's frames (tests) */
#define GI_FLAG_X_WF 16u         /* Mode X: the wavefront form (one launch per bounce over a compacted queue of
                                    live paths, gi_wf.hip) whatever the scene; same frame bit for bit.  A test
                                    reference (slower everywhere) */
#define GI_FLAG_X_MEGA 32u       /* Mode X: the persistent path-state kernel (k_mode_x) whatever the scene */
#define GI_FLAG_X_SEG 64u        /* Mode X: the segment-synchronous persistent form (k_seg: every loop
                                    iteration one whole path segment per lane).  None of the three form
                                    flags: chosen per launch (GI_X_WF=0/1/2 overrides) */

typedef struct gi_opts {
    int32_t mode;          /* gi_mode */
    int32_t spp;           /* Mode X samples per pixel (>= 1) */
    int32_t depth;         /* Mode X path length (>= 1) */
    int32_t shard_count;   /* >= 1: number of ranks the frame is split over */
    int32_t shard_index;   /* this rank, 0 <= shard_index < shard_count */
    int32_t band_rows;     /* gi_render only: rows per progressive band (0 = whole frame) */
    uint32_t flags;        /* GI_FLAG_* */
    int32_t reserved;
    uint64_t seed;         /* Mode X RNG seed */
    uint64_t* stats;       /* device pointer to GI_STATS_N uint64 counters (GI_FLAG_STATS) */
    /* Mode X progressive passes (ABI 10; both 0: the whole frame at once).  A pass renders samples
     * [sample_begin, sample_end) of the spp-sample frame (spp > 1) and delivers the running estimate
     * min(sum over samples s < sample_end / sample_end, 1) -- for sample_end > 1 exactly the frame of
     * spp = sample_end, since the samples' jitter and paths do not depend on spp (a pass ending at
     * sample 1 holds the JITTERED sample 0 of the spp-sample frame, while a real spp = 1 frame is not
     * jittered); the pass with sample_end == spp is the one-shot frame bit for bit.  A pass is
     * accepted when it has been issued: a device error that surfaces later (a failed launch, a
     * fault) ends the progressive frame -- the next continuation is refused (GI_ERR_DEVICE) and the
     * frame restarts at sample 0.  Passes continue one frame: they are issued on one scene in
     * order (sample_begin = the previous pass's sample_end, the first at 0) with the same camera,
     * light, size, spp, depth, seed and shard, and no other render of the scene in between; the
     * scene keeps the frame's per-sample radiance rows and work list between them (GI_ERR_ARG
     * otherwise).  gi_render: whole-frame bands only (band_rows 0 or >= h). */
    int32_t sample_begin;
    int32_t sample_end;
} gi_opts;

/* stats[] slots */
#define GI_STAT_RAYS 0        /* rays traced (primary + bounce + shadow) */
#define GI_STAT_NODES 1       /* octree node records fetched & tested */
#define GI_STAT_PRIMS 2       /* primitive records fetched & tested in fp64 */
#define GI_STAT_PIXELS 3
#define GI_STAT_X_PATH_MAX 4  /* Mode X: the longest sample path (primary ray to its end), a maximum:
                                 (ticks of the device's 100 MHz constant clock << 32) | (wave loop
                                 iterations << 16) | (that lane's traversal steps), both <= 65535 */
#define GI_STAT_X_ITERS 5     /* Mode X: wave loop iterations (per wave) */
#define GI_STAT_X_TRAV 6      /* Mode X: lane traversal steps (sum of active lanes over iterations) */
#define GI_STAT_X_HANDLE 7    /* Mode X: shading-handler executions (per wave) */
#define GI_STAT_X_HLANES 8    /* Mode X: lanes running the handler (sum over executions) */
#define GI_STAT_X_HCLOSE 9    /* Mode X: of those, lanes consuming a closest hit */
#define GI_STAT_X_HSHADOW 10  /* Mode X: of those, lanes consuming a shadow query */
#define GI_STAT_X_CYC_TRAV 11 /* Mode X: wave clock cycles in traversal steps */
#define GI_STAT_X_CYC_HIT 12  /* Mode X: wave clock cycles consuming finished rays (shading) */
#define GI_STAT_X_CYC_NEXT 13 /* Mode X: wave clock cycles starting rays (raygen, pixel fetch, root test) */
#define GI_STAT_X_CYC_ALL 14  /* Mode X: wave clock cycles in the whole loop */
#define GI_STAT_X_RESOLVED 15 /* Mode X: primary samples resolved without traversal (pixel-frustum classify
                                 and root-box pretest misses; each still adds exactly +0, as traced) */
/* Mode X divergence profile (wave-level): loop iterations in which some lane ran a node test (IT_NODE)
   and the lane node tests (LN_NODE); the same for leaf tests, inline bounce restarts (RS) and passes of
   the handler's ray-start loop (ST: lanes = lanes in the handler during the pass) */
#define GI_STAT_X_IT_NODE 16
#define GI_STAT_X_LN_NODE 17
#define GI_STAT_X_IT_LEAF 18
#define GI_STAT_X_LN_LEAF 19
#define GI_STAT_X_IT_RS 20
#define GI_STAT_X_LN_RS 21
#define GI_STAT_X_IT_ST 22
#define GI_STAT_X_LN_ST 23
#define GI_STAT_R_PAIRS 24      /* Mode R flat phases: candidate pairs (pixel, entity) the walk stored */
#define GI_STAT_R_OVF_TILES 25  /* Mode R flat phases: tiles whose candidates did not fit the pair
                                   buffer, rendered by the fallback kernel (k_mode_r_batch) instead */
#define GI_STATS_N 26

#define GI_TILE 8             /* shard granularity: 8x8 pixel tiles, dealt round-robin to ranks */

typedef struct gi_scene gi_scene;

typedef struct gi_scene_info {
    int32_t n_entities;
    int32_t n_nodes;          /* reference octree nodes (Mode R) */
    int32_t n_leaves;
    int32_t max_depth;
    int32_t n_reachable;      /* entities referenced by at least one leaf */
    int32_t n_dropped;        /* entities whose bbox misses the root (A.14) */
    int32_t x_nodes;          /* Mode X octree nodes */
    int32_t x_prims;          /* Mode X primitives */
    int64_t device_bytes;     /* scene bytes resident in HBM */
    int32_t x_node_bytes;     /* Mode X traversal node record: 256 (XWNode) or 128 (quantised XCNode,
                                 large HBM-resident scenes) -- bench.py's algorithmic bytes per visit */
    int32_t x_lds_resident;   /* 1: Mode X stages the scene in LDS per workgroup */
} gi_scene_info;

typedef struct gi_hit {
    int32_t entity;           /* -1: no hit */
    int32_t u, v;             /* getTextureCoord */
    double point[3], normal[3];
} gi_hit;

/* progressive-display callback: rgb8 rows [y0, y0+rows) of the frame are final */
typedef void (*gi_tile_cb)(void* user, int y0, int rows, const uint8_t* rgb8_rows, const double* rgb_rows);

int gi_abi_version(void);
const char* gi_last_error(void);
/* gfx950 devices visible to this process (0 when there is none). */
int gi_device_count(void);
/* Their HIP device indices (a node may mix architectures): min(count, cap) indices written to out
 * (out may be NULL when cap is 0); returns the count. */
int gi_device_list(int32_t* out, int cap);
/* Provenance: a hash of the kernel and host sources this library was compiled from (build.py
 * passes it at compile time; tests compare it with the sources in the tree). */
const char* gi_build_id(void);

int gi_camera_init(const double pos[3], const double look_at[3], double focal, gi_camera* out);

/* Builds the reference octree and the Mode X acceleration structure on the host and uploads the
 * scene to the current HIP device (the scene is bound to that device). */
int gi_scene_create(const gi_scene_desc* desc, gi_scene** out);
void gi_scene_destroy(gi_scene* scene);
int gi_scene_get_info(const gi_scene* scene, gi_scene_info* info);

/* Renders a w x h frame into host buffers (rgb: w*h*3 fp64, rgb8: w*h*3 RGB888; either may be
 * NULL).  Polls *cancel (if non-NULL) between bands; calls cb (if non-NULL) after each band.
 * Threading: a scene may be used from any host thread; calls on one scene are serialised by the
 * library (a mutex for the host side, and every render of a scene is ordered on the device behind
 * the scene's previous one, whatever stream each was issued on: they share the Mode X work list). */
int gi_render(gi_scene* scene, const gi_camera* cam, const double light[3], int w, int h,
              const gi_opts* opts, double* rgb, uint8_t* rgb8, const volatile int* cancel,
              gi_tile_cb cb, void* user);

/* Device-resident variant, asynchronous on `stream` (hipStream_t; NULL = default stream).
 * shard_count == 1: d_rgb / d_rgb8 are row-major frames.  shard_count > 1: they hold this rank's
 * tiles packed as [gi_shard_tiles(w,h,n)][GI_TILE*GI_TILE][3], tile t = shard_index + k*n. */
int gi_render_device(gi_scene* scene, const gi_camera* cam, const double light[3], int w, int h,
                     const gi_opts* opts, double* d_rgb, uint8_t* d_rgb8, void* stream);

/* Tiles per rank (the packed buffer of every rank has this many tiles, padded). */
int64_t gi_shard_tiles(int w, int h, int shard_count);

/* d_packed: shard_count consecutive per-rank packed buffers (as gathered); writes row-major frames. */
int gi_unshard_device(int w, int h, int shard_count, const double* d_packed, const uint8_t* d_packed8,
                      double* d_rgb, uint8_t* d_rgb8, void* stream);

/* One ray through the Mode R per-pixel body (raytracer.h:43-82) on the device: origin, dir (the
 * Ray ctor normalises it), light.  rgb receives the shaded colour (0 if no hit). */
int gi_trace_ray(gi_scene* scene, const double origin[3], const double dir[3], const double light[3],
                 gi_hit* hit, double rgb[3]);

/* Average duration in ms of the dominant kernel over the scene's renders issued with GI_FLAG_TIME
 * since the previous call (waits for the last one; *n = how many, may be NULL), then resets.
 * GI_ERR_ARG if there was none. */
int gi_scene_kernel_ms(gi_scene* scene, float* avg_ms, int64_t* n);
/* Mode X form a render of `scene` with `opts` would run (bench labels, tests): 0 = the persistent
 * path-state kernel k_mode_x, 1 = the wavefront form (k_wf_bounce once per bounce), 2 = the
 * segment-synchronous form (k_seg); Mode R: 0. */
int gi_scene_x_form(gi_scene* scene, const gi_opts* opts, int32_t* form);
/* Mode R kernel a render of `scene` with `opts` would run (ABI 10; bench labels, tests): 0 = k_mode_r
 * (one lane per pixel: small scenes, GI_FLAG_R_DFS), 1 = the flat phases (k_rf_walk, k_rf_hit,
 * k_rf_scan, k_rf_reach, k_rf_shade; scenes of more than 4096 entities; their overflowed tiles by
 * k_mode_r_batch), 2 = k_mode_r_batch for the whole frame -- also where the flat phases' buffers
 * could not be allocated for the scene's last frame size (not retried for that size or larger).
 * Mode X: 0. */
int gi_scene_r_kernel(gi_scene* scene, const gi_opts* opts, int32_t* kernel);

/* ---- host-side reference octree (no device needed) --------------------------------------------
 * gi_octree_create builds the reference octree from the same descriptors as gi_scene_create (push
 * order, node boxes, lost entities A.6, silent drop A.14 -- bit for bit the reference's tree).
 * gi_octree_intersect returns Octree::intersect(Ray(origin, dir))'s candidate list: DFS over the
 * children 0..7, a child skipped when its list is empty (octree.h:140), else tested by the ExpBox
 * node test (A.4) and descended; leaves contribute their lists; duplicates kept.  `dir` is used as
 * given (the reference's Ray ctor has already normalised it, ray.h:6).  Entity indices are push
 * order; min(*n, cap) of them are written to out, *n = the full length. */
typedef struct gi_octree gi_octree;
int gi_octree_create(const gi_scene_desc* desc, gi_octree** out);
void gi_octree_destroy(gi_octree* octree);
int gi_octree_intersect(const gi_octree* octree, const double origin[3], const double dir[3], int32_t* out,
                        int64_t cap, int64_t* n);

/* ---- several GPUs of one process ------------------------------------------------------------
 * gi_multi_create: n_shards >= 1 shards, shard i rendered on HIP device devices[i] (duplicates
 * allowed: several shards on one device render one after the other).  devices[0] is the root that
 * assembles the frame.  The frame's 8x8 tiles are dealt round-robin over the shards (tile t ->
 * shard t % n_shards, as gi_render_device's shard_count/shard_index); each shard renders its tiles
 * into a packed buffer on its device, and one RCCL group of ncclSend/ncclRecv (rccl.h:700-725;
 * librccl is loaded when a second device is used) brings them to the root over xGMI, where
 * gi_unshard_device's kernel reassembles the frame.  Shards on the root device need no copy.
 * gi_multi_render: as gi_render (bands, cancel, callback, host buffers); opts->shard_count and
 * shard_index must be 1 and 0 (the multi handle does the sharding).  Results are bit-identical to
 * gi_render on one device. */
typedef struct gi_multi gi_multi;
int gi_multi_create(const gi_scene_desc* desc, int n_shards, const int* devices, gi_multi** out);
void gi_multi_destroy(gi_multi* multi);
int gi_multi_info(const gi_multi* multi, int* n_shards, int* n_devices, int* uses_rccl);
int gi_multi_render(gi_multi* multi, const gi_camera* cam, const double light[3], int w, int h, const gi_opts* opts,
                    double* rgb, uint8_t* rgb8, const volatile int* cancel, gi_tile_cb cb, void* user);

/* ---- scene I/O --------------------------------------------------------------------------------
 * gi_obj_parse: Wavefront OBJ text (len bytes, need not be terminated) -> GI_IMP_TRIANGLE
 * descriptors, one per triangle of each face's fan (v0, v_k, v_k+1) in file order, args = the three
 * vertices.  Each descriptor is a copy of *tmpl (its material fields; NULL: zeroed, i.e. the
 * reference's default ImpTriangle material) with kind and args set.  Accepts v (extra values
 * ignored), f with i, i/t, i//n, i/t/n references (1-based, negative = relative), comments and
 * '\' continuations; vt, vn, vp, o, g, s, usemtl, mtllib, l, p are skipped.  min(*n, cap)
 * descriptors are written to out, *n = the full count (call with cap = 0 to size the buffer).
 * GI_ERR_ARG with the line number on a malformed v / f line or a vertex reference out of range. */
int gi_obj_parse(const char* text, int64_t len, const gi_entity_desc* tmpl, gi_entity_desc* out, int64_t cap,
                 int64_t* n);

/* Known-answer hook: the device's ExpBox node test (entities.h:379-440 as octree.h:141-146 uses
 * it) over n host records (min[3], max[3], origin[3], dir[3]); out[i] = 0/1. */
int gi_kat_expbox(int n, const double* recs, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* GI_H_ */
