// gi_capi.cpp — the extern "C" boundary (include/gi.h).  Host-side only: validates arguments,
// builds the scene (gi_build.cpp), owns its HBM copy, and launches the gfx950 kernels
// (gi_kernels.hip).  There is no CPU rendering path: without a gfx950 device every render fails.
// No exception crosses the boundary: every entry point that can allocate runs inside guard(),
// which maps std::bad_alloc to GI_ERR_NOMEM and anything else to GI_ERR_INTERNAL.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "gi.h"
#include "gi_internal.h"
#include "gi_scene.h"

namespace gi {
bool build_host_scene(const gi_scene_desc& desc, HostScene& hs, std::string& err);
long long shard_tiles(int w, int h, int shard_count);
hipError_t x_launch_config(const DevScene& sc, int device, XLaunchCfg& cfg);
int x_form_choice(const DevScene& sc, const XLaunchCfg& xc, const gi_opts& o);
long long x_wf_chunk();
int x_env_rf_per_slot();
int r_kernel_choice(const DevScene& sc, const gi_opts& o);
unsigned rf_own_pairs();
unsigned rf_page_pairs();
unsigned rf_max_pages();
unsigned rf_seg_pairs();
hipError_t launch_render(const DevScene& sc, const XLaunchCfg& xc, const CamDev& cam, V3 light, int w, int h, int y0,
                         const gi_opts& o, double* rgb, uint8_t* rgb8, const XScratch& xs, KTimer* kt,
                         hipStream_t stream);
hipError_t launch_unshard(int w, int h, int shard_count, const double* packed, const uint8_t* packed8, double* rgb,
                          uint8_t* rgb8, hipStream_t stream);
hipError_t launch_trace_ray(const DevScene& sc, V3 o, V3 d, V3 light, int32_t* out_i, double* out_d, hipStream_t stream);
hipError_t launch_box_kat(int n, const double* recs, int32_t* out, hipStream_t stream);
}  // namespace gi

using namespace gi;

// gi_render's band pipeline, owned by the scene handle and created on first use: band i renders
// into device slot i % 2 on `render` while band i-1 is copied to pinned staging on `copy`; the
// host then copies a finished band into the caller's buffers (or hands the staging to the
// callback).  Slots are reused only after their copy has completed (event `copied`).
struct HostPath {
    static constexpr int kSlots = 2;
    hipStream_t render = nullptr, copy = nullptr;
    hipEvent_t rendered[kSlots] = {}, copied[kSlots] = {};
    double* d_rgb[kSlots] = {};
    uint8_t* d_rgb8[kSlots] = {};
    double* h_rgb[kSlots] = {};    // pinned
    uint8_t* h_rgb8[kSlots] = {};  // pinned
    size_t cap_px = 0;             // pixels per slot
    int n_alloc = 0;               // slots allocated (1 for whole-frame renders)
};

struct gi_scene {
    HostScene host;
    DevScene dev;
    XLaunchCfg xcfg;   // Mode X launch configuration on this scene's device
    std::vector<void*> allocs;
    XScratch xs;       // Mode X work list + per-sample radiance, grown on demand
    KTimer kt;         // GI_FLAG_TIME events
    HostPath hp;       // gi_render's band pipeline (streams, device band slots, pinned staging)
    // every render launch of this scene waits on the device for the previous one (they share xs
    // and the work counters), whatever stream each is issued on
    hipEvent_t last = nullptr;
    bool launched = false;
    uint64_t prog_key = 0;   // progressive passes: the frame's key and the next pass's sample_begin
    int prog_next = -1;
    std::mutex mu;     // host-side calls on one scene are serialised
    int device = -1;
    int64_t bytes = 0;
};

struct gi_octree {
    HostScene host;
};

namespace {
thread_local std::string g_err;

int fail(int code, const char* msg) noexcept {
    try {
        g_err = msg;
    } catch (...) {
        // the message is best effort; the status code is what the caller acts on
    }
    return code;
}
int fail(int code, const std::string& msg) noexcept { return fail(code, msg.c_str()); }
int hip_fail(hipError_t e, const char* what) noexcept {
    try {
        return fail(GI_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    } catch (...) {
        return GI_ERR_DEVICE;
    }
}

template <typename T>
hipError_t upload(gi_scene* s, const std::vector<T>& v, const T** out) {
    *out = nullptr;
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) return e;
    s->allocs.push_back(p);
    s->bytes += (int64_t)bytes;
    if (!v.empty()) {
        e = hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
        if (e != hipSuccess) return e;
    }
    *out = static_cast<const T*>(p);
    return hipSuccess;
}

void free_rflat(XScratch& x) {
    for (void* p : {(void*)x.rf_pairs, (void*)x.rf_pt, (void*)x.rf_best, (void*)x.rf_dir, (void*)x.rf_cnt, (void*)x.rf_ovf,
                    (void*)x.rf_rcnt, (void*)x.rf_soff, (void*)x.rf_shc, (void*)x.rf_sreg, (void*)x.rf_hoff})
        (void)hipFree(p);
    x.rf_pairs = x.rf_pt = x.rf_cnt = x.rf_ovf = x.rf_rcnt = x.rf_soff = x.rf_shc = x.rf_sreg = x.rf_hoff = nullptr;
    x.rf_best = nullptr;
    x.rf_dir = nullptr;
    x.rf_pages = 0;
    x.rf_slots = 0;
    x.rf_bytes = 0;
}

// Mode X work buffers for a frame of w x h pixels cut into this call's shard (k_x_classify's list,
// k_mode_x's per-sample radiance for spp > 1); grown, never shrunk.  hipFree synchronises with
// work still using them.
int ensure_xscratch(gi_scene* s, int w, int h, const gi_opts* o) {
    const long long need = shard_tiles(w, h, o->shard_count) * GI_TILE * GI_TILE;
    hipError_t e;
    if (o->mode == GI_MODE_R) {
        // the flat Mode R phases' buffers, only when this launch runs them (r_kernel_choice == 1).
        // Pairs are one word: per tile its own GI_RF_S0 (8 per pixel slot), plus a shared pool of
        // GI_RF_PER_SLOT (16) per pixel slot in pages; with the per-slot directions and best ranks a
        // 1080p frame takes 0.28 GB (R-C4 writes 5.0 M pairs: 20 MB).  A tile whose candidates do not
        // fit is rendered by k_mode_r_batch; if the buffers cannot be had at all, the whole frame is.
        XScratch& x = s->xs;
        if (r_kernel_choice(s->dev, *o) == 1 && x.rf_slots < need && !(x.rf_failed > 0 && need >= x.rf_failed)) {
            free_rflat(x);
            const hipError_t prior = hipPeekAtLastError();   // (a caller's unchecked error is left as it was)
            const long long tiles = need / 64;
            const long long pages = (long long)x_env_rf_per_slot() * need / (long long)rf_page_pairs();
            const size_t pairs = (size_t)tiles * rf_own_pairs() + (size_t)pages * rf_page_pairs();
            // segments of k_rf_hit: a tile's pairs cut every rf_seg_pairs(), so at most one per tile
            // plus one per rf_seg_pairs() of the buffer
            const size_t segs = (size_t)tiles + pairs / rf_seg_pairs() + 1;
            const bool ok =
                hipMalloc((void**)&x.rf_pairs, pairs * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_pt, (size_t)tiles * rf_max_pages() * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_best, (size_t)need * sizeof(unsigned long long)) == hipSuccess &&
                hipMalloc((void**)&x.rf_dir, (size_t)need * 3 * sizeof(double)) == hipSuccess &&
                hipMalloc((void**)&x.rf_cnt, 8 * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_ovf, (size_t)tiles * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_rcnt, (size_t)tiles * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_soff, (size_t)(tiles + 1) * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_shc, (size_t)segs * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_sreg, (size_t)segs * sizeof(unsigned)) == hipSuccess &&
                hipMalloc((void**)&x.rf_hoff, (size_t)(segs + 1) * sizeof(unsigned)) == hipSuccess;
            if (!ok) {   // rendered by k_mode_r_batch (gi_scene_r_kernel reports 2); not retried per frame
                if (prior == hipSuccess) (void)hipGetLastError();   // (clears this allocation's error only)
                free_rflat(x);
                x.rf_failed = need;
                return GI_OK;
            }
            x.rf_failed = 0;
            x.rf_pages = (unsigned)pages;
            x.rf_slots = need;
            x.rf_bytes = pairs * sizeof(unsigned) + (size_t)tiles * (rf_max_pages() + 4) * sizeof(unsigned) + segs * 12 +
                         (size_t)need * (sizeof(unsigned long long) + 3 * sizeof(double));
        }
        return GI_OK;
    }
    if (o->mode != GI_MODE_X) return GI_OK;
    if ((unsigned long long)need >= 0xFFFFFFFFull) return fail(GI_ERR_ARG, "mode X frame too large: 2^32 pixel slots");
    XScratch& x = s->xs;
    if (x.cap < need) {
        (void)hipFree(x.list);
        (void)hipFree(x.part);
        x.list = nullptr;
        x.part = nullptr;
        x.cap = 0;
        x.spp = 0;
        if ((e = hipMalloc((void**)&x.list, (size_t)need * sizeof(unsigned))) != hipSuccess) return hip_fail(e, "hipMalloc (work list)");
        x.cap = need;
    }
    if (o->spp > 1 && x.spp < o->spp) {
        (void)hipFree(x.part);
        x.part = nullptr;
        x.spp = 0;
        if ((e = hipMalloc((void**)&x.part, (size_t)o->spp * (size_t)x.cap * 3 * sizeof(double))) != hipSuccess)
            return hip_fail(e, "hipMalloc (per-sample radiance)");
        x.spp = o->spp;
    }
    const int form = x_form_choice(s->dev, s->xcfg, *o);
    if (form) {   // wavefront forms: counters; form 1 also path queues sized to a chunk of units
        const long long want = std::max(64ll, std::min(x_wf_chunk(), need * (long long)o->spp));
        if (!x.wcnt) {
            if ((e = hipMalloc((void**)&x.wcnt, 2 * 64 * sizeof(unsigned))) != hipSuccess) return hip_fail(e, "hipMalloc (wavefront counters)");
        }
        if (form == 1 && x.wcap < want) {
            for (int q = 0; q < 2; ++q) {
                (void)hipFree(x.wq[q]);
                (void)hipFree(x.wid[q]);
                x.wq[q] = nullptr;
                x.wid[q] = nullptr;
            }
            x.wcap = 0;
            for (int q = 0; q < 2; ++q) {
                if ((e = hipMalloc((void**)&x.wq[q], (size_t)want * 12 * sizeof(double))) != hipSuccess ||
                    (e = hipMalloc((void**)&x.wid[q], (size_t)want * 2 * sizeof(unsigned))) != hipSuccess)
                    return hip_fail(e, "hipMalloc (wavefront path queues)");
            }
            x.wcap = want;
        }
    }
    return GI_OK;
}

// folds ring slot i (its end event has been recorded) into the running sum
hipError_t fold_timer(KTimer& kt, int i) {
    hipError_t e = hipEventSynchronize(static_cast<hipEvent_t>(kt.ev1[i]));
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, static_cast<hipEvent_t>(kt.ev0[i]), static_cast<hipEvent_t>(kt.ev1[i]));
    if (e == hipSuccess) { kt.sum_ms += ms; kt.folded++; }
    return e;
}

// GI_FLAG_TIME: create the event ring on first use; fold the pair the next launch will reuse
int ensure_timer(gi_scene* s, const gi_opts* o) {
    if (!(o->flags & GI_FLAG_TIME)) return GI_OK;
    KTimer& kt = s->kt;
    if (!kt.ev0[0]) {
        for (int i = 0; i < KTimer::kRing; i++) {
            hipEvent_t a = nullptr, b = nullptr;
            hipError_t e = hipEventCreate(&a);
            if (e == hipSuccess) e = hipEventCreate(&b);
            if (e != hipSuccess) {
                if (a) (void)hipEventDestroy(a);
                return hip_fail(e, "hipEventCreate");
            }
            kt.ev0[i] = a;
            kt.ev1[i] = b;
        }
    }
    if (kt.recorded >= KTimer::kRing) {
        const hipError_t e = fold_timer(kt, (int)(kt.recorded % KTimer::kRing));
        if (e != hipSuccess) return hip_fail(e, "timer event");
    }
    return GI_OK;
}

// One render launch of scene s on `stream`, ordered behind the scene's previous launch.
int issue_render(gi_scene* s, const CamDev& cd, V3 light, int w, int h, int y0, const gi_opts& o, double* d_rgb,
                 uint8_t* d_rgb8, hipStream_t stream, bool timer) {
    hipError_t e = hipSuccess;
    if (!s->last && (e = hipEventCreateWithFlags(&s->last, hipEventDisableTiming)) != hipSuccess)
        return hip_fail(e, "hipEventCreate");
    if (s->launched && (e = hipStreamWaitEvent(stream, s->last, 0)) != hipSuccess) return hip_fail(e, "hipStreamWaitEvent");
    e = launch_render(s->dev, s->xcfg, cd, light, w, h, y0, o, d_rgb, d_rgb8, s->xs, timer ? &s->kt : nullptr, stream);
    if (e != hipSuccess) return hip_fail(e, "render launch");
    if ((e = hipEventRecord(s->last, stream)) != hipSuccess) return hip_fail(e, "hipEventRecord");
    s->launched = true;
    return GI_OK;
}

void free_hostpath_buffers(HostPath& hp) {
    for (int i = 0; i < HostPath::kSlots; i++) {
        (void)hipFree(hp.d_rgb[i]);
        (void)hipFree(hp.d_rgb8[i]);
        (void)hipHostFree(hp.h_rgb[i]);
        (void)hipHostFree(hp.h_rgb8[i]);
        hp.d_rgb[i] = nullptr;
        hp.d_rgb8[i] = nullptr;
        hp.h_rgb[i] = nullptr;
        hp.h_rgb8[i] = nullptr;
    }
    hp.cap_px = 0;
    hp.n_alloc = 0;
}

// streams and events on first use; `slots` band slots of `px` pixels (grown, never shrunk)
int ensure_hostpath(gi_scene* s, size_t px, int slots) {
    HostPath& hp = s->hp;
    hipError_t e = hipSuccess;
    if (!hp.render) {
        if ((e = hipStreamCreateWithFlags(&hp.render, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
        if ((e = hipStreamCreateWithFlags(&hp.copy, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
        for (int i = 0; i < HostPath::kSlots; i++) {
            if ((e = hipEventCreateWithFlags(&hp.rendered[i], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&hp.copied[i], hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        }
    }
    if (hp.cap_px < px || hp.n_alloc < slots) {
        px = std::max(px, hp.cap_px);
        slots = std::max(slots, hp.n_alloc);
        free_hostpath_buffers(hp);
        for (int i = 0; i < slots; i++) {
            if ((e = hipMalloc((void**)&hp.d_rgb[i], px * 3 * sizeof(double))) != hipSuccess ||
                (e = hipMalloc((void**)&hp.d_rgb8[i], px * 3)) != hipSuccess ||
                (e = hipHostMalloc((void**)&hp.h_rgb[i], px * 3 * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
                (e = hipHostMalloc((void**)&hp.h_rgb8[i], px * 3, hipHostMallocDefault)) != hipSuccess) {
                free_hostpath_buffers(hp);
                return hip_fail(e, "band buffers");
            }
        }
        hp.cap_px = px;
        hp.n_alloc = slots;
    }
    return GI_OK;
}

void destroy_scene(gi_scene* s) noexcept {
    if (!s) return;
    if (s->device >= 0) (void)hipSetDevice(s->device);
    HostPath& hp = s->hp;
    if (hp.render) (void)hipStreamSynchronize(hp.render);
    if (hp.copy) (void)hipStreamSynchronize(hp.copy);
    if (s->last) (void)hipEventSynchronize(s->last);
    for (void* p : s->allocs) (void)hipFree(p);
    (void)hipFree(s->xs.list);
    (void)hipFree(s->xs.part);
    for (int q = 0; q < 2; ++q) {
        (void)hipFree(s->xs.wq[q]);
        (void)hipFree(s->xs.wid[q]);
    }
    (void)hipFree(s->xs.wcnt);
    free_rflat(s->xs);
    for (int i = 0; i < KTimer::kRing; i++) {
        if (s->kt.ev0[i]) (void)hipEventDestroy(static_cast<hipEvent_t>(s->kt.ev0[i]));
        if (s->kt.ev1[i]) (void)hipEventDestroy(static_cast<hipEvent_t>(s->kt.ev1[i]));
    }
    free_hostpath_buffers(hp);
    for (int i = 0; i < HostPath::kSlots; i++) {
        if (hp.rendered[i]) (void)hipEventDestroy(hp.rendered[i]);
        if (hp.copied[i]) (void)hipEventDestroy(hp.copied[i]);
    }
    if (hp.render) (void)hipStreamDestroy(hp.render);
    if (hp.copy) (void)hipStreamDestroy(hp.copy);
    if (s->last) (void)hipEventDestroy(s->last);
    delete s;
}

// host-side reference octree query: Octree::intersect -> Node::intersect (octree.h:46-68, 132-155)
void octree_query(const HostScene& h, int ni, V3 o, V3 d, std::vector<int32_t>& out) {
    const RNode& nd = h.rnodes[(size_t)ni];
    if (nd.child0 < 0) {   // leaf: a copy of its list (octree.h:133-135)
        out.insert(out.end(), h.leaf_ents.begin() + nd.ent_off, h.leaf_ents.begin() + nd.ent_off + nd.ent_cnt);
        return;
    }
    for (int c = 0; c < 8; ++c) {   // children 0..7 (octree.h:139-152)
        const RNode& ch = h.rnodes[(size_t)nd.child0 + c];
        if (ch.ent_cnt == 0) continue;   // octree.h:140
        if (box_hit(ld3(ch.mn), ld3(ch.mx), o, d)) octree_query(h, nd.child0 + c, o, d, out);
    }
}

}  // namespace

// ---- internal entry points shared with gi_multi.cpp (gi_internal.h) -------------------------
namespace gi {

int error(int code, const std::string& msg) noexcept { return fail(code, msg); }
int hip_error(hipError_t e, const char* what) noexcept { return hip_fail(e, what); }

int bind_device(int device) {
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    if (cur != device) {
        e = hipSetDevice(device);
        if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    }
    return GI_OK;
}

int check_device(int dev) {
    hipDeviceProp_t prop;
    const hipError_t e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(GI_ERR_DEVICE, std::string("device ") + std::to_string(dev) + " is " + prop.gcnArchName +
                                       ", libgi is built for gfx950 only");
    return GI_OK;
}

// raytracer.h:26-30: camera basis and the frame's top-left (vertical offset uses w)
CamDev make_cam(const gi_camera& c, int w) {
    CamDev d;
    d.pos = v3(c.pos[0], c.pos[1], c.pos[2]);
    d.up = v3(c.up[0], c.up[1], c.up[2]);
    const V3 fwd = v3(c.forward[0], c.forward[1], c.forward[2]);
    d.rx = 0.0002;
    d.ry = 0.0002;
    d.left = normalize(cross(d.up, fwd));
    d.top_left = (((d.pos + c.focal * fwd) + ((d.left * (double)w) * 0.5) * d.rx) + ((d.up * (double)w) * 0.5) * d.ry) - d.pos;
    return d;
}

int check_opts(int w, int h, const gi_opts* o) {
    if (!o) return fail(GI_ERR_ARG, "null opts");
    if (w <= 0 || h <= 0 || (int64_t)w * h > (int64_t)1 << 34) return fail(GI_ERR_ARG, "bad frame size");
    if (o->mode != GI_MODE_R && o->mode != GI_MODE_X) return fail(GI_ERR_ARG, "bad mode");
    if (o->shard_count < 1 || o->shard_index < 0 || o->shard_index >= o->shard_count) return fail(GI_ERR_ARG, "bad shard");
    if (o->mode == GI_MODE_X && (o->spp < 1 || o->depth < 1 || o->depth > 0xFFFF))
        return fail(GI_ERR_ARG, "mode X needs spp >= 1, 1 <= depth <= 65535");
    if ((o->flags & GI_FLAG_STATS) && !o->stats) return fail(GI_ERR_ARG, "GI_FLAG_STATS without stats buffer");
    if ((o->sample_begin != 0 || o->sample_end != 0) &&
        (o->mode != GI_MODE_X || o->spp < 2 || o->sample_begin < 0 || o->sample_begin >= o->sample_end || o->sample_end > o->spp))
        return fail(GI_ERR_ARG, "progressive pass: mode X, spp > 1, 0 <= sample_begin < sample_end <= spp");
    return GI_OK;
}

// Progressive passes (gi_opts sample_begin / sample_end) continue one frame on one scene: the first
// pass (sample_begin 0) records the frame's key, a later one must match it and start where the
// previous pass ended.  Any other render of the scene ends the frame.
uint64_t prog_key(const gi_camera& c, const double light[3], int w, int h, const gi_opts& o) {
    uint64_t k = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; ++i) k = (k ^ static_cast<const unsigned char*>(p)[i]) * 1099511628211ull;
    };
    mix(&c, sizeof c);
    mix(light, 3 * sizeof(double));
    const int64_t v[8] = {w, h, o.spp, o.depth, (int64_t)o.seed, o.shard_count, o.shard_index,
                          (int64_t)(o.flags & ~(GI_FLAG_STATS | GI_FLAG_TIME))};
    mix(v, sizeof v);
    return k;
}
int prog_check(gi_scene* s, const gi_camera& c, const double light[3], int w, int h, const gi_opts& o) {
    if (o.sample_end == 0) {
        s->prog_next = -1;
        return GI_OK;
    }
    const uint64_t key = prog_key(c, light, w, h, o);
    if (o.sample_begin > 0 && s->prog_next == o.sample_begin && s->launched) {
        // the previous pass was accepted when issued: a device error since ends the frame
        const hipError_t e = hipEventQuery(s->last);
        if (e != hipSuccess && e != hipErrorNotReady) {
            s->prog_next = -1;
            return hip_fail(e, "progressive pass: the previous pass failed on the device; restart the frame at sample 0");
        }
    }
    if (o.sample_begin > 0 && (s->prog_next != o.sample_begin || s->prog_key != key)) {
        s->prog_next = -1;
        return fail(GI_ERR_ARG, "progressive pass out of order: a pass continues the previous pass's frame "
                                "(same camera, light, size, spp, depth, seed, shard) from its sample_end");
    }
    s->prog_key = key;
    s->prog_next = -1;   // set once this pass has been issued
    return GI_OK;
}
void prog_done(gi_scene* s, const gi_opts& o) {
    s->prog_next = (o.sample_end > 0 && o.sample_end < o.spp) ? o.sample_end : -1;
}

int band_rows_of(const gi_opts* o, int h) {
    int band = o->band_rows > 0 ? o->band_rows : h;
    band = ((band + GI_TILE - 1) / GI_TILE) * GI_TILE;
    return std::min(band, ((h + GI_TILE - 1) / GI_TILE) * GI_TILE);
}

// Builds the scene on the host and uploads it to `device` (made current).
int scene_create_on(const gi_scene_desc* desc, int device, gi_scene** out) {
    *out = nullptr;
    int rc = bind_device(device);
    if (rc || (rc = check_device(device))) return rc;
    std::unique_ptr<gi_scene, void (*)(gi_scene*)> s(new gi_scene(), [](gi_scene* p) { destroy_scene(p); });
    s->device = device;
    std::string err;
    if (!build_host_scene(*desc, s->host, err)) return fail(GI_ERR_SCENE, err);
    DevScene& d = s->dev;
    memset(&d, 0, sizeof d);
    const HostScene& h = s->host;
    hipError_t e;
    gi_scene* sp = s.get();
    if ((e = upload(sp, h.rnodes, &d.rnodes)) != hipSuccess || (e = upload(sp, h.leaf_ents, &d.leaf_ents)) != hipSuccess ||
        (e = upload(sp, h.ents, &d.ents)) != hipSuccess || (e = upload(sp, h.tris, &d.tris)) != hipSuccess ||
        (e = upload(sp, h.xwnodes, &d.xwnodes)) != hipSuccess || (e = upload(sp, h.xhot, &d.xhot)) != hipSuccess ||
        (e = upload(sp, h.xbox, &d.xbox)) != hipSuccess ||
        (e = upload(sp, h.xprims, &d.xprims)) != hipSuccess ||
        (e = upload(sp, std::vector<unsigned>(16, 0u), const_cast<const unsigned**>(&d.work))) != hipSuccess ||
        (e = upload(sp, h.app_off, &d.app_off)) != hipSuccess || (e = upload(sp, h.app_rec, &d.app_rec)) != hipSuccess ||
        (e = upload(sp, h.rpath_rec, &d.rpath_rec)) != hipSuccess || (e = upload(sp, h.rc_nodes, &d.rc_nodes)) != hipSuccess ||
        (e = upload(sp, h.rc_ent, &d.rc_ent)) != hipSuccess || (e = upload(sp, h.rc_maxkey, &d.rc_maxkey)) != hipSuccess ||
        (e = upload(sp, h.r_always, &d.r_always)) != hipSuccess ||
        (e = upload(sp, h.r_leaf_of_rank, &d.r_leaf_of_rank)) != hipSuccess)
        return hip_fail(e, "scene upload");
    d.n_rnodes = (int32_t)h.rnodes.size();
    d.n_ents = (int32_t)h.ents.size();
    d.n_xwnodes = (int32_t)h.xwnodes.size();
    d.n_xprims = (int32_t)h.xprims.size();
    d.x_max_depth = h.x_max_depth;
    d.x_handle8 = h.x_handle8;
    d.x_flags = h.x_flags;
    d.x_skip_a = h.x_skip_a;
    d.x_skip_b = h.x_skip_b;
    d.n_xhot = (int32_t)h.xhot.size();
    d.n_r_always = (int32_t)h.r_always.size();
    d.rc_ext = (float)h.rc_ext;
    {   // LDS-resident traversal + shading records for small scenes (<= 40 KB per workgroup: three
        // 256-thread workgroups per CU stay resident within the CU's 160 KB of LDS)
        const size_t bytes = h.xwnodes.size() * sizeof(XWNode) + h.xhot.size() * sizeof(XHot) +
                             h.xprims.size() * sizeof(XPrim) + h.ents.size() * sizeof(REnt);
        d.x_lds_bytes = bytes <= 40 * 1024 ? (int32_t)bytes : 0;
        // light shading (no acos texture mapping, no sphere primitives): 4 waves per SIMD pay off,
        // provided four workgroups fit a CU's 160 KB: each holds the scene, the per-lane path slots
        // (256 lanes x 80 B) and the per-wave unit blocks (4 x 68 x 4 B)
        const size_t per_wg = bytes + 256 * 10 * sizeof(double) + 4 * 68 * sizeof(unsigned);
        d.x_waves4 = (d.x_lds_bytes > 0 && 4 * per_wg <= 160 * 1024) ? 1 : 0;
        d.x_tri_only = 1;
        for (const REnt& r : h.ents)
            if (r.kind == K_IMP_SPHERE || r.kind == K_EXP_SPHERE || r.kind == K_EXP_CONE || r.kind == K_EXP_RECTANGLE) {
                d.x_waves4 = 0;
                d.x_tri_only = 0;
            }
        for (const XPrim& xp : h.xprims)
            if (xp.kind != 0) d.x_tri_only = 0;
        d.r_tri_only = 1;
        for (const REnt& r : h.ents)
            if (r.kind != K_IMP_TRIANGLE) d.r_tri_only = 0;
    }
    // HBM-resident scenes whose XWNode tree outgrows an XCD's L2 share (> 2 MB) traverse quantised
    // nodes (XCNode: one 128-byte line per node instead of two): C5 287 -> 270 ms; the 1k soup, whose
    // 84 KB tree stays in L2 anyway, pays the decoding (+6%) and keeps XWNode.
    const bool want_cn = h.xwnodes.size() * sizeof(XWNode) > (size_t)2 << 20;
    if (d.x_lds_bytes == 0 && want_cn && encode_xcnodes(h.xwnodes, s->host.xcnodes) &&
        (e = upload(sp, h.xcnodes, &d.xcnodes)) != hipSuccess)
        return hip_fail(e, "scene upload (quantised nodes)");
    for (int k = 0; k < 3; ++k) { d.root_lo[k] = INFINITY; d.root_hi[k] = -INFINITY; }
    if (!h.xwnodes.empty())
        for (int c = 0; c < 8; ++c)
            if (h.xwnodes[0].child[c] != XEMPTY)
                for (int k = 0; k < 3; ++k) {
                    d.root_lo[k] = std::min(d.root_lo[k], h.xwnodes[0].lo[k][c]);
                    d.root_hi[k] = std::max(d.root_hi[k], h.xwnodes[0].hi[k][c]);
                }
    if ((e = x_launch_config(d, device, s->xcfg)) != hipSuccess) return hip_fail(e, "occupancy query");
    *out = s.release();
    return GI_OK;
}

void scene_destroy(gi_scene* s) noexcept { destroy_scene(s); }
int scene_device(const gi_scene* s) { return s->device; }
std::mutex& scene_mutex(gi_scene* s) { return s->mu; }

// Asynchronous render of a band (rows [y0, y0 + h) of a frame w pixels wide; the whole frame for
// y0 = 0, h = its height) or of one shard of it, into device buffers on `stream`.
int scene_render_band(gi_scene* s, const CamDev& cd, const double light[3], int w, int h, int y0, const gi_opts& o,
                      double* d_rgb, uint8_t* d_rgb8, hipStream_t stream, bool timer) {
    int rc = bind_device(s->device);
    if (rc || (rc = ensure_xscratch(s, w, h, &o)) || (timer && (rc = ensure_timer(s, &o)))) return rc;
    return issue_render(s, cd, v3(light[0], light[1], light[2]), w, h, y0, o, d_rgb, d_rgb8, stream, timer);
}

int unshard(int w, int h, int n, const double* packed, const uint8_t* packed8, double* rgb, uint8_t* rgb8,
            hipStream_t stream) {
    const hipError_t e = launch_unshard(w, h, n, packed, packed8, rgb, rgb8, stream);
    return e == hipSuccess ? GI_OK : hip_fail(e, "unshard launch");
}

}  // namespace gi

extern "C" {

int gi_abi_version(void) { return GI_ABI_VERSION; }
const char* gi_last_error(void) { return g_err.c_str(); }

int gi_device_list(int32_t* out, int cap) {
    int ndev = 0, n = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return 0;
    for (int d = 0; d < ndev; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) {
            if (out && n < cap) out[n] = d;
            ++n;
        }
    }
    return n;
}

int gi_device_count(void) { return gi_device_list(nullptr, 0); }

#ifndef GI_BUILD_ID
#define GI_BUILD_ID "unknown"
#endif
const char* gi_build_id(void) { return GI_BUILD_ID; }

int gi_camera_init(const double pos[3], const double look_at[3], double focal, gi_camera* out) {
    if (!pos || !look_at || !out) return fail(GI_ERR_ARG, "null argument");
    // Camera(pos, lookAt, focal) (camera.h:8-10): up = (0,0,1); forward = normalize(lookAt - pos)
    const V3 p = v3(pos[0], pos[1], pos[2]);
    const V3 f = normalize(v3(look_at[0], look_at[1], look_at[2]) - p);
    st3(out->pos, p);
    out->up[0] = 0; out->up[1] = 0; out->up[2] = 1.0;
    st3(out->forward, f);
    out->focal = focal;
    return GI_OK;
}

int gi_scene_create(const gi_scene_desc* desc, gi_scene** out) {
    return guard([&]() -> int {
        if (!desc || !out || desc->n_entities < 0 || (desc->n_entities > 0 && !desc->entities))
            return fail(GI_ERR_ARG, "bad scene descriptor");
        *out = nullptr;
        int ndev = 0;
        hipError_t e = hipGetDeviceCount(&ndev);
        if (e != hipSuccess || ndev <= 0) return fail(GI_ERR_DEVICE, "no HIP device (libgi renders only on gfx950)");
        int dev = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return hip_fail(e, "hipGetDevice");
        return scene_create_on(desc, dev, out);
    });
}

void gi_scene_destroy(gi_scene* s) { destroy_scene(s); }

int gi_scene_get_info(const gi_scene* s, gi_scene_info* info) {
    if (!s || !info) return fail(GI_ERR_ARG, "null argument");
    info->n_entities = (int32_t)s->host.ents.size();
    info->n_nodes = (int32_t)s->host.rnodes.size();
    info->n_leaves = s->host.n_leaves;
    info->max_depth = s->host.max_depth;
    info->n_reachable = s->host.n_reachable;
    info->n_dropped = s->host.n_dropped;
    info->x_nodes = (int32_t)(s->host.xnodes.empty() ? s->host.xwnodes.size() : s->host.xnodes.size());
    info->x_prims = (int32_t)s->host.xprims.size();
    info->device_bytes = s->bytes;
    info->x_node_bytes = s->dev.xcnodes ? (int32_t)sizeof(XCNode) : (int32_t)sizeof(XWNode);
    info->x_lds_resident = s->dev.x_lds_bytes > 0 ? 1 : 0;
    return GI_OK;
}

int64_t gi_shard_tiles(int w, int h, int shard_count) {
    if (w <= 0 || h <= 0 || shard_count < 1) return -1;
    return shard_tiles(w, h, shard_count);
}

int gi_render_device(gi_scene* s, const gi_camera* cam, const double light[3], int w, int h, const gi_opts* o,
                     double* d_rgb, uint8_t* d_rgb8, void* stream) {
    return guard([&]() -> int {
        DeviceRestore keep;   // the caller's current device, restored on return
        if (!s) return fail(GI_ERR_ARG, "null scene");
        int rc = check_opts(w, h, o);
        if (rc) return rc;
        if (!cam || !light) return fail(GI_ERR_ARG, "null camera or light");
        std::lock_guard<std::mutex> lk(s->mu);
        if ((rc = prog_check(s, *cam, light, w, h, *o))) return rc;
        rc = scene_render_band(s, make_cam(*cam, w), light, w, h, 0, *o, d_rgb, d_rgb8, static_cast<hipStream_t>(stream),
                               true);
        if (rc == GI_OK) prog_done(s, *o);
        return rc;
    });
}

int gi_render(gi_scene* s, const gi_camera* cam, const double light[3], int w, int h, const gi_opts* o, double* rgb,
              uint8_t* rgb8, const volatile int* cancel, gi_tile_cb cb, void* user) {
    return guard([&]() -> int {
        DeviceRestore keep;   // the caller's current device, restored on return
        if (!s) return fail(GI_ERR_ARG, "null scene");
        int rc = check_opts(w, h, o);
        if (rc) return rc;
        if (!cam || !light) return fail(GI_ERR_ARG, "null camera or light");
        if (o->shard_count != 1) return fail(GI_ERR_ARG, "gi_render renders whole frames; use gi_render_device or gi_multi to shard");
        std::lock_guard<std::mutex> lk(s->mu);
        if ((rc = bind_device(s->device))) return rc;
        // progressive bands of whole tile rows (the reference fills rows in order, raytracer.h:32-33,
        // and the Viewer repaints what is done, viewer.h:18-21); cancel is polled between bands.
        const int band = band_rows_of(o, h);
        const size_t band_px = (size_t)w * (size_t)band;
        const int n_bands = (h + band - 1) / band;
        if (o->sample_end > 0 && n_bands > 1)   // (a pass's rows are the whole frame's work list)
            return fail(GI_ERR_ARG, "progressive passes render whole frames: band_rows 0 or >= h");
        if ((rc = prog_check(s, *cam, light, w, h, *o))) return rc;
        if ((rc = ensure_hostpath(s, band_px, std::min(n_bands, HostPath::kSlots)))) return rc;
        HostPath& hp = s->hp;
        const CamDev cd = make_cam(*cam, w);
        const bool want_rgb = rgb || cb, want_rgb8 = rgb8 || cb;
        // a whole-frame call copies straight into the caller's buffers (no staging, nothing to overlap)
        const bool direct = n_bands == 1;
        double* const dst_rgb = direct && rgb ? rgb : hp.h_rgb[0];
        uint8_t* const dst_rgb8 = direct && rgb8 ? rgb8 : hp.h_rgb8[0];
        // band i: render into slot i % 2 (after that slot's previous copy), then copy to its staging
        auto issue = [&](int i) -> int {
            const int k = i % HostPath::kSlots, y0 = i * band, rows = std::min(band, h - y0);
            const size_t n = (size_t)w * rows * 3;
            hipError_t e = hipSuccess;
            if (i >= HostPath::kSlots && (e = hipStreamWaitEvent(hp.render, hp.copied[k], 0)) != hipSuccess)
                return hip_fail(e, "render");
            const int r = scene_render_band(s, cd, light, w, rows, y0, *o, hp.d_rgb[k], hp.d_rgb8[k], hp.render, false);
            if (r) return r;
            e = hipEventRecord(hp.rendered[k], hp.render);
            if (e == hipSuccess) e = hipStreamWaitEvent(hp.copy, hp.rendered[k], 0);
            double* const to = i == 0 ? dst_rgb : hp.h_rgb[k];
            uint8_t* const to8 = i == 0 ? dst_rgb8 : hp.h_rgb8[k];
            if (e == hipSuccess && want_rgb) e = hipMemcpyAsync(to, hp.d_rgb[k], n * sizeof(double), hipMemcpyDeviceToHost, hp.copy);
            if (e == hipSuccess && want_rgb8) e = hipMemcpyAsync(to8, hp.d_rgb8[k], n, hipMemcpyDeviceToHost, hp.copy);
            if (e == hipSuccess) e = hipEventRecord(hp.copied[k], hp.copy);
            return e == hipSuccess ? GI_OK : hip_fail(e, "render");
        };
        hipError_t e = hipSuccess;
        if (cancel && *cancel) rc = fail(GI_ERR_CANCELLED, "cancelled");
        else rc = issue(0);
        for (int i = 0; rc == GI_OK && i < n_bands; i++) {
            // the next band goes to the GPU before this one is delivered; cancel is polled between bands
            if (i + 1 < n_bands) {
                if (cancel && *cancel) { rc = fail(GI_ERR_CANCELLED, "cancelled"); break; }
                if ((rc = issue(i + 1)) != GI_OK) break;
            }
            const int k = i % HostPath::kSlots, y0 = i * band, rows = std::min(band, h - y0);
            const size_t n = (size_t)w * rows * 3;
            if ((e = hipEventSynchronize(hp.copied[k])) != hipSuccess) { rc = hip_fail(e, "render"); break; }
            const double* hr = i == 0 ? dst_rgb : hp.h_rgb[k];
            const uint8_t* hr8 = i == 0 ? dst_rgb8 : hp.h_rgb8[k];
            if (rgb && hr != rgb) { std::memcpy(rgb + (size_t)y0 * w * 3, hr, n * sizeof(double)); hr = rgb + (size_t)y0 * w * 3; }
            if (rgb8 && hr8 != rgb8) { std::memcpy(rgb8 + (size_t)y0 * w * 3, hr8, n); hr8 = rgb8 + (size_t)y0 * w * 3; }
            if (cb) cb(user, y0, rows, hr8, hr);
        }
        // nothing of this call stays in flight (a cancelled or failed call drains its bands)
        const hipError_t e1 = hipStreamSynchronize(hp.render), e2 = hipStreamSynchronize(hp.copy);
        if (rc == GI_OK && (e1 != hipSuccess || e2 != hipSuccess)) rc = hip_fail(e1 != hipSuccess ? e1 : e2, "render");
        if (rc == GI_OK) prog_done(s, *o);
        return rc;
    });
}

int gi_scene_kernel_ms(gi_scene* s, float* avg_ms, int64_t* n) {
    return guard([&]() -> int {
        DeviceRestore keep;   // the caller's current device, restored on return
        if (!s || !avg_ms) return fail(GI_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        KTimer& kt = s->kt;
        if (kt.recorded == 0) return fail(GI_ERR_ARG, "no render issued with GI_FLAG_TIME since the last read");
        int rc = bind_device(s->device);
        if (rc) return rc;
        // the unfolded pairs are the last min(recorded, kRing) slots
        const long long first = kt.recorded > KTimer::kRing ? kt.recorded - KTimer::kRing : 0;
        for (long long r = std::max(first, kt.folded); r < kt.recorded; r++) {
            const hipError_t e = fold_timer(kt, (int)(r % KTimer::kRing));
            if (e != hipSuccess) return hip_fail(e, "gi_scene_kernel_ms");
        }
        *avg_ms = (float)(kt.sum_ms / (double)kt.folded);
        if (n) *n = kt.folded;
        kt.recorded = 0;
        kt.folded = 0;
        kt.sum_ms = 0.0;
        return GI_OK;
    });
}

int gi_scene_x_form(gi_scene* s, const gi_opts* o, int32_t* form) {
    return guard([&]() -> int {
        if (!s || !o || !form) return fail(GI_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        *form = x_form_choice(s->dev, s->xcfg, *o);
        return GI_OK;
    });
}

int gi_scene_r_kernel(gi_scene* s, const gi_opts* o, int32_t* kernel) {
    return guard([&]() -> int {
        if (!s || !o || !kernel) return fail(GI_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        *kernel = r_kernel_choice(s->dev, *o);
        if (*kernel == 1 && s->xs.rf_failed > 0 && s->xs.rf_slots == 0) *kernel = 2;   // (its buffers failed)
        return GI_OK;
    });
}

int gi_unshard_device(int w, int h, int shard_count, const double* d_packed, const uint8_t* d_packed8, double* d_rgb,
                      uint8_t* d_rgb8, void* stream) {
    return guard([&]() -> int {
        if (w <= 0 || h <= 0 || shard_count < 1) return fail(GI_ERR_ARG, "bad unshard arguments");
        if ((d_rgb && !d_packed) || (d_rgb8 && !d_packed8)) return fail(GI_ERR_ARG, "missing packed input");
        return unshard(w, h, shard_count, d_packed, d_packed8, d_rgb, d_rgb8, static_cast<hipStream_t>(stream));
    });
}

int gi_trace_ray(gi_scene* s, const double origin[3], const double dir[3], const double light[3], gi_hit* hit,
                 double rgb[3]) {
    return guard([&]() -> int {
        DeviceRestore keep;   // the caller's current device, restored on return
        if (!s || !origin || !dir || !light || !hit || !rgb) return fail(GI_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(s->mu);
        int rc = bind_device(s->device);
        if (rc) return rc;
        int32_t* d_i = nullptr;
        double* d_d = nullptr;
        hipError_t e;
        if ((e = hipMalloc((void**)&d_i, 4 * sizeof(int32_t))) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = hipMalloc((void**)&d_d, 9 * sizeof(double))) != hipSuccess) { (void)hipFree(d_i); return hip_fail(e, "hipMalloc"); }
        const V3 o = v3(origin[0], origin[1], origin[2]);
        const V3 d = normalize(v3(dir[0], dir[1], dir[2]));   // Ray ctor (ray.h:6)
        e = launch_trace_ray(s->dev, o, d, v3(light[0], light[1], light[2]), d_i, d_d, nullptr);
        int32_t hi[3] = {-1, 0, 0};
        double hd[9] = {0};
        if (e == hipSuccess) e = hipMemcpy(hi, d_i, 3 * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(hd, d_d, 9 * sizeof(double), hipMemcpyDeviceToHost);
        (void)hipFree(d_i);
        (void)hipFree(d_d);
        if (e != hipSuccess) return hip_fail(e, "trace_ray");
        hit->entity = hi[0];
        hit->u = hi[1];
        hit->v = hi[2];
        for (int k = 0; k < 3; ++k) { hit->point[k] = hd[k]; hit->normal[k] = hd[3 + k]; rgb[k] = hd[6 + k]; }
        return GI_OK;
    });
}

int gi_kat_expbox(int n, const double* recs, int32_t* out) {
    return guard([&]() -> int {
        if (n < 0 || (n > 0 && (!recs || !out))) return fail(GI_ERR_ARG, "bad arguments");
        if (n == 0) return GI_OK;
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(GI_ERR_DEVICE, "no HIP device");
        double* d_r = nullptr;
        int32_t* d_o = nullptr;
        hipError_t e;
        if ((e = hipMalloc((void**)&d_r, (size_t)n * 12 * sizeof(double))) != hipSuccess) return hip_fail(e, "hipMalloc");
        if ((e = hipMalloc((void**)&d_o, (size_t)n * sizeof(int32_t))) != hipSuccess) { (void)hipFree(d_r); return hip_fail(e, "hipMalloc"); }
        e = hipMemcpy(d_r, recs, (size_t)n * 12 * sizeof(double), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = launch_box_kat(n, d_r, d_o, nullptr);
        if (e == hipSuccess) e = hipMemcpy(out, d_o, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost);
        (void)hipFree(d_r);
        (void)hipFree(d_o);
        return e == hipSuccess ? GI_OK : hip_fail(e, "gi_kat_expbox");
    });
}

int gi_octree_create(const gi_scene_desc* desc, gi_octree** out) {
    return guard([&]() -> int {
        if (!desc || !out || desc->n_entities < 0 || (desc->n_entities > 0 && !desc->entities))
            return fail(GI_ERR_ARG, "bad scene descriptor");
        *out = nullptr;
        std::unique_ptr<gi_octree> t(new gi_octree());
        std::string err;
        if (!build_host_scene(*desc, t->host, err)) return fail(GI_ERR_SCENE, err);
        *out = t.release();
        return GI_OK;
    });
}

void gi_octree_destroy(gi_octree* t) { delete t; }

int gi_octree_intersect(const gi_octree* t, const double origin[3], const double dir[3], int32_t* out, int64_t cap,
                        int64_t* n) {
    return guard([&]() -> int {
        if (!t || !origin || !dir || !n || cap < 0 || (cap > 0 && !out)) return fail(GI_ERR_ARG, "bad arguments");
        std::vector<int32_t> list;
        if (!t->host.rnodes.empty())
            octree_query(t->host, 0, v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2]), list);
        *n = (int64_t)list.size();
        const int64_t k = std::min<int64_t>(cap, (int64_t)list.size());
        if (k > 0) std::memcpy(out, list.data(), (size_t)k * sizeof(int32_t));
        return GI_OK;
    });
}

}  // extern "C"
