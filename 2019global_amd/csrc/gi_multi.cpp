// gi_multi.cpp — RayTracer::run (raytracer.h:23-87) over several GPUs of one process (gi.h
// gi_multi_*).  Pixels are independent (raytracer.h:32-86), so the frame shards: 8x8 tiles are
// dealt round-robin over the shards (tile t -> shard t % n, the same map as gi_render_device's
// shard_count / shard_index), every shard renders its tiles into a packed buffer on its device,
// and one RCCL group of ncclSend/ncclRecv (rccl.h:700-725) moves the packed tiles to the root
// device over xGMI -- one point-to-point stream per peer, each on its own link -- where the
// unshard kernel reassembles the band.  Shards on the root device render straight into the
// gather buffer.  Bands are pipelined two deep (issue_band), as gi_render's.  librccl is loaded (dlopen) only when a second device takes part; the results
// are bit-identical to a one-device render (pixels do not depend on the shard count).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gi.h"
#include "gi_internal.h"
#include "gi_scene.h"

using namespace gi;

namespace {

// RCCL entry points, resolved from librccl on first use (single-device users never load it)
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string load_error;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            r.load_error = std::string("cannot load librccl: ") + (e ? e : "?");
            return;
        }
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        if (!r.comm_init_all || !r.comm_destroy || !r.send || !r.recv || !r.group_start || !r.group_end || !r.error_string)
            r.load_error = "librccl lacks an entry point (ncclCommInitAll / ncclSend / ncclRecv / ncclGroup*)";
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char* what) {
    const Rccl& r = rccl();
    return error(GI_ERR_DEVICE, std::string(what) + ": " + (r.error_string ? r.error_string(e) : "RCCL error"));
}

}  // namespace

// Band pipeline: band i uses slot i % 2 of every buffer below, so band i+1 renders, gathers and is
// reassembled while band i's frame is copied to pinned memory (on the root's copy stream) and
// delivered to the caller; a slot's device buffers are reused only after its copy has completed.
constexpr int kSlots = 2;

struct gi_multi {
    int n_shards = 0;
    std::vector<int> shard_k;          // shard -> index into devs
    std::vector<int> shard_slot;       // remote shard -> its slot in its device's staging buffer
    std::vector<int> devs;             // distinct devices; devs[0] (= devices[0]) is the root
    std::vector<int> remote_count;     // per device: shards routed through RCCL
    std::vector<gi_scene*> scenes;     // one replica per device
    std::vector<hipStream_t> streams;  // one per device (render, RCCL, reassembly)
    hipStream_t copy = nullptr;        // root: device-to-host copies of finished bands
    hipEvent_t assembled[kSlots] = {}, copied[kSlots] = {};
    std::vector<ncclComm_t> comms;     // one per device when RCCL carries the gather
    bool use_rccl = false;
    // buffers per slot, grown on demand
    size_t per_cap = 0;                // elements (pixel slots x 3) of one shard's packed buffer
    std::vector<double*> stage[kSlots];    // per device: packed rgb of its RCCL-routed shards
    std::vector<uint8_t*> stage8[kSlots];
    double* gather[kSlots] = {};       // root: every shard's packed rgb, shard s at s * per
    uint8_t* gather8[kSlots] = {};
    size_t frame_cap = 0;              // pixels
    double* frame[kSlots] = {};        // root: the band, row-major
    uint8_t* frame8[kSlots] = {};
    double* h_rgb[kSlots] = {};        // pinned
    uint8_t* h_rgb8[kSlots] = {};
    std::mutex mu;

    bool remote(int s) const { return use_rccl && (shard_k[(size_t)s] != 0 || self_rccl); }
    bool self_rccl = false;            // GI_MULTI_RCCL=1: root shards also travel through RCCL (to self)
};

namespace {

void free_buffers(gi_multi* m) {
    for (int j = 0; j < kSlots; ++j) {
        for (size_t k = 0; k < m->devs.size(); ++k) {
            (void)hipSetDevice(m->devs[k]);
            if (k < m->stage[j].size()) { (void)hipFree(m->stage[j][k]); m->stage[j][k] = nullptr; }
            if (k < m->stage8[j].size()) { (void)hipFree(m->stage8[j][k]); m->stage8[j][k] = nullptr; }
        }
        if (!m->devs.empty()) (void)hipSetDevice(m->devs[0]);
        (void)hipFree(m->gather[j]);
        (void)hipFree(m->gather8[j]);
        (void)hipFree(m->frame[j]);
        (void)hipFree(m->frame8[j]);
        (void)hipHostFree(m->h_rgb[j]);
        (void)hipHostFree(m->h_rgb8[j]);
        m->gather[j] = m->frame[j] = m->h_rgb[j] = nullptr;
        m->gather8[j] = m->frame8[j] = m->h_rgb8[j] = nullptr;
    }
    m->per_cap = m->frame_cap = 0;
}

void destroy_multi(gi_multi* m) noexcept {
    if (!m) return;
    for (size_t k = 0; k < m->streams.size(); ++k) {
        (void)hipSetDevice(m->devs[k]);
        if (m->streams[k]) (void)hipStreamSynchronize(m->streams[k]);
    }
    if (!m->devs.empty()) (void)hipSetDevice(m->devs[0]);
    if (m->copy) (void)hipStreamSynchronize(m->copy);
    if (!m->comms.empty() && rccl().comm_destroy)
        for (ncclComm_t c : m->comms)
            if (c) (void)rccl().comm_destroy(c);
    free_buffers(m);
    if (!m->devs.empty()) (void)hipSetDevice(m->devs[0]);
    for (int j = 0; j < kSlots; ++j) {
        if (m->assembled[j]) (void)hipEventDestroy(m->assembled[j]);
        if (m->copied[j]) (void)hipEventDestroy(m->copied[j]);
    }
    if (m->copy) (void)hipStreamDestroy(m->copy);
    for (size_t k = 0; k < m->streams.size(); ++k) {
        (void)hipSetDevice(m->devs[k]);
        if (m->streams[k]) (void)hipStreamDestroy(m->streams[k]);
    }
    for (gi_scene* s : m->scenes) scene_destroy(s);
    delete m;
}

// per-shard packed buffers of `per` elements, band frames of `px` pixels, both slots (grown, never
// shrunk; the caller has drained the pipeline)
int ensure_buffers(gi_multi* m, size_t per, size_t px) {
    hipError_t e = hipSuccess;
    if (m->per_cap < per) {
        for (int j = 0; j < kSlots; ++j) {
            for (size_t k = 0; k < m->devs.size(); ++k) {
                (void)hipSetDevice(m->devs[k]);
                (void)hipFree(m->stage[j][k]);
                (void)hipFree(m->stage8[j][k]);
                m->stage[j][k] = nullptr;
                m->stage8[j][k] = nullptr;
                const size_t n = (size_t)m->remote_count[k] * per;
                if (n == 0) continue;
                if ((e = hipMalloc((void**)&m->stage[j][k], n * sizeof(double))) != hipSuccess ||
                    (e = hipMalloc((void**)&m->stage8[j][k], n)) != hipSuccess)
                    return hip_error(e, "hipMalloc (shard staging)");
            }
            (void)hipSetDevice(m->devs[0]);
            (void)hipFree(m->gather[j]);
            (void)hipFree(m->gather8[j]);
            m->gather[j] = nullptr;
            m->gather8[j] = nullptr;
            const size_t n = (size_t)m->n_shards * per;
            if ((e = hipMalloc((void**)&m->gather[j], n * sizeof(double))) != hipSuccess ||
                (e = hipMalloc((void**)&m->gather8[j], n)) != hipSuccess)
                return hip_error(e, "hipMalloc (gather)");
        }
        m->per_cap = per;
    }
    if (m->frame_cap < px) {
        (void)hipSetDevice(m->devs[0]);
        for (int j = 0; j < kSlots; ++j) {
            (void)hipFree(m->frame[j]);
            (void)hipFree(m->frame8[j]);
            (void)hipHostFree(m->h_rgb[j]);
            (void)hipHostFree(m->h_rgb8[j]);
            m->frame[j] = m->h_rgb[j] = nullptr;
            m->frame8[j] = m->h_rgb8[j] = nullptr;
            if ((e = hipMalloc((void**)&m->frame[j], px * 3 * sizeof(double))) != hipSuccess ||
                (e = hipMalloc((void**)&m->frame8[j], px * 3)) != hipSuccess ||
                (e = hipHostMalloc((void**)&m->h_rgb[j], px * 3 * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
                (e = hipHostMalloc((void**)&m->h_rgb8[j], px * 3, hipHostMallocDefault)) != hipSuccess)
                return hip_error(e, "band buffers");
        }
        m->frame_cap = px;
    }
    return GI_OK;
}

// Issues one band into slot j (asynchronous): every shard renders on its device, RCCL brings the
// remote shards to the root, the root reassembles the band, and the root's copy stream moves it to
// the slot's pinned buffers (event copied[j]).  The slot's previous copy must have completed
// (first_use: it had none).
int issue_band(gi_multi* m, int j, bool first_use, const CamDev& cd, const double light[3], int w, int rows, int y0,
               const gi_opts& o, bool want_rgb, bool want_rgb8) {
    const int n = m->n_shards;
    const size_t per = (size_t)gi_shard_tiles(w, rows, n) * GI_TILE * GI_TILE * 3;
    gi_opts os = o;
    os.shard_count = n;
    os.band_rows = 0;
    os.flags &= ~(uint32_t)GI_FLAG_TIME;
    int rc = GI_OK;
    // the root's reassembly (or, for one shard, its render) writes slot j: after slot j's last copy
    if (!first_use) {
        if ((rc = bind_device(m->devs[0]))) return rc;
        const hipError_t e = hipStreamWaitEvent(m->streams[0], m->copied[j], 0);
        if (e != hipSuccess) return hip_error(e, "hipStreamWaitEvent");
    }
    for (int s = 0; s < n; ++s) {   // asynchronous launches: the devices render concurrently
        const int k = m->shard_k[(size_t)s];
        const size_t slot_off = m->remote(s) ? (size_t)m->shard_slot[(size_t)s] * per : (size_t)s * per;
        double* dst = (m->remote(s) ? m->stage[j][(size_t)k] : m->gather[j]) + slot_off;
        uint8_t* dst8 = (m->remote(s) ? m->stage8[j][(size_t)k] : m->gather8[j]) + slot_off;
        os.shard_index = s;
        if ((rc = scene_render_band(m->scenes[(size_t)k], cd, light, w, rows, y0, os, dst, dst8, m->streams[(size_t)k], false)))
            return rc;
    }
    if (m->use_rccl) {   // the gather: one send/recv pair per remote shard, fused in one group
        const Rccl& r = rccl();
        ncclResult_t e = r.group_start();
        for (int s = 0; e == ncclSuccess && s < n; ++s) {
            if (!m->remote(s)) continue;
            const size_t k = (size_t)m->shard_k[(size_t)s];
            const size_t off = (size_t)m->shard_slot[(size_t)s] * per;
            if (want_rgb) {
                e = r.send(m->stage[j][k] + off, per, ncclFloat64, 0, m->comms[k], m->streams[k]);
                if (e == ncclSuccess) e = r.recv(m->gather[j] + (size_t)s * per, per, ncclFloat64, (int)k, m->comms[0], m->streams[0]);
            }
            if (want_rgb8 && e == ncclSuccess) {
                e = r.send(m->stage8[j][k] + off, per, ncclUint8, 0, m->comms[k], m->streams[k]);
                if (e == ncclSuccess) e = r.recv(m->gather8[j] + (size_t)s * per, per, ncclUint8, (int)k, m->comms[0], m->streams[0]);
            }
        }
        const ncclResult_t e2 = r.group_end();
        if (e != ncclSuccess) return nccl_fail(e, "RCCL gather");
        if (e2 != ncclSuccess) return nccl_fail(e2, "RCCL gather");
    }
    if ((rc = bind_device(m->devs[0]))) return rc;
    hipStream_t st = m->streams[0];
    // one shard renders row-major already (gi_render_device with shard_count 1): no reassembly
    const double* fr = n == 1 ? m->gather[j] : m->frame[j];
    const uint8_t* fr8 = n == 1 ? m->gather8[j] : m->frame8[j];
    if (n > 1 && (rc = unshard(w, rows, n, m->gather[j], m->gather8[j], want_rgb ? m->frame[j] : nullptr,
                               want_rgb8 ? m->frame8[j] : nullptr, st)))
        return rc;
    const size_t cnt = (size_t)w * rows * 3;
    hipError_t e = hipEventRecord(m->assembled[j], st);
    if (e == hipSuccess) e = hipStreamWaitEvent(m->copy, m->assembled[j], 0);
    if (e == hipSuccess && want_rgb) e = hipMemcpyAsync(m->h_rgb[j], fr, cnt * sizeof(double), hipMemcpyDeviceToHost, m->copy);
    if (e == hipSuccess && want_rgb8) e = hipMemcpyAsync(m->h_rgb8[j], fr8, cnt, hipMemcpyDeviceToHost, m->copy);
    if (e == hipSuccess) e = hipEventRecord(m->copied[j], m->copy);
    return e == hipSuccess ? GI_OK : hip_error(e, "band copy-back");
}

// waits for every stream of the handle (a failed or cancelled frame leaves nothing in flight)
void drain(gi_multi* m) {
    for (size_t k = 0; k < m->streams.size(); ++k) {
        (void)hipSetDevice(m->devs[k]);
        (void)hipStreamSynchronize(m->streams[k]);
    }
    if (!m->devs.empty()) (void)hipSetDevice(m->devs[0]);
    if (m->copy) (void)hipStreamSynchronize(m->copy);
}

}  // namespace

extern "C" {

int gi_multi_create(const gi_scene_desc* desc, int n_shards, const int* devices, gi_multi** out) {
    return guard([&]() -> int {
        DeviceRestore keep;   // the caller's current device, restored on return
        if (!desc || !out || n_shards < 1 || !devices || desc->n_entities < 0 || (desc->n_entities > 0 && !desc->entities))
            return error(GI_ERR_ARG, "bad gi_multi_create arguments");
        *out = nullptr;
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return error(GI_ERR_DEVICE, "no HIP device");
        std::unique_ptr<gi_multi, void (*)(gi_multi*)> m(new gi_multi(), [](gi_multi* p) { destroy_multi(p); });
        m->n_shards = n_shards;
        for (int s = 0; s < n_shards; ++s) {
            const int d = devices[s];
            if (d < 0 || d >= ndev) return error(GI_ERR_ARG, "device index out of range");
            auto it = std::find(m->devs.begin(), m->devs.end(), d);
            if (it == m->devs.end()) { m->devs.push_back(d); it = m->devs.end() - 1; }
            m->shard_k.push_back((int)(it - m->devs.begin()));
        }
        const char* env = std::getenv("GI_MULTI_RCCL");
        m->self_rccl = env && std::atoi(env) != 0;
        m->use_rccl = m->devs.size() > 1 || m->self_rccl;
        const size_t nd = m->devs.size();
        m->scenes.assign(nd, nullptr);
        m->streams.assign(nd, nullptr);
        for (int j = 0; j < kSlots; ++j) {
            m->stage[j].assign(nd, nullptr);
            m->stage8[j].assign(nd, nullptr);
        }
        m->remote_count.assign(nd, 0);
        m->shard_slot.assign((size_t)n_shards, -1);
        for (int s = 0; s < n_shards; ++s)
            if (m->remote(s)) m->shard_slot[(size_t)s] = m->remote_count[(size_t)m->shard_k[(size_t)s]]++;
        for (size_t k = 0; k < nd; ++k) {   // a scene replica and a stream per device
            int rc = scene_create_on(desc, m->devs[k], &m->scenes[k]);
            if (rc) return rc;
            const hipError_t e = hipStreamCreateWithFlags(&m->streams[k], hipStreamNonBlocking);
            if (e != hipSuccess) return hip_error(e, "hipStreamCreate");
        }
        {   // the root's copy stream and the band pipeline's events
            int rc = bind_device(m->devs[0]);
            if (rc) return rc;
            hipError_t e = hipStreamCreateWithFlags(&m->copy, hipStreamNonBlocking);
            for (int j = 0; e == hipSuccess && j < kSlots; ++j) {
                e = hipEventCreateWithFlags(&m->assembled[j], hipEventDisableTiming);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&m->copied[j], hipEventDisableTiming);
            }
            if (e != hipSuccess) return hip_error(e, "band pipeline streams / events");
        }
        if (m->use_rccl) {   // one communicator per device, rank k = devs[k] (rank 0 = the root)
            const Rccl& r = rccl();
            if (!r.load_error.empty()) return error(GI_ERR_DEVICE, r.load_error);
            m->comms.assign(nd, nullptr);
            const ncclResult_t e = r.comm_init_all(m->comms.data(), (int)nd, m->devs.data());
            if (e != ncclSuccess) {
                m->comms.clear();
                return nccl_fail(e, "ncclCommInitAll");
            }
        }
        *out = m.release();
        return GI_OK;
    });
}

void gi_multi_destroy(gi_multi* m) { destroy_multi(m); }

int gi_multi_info(const gi_multi* m, int* n_shards, int* n_devices, int* uses_rccl) {
    if (!m) return error(GI_ERR_ARG, "null multi");
    if (n_shards) *n_shards = m->n_shards;
    if (n_devices) *n_devices = (int)m->devs.size();
    if (uses_rccl) *uses_rccl = m->use_rccl ? 1 : 0;
    return GI_OK;
}

int gi_multi_render(gi_multi* m, const gi_camera* cam, const double light[3], int w, int h, const gi_opts* o,
                    double* rgb, uint8_t* rgb8, const volatile int* cancel, gi_tile_cb cb, void* user) {
    return guard([&]() -> int {
        if (!m) return error(GI_ERR_ARG, "null multi");
        int rc = check_opts(w, h, o);
        if (rc) return rc;
        if (!cam || !light) return error(GI_ERR_ARG, "null camera or light");
        if (o->shard_count != 1 || o->shard_index != 0)
            return error(GI_ERR_ARG, "gi_multi_render shards by itself: opts shard_count must be 1");
        if (o->flags & GI_FLAG_STATS) return error(GI_ERR_ARG, "GI_FLAG_STATS is per device: use gi_render_device");
        if (o->sample_end != 0) return error(GI_ERR_ARG, "progressive passes: gi_render / gi_render_device of one scene");
        DeviceRestore keep;   // the caller's current device, restored on return
        std::lock_guard<std::mutex> lk(m->mu);
        const int band = band_rows_of(o, h);
        const int n_bands = (h + band - 1) / band;
        const bool want_rgb = rgb || cb, want_rgb8 = rgb8 || cb;
        drain(m);   // nothing of an earlier call is in flight: buffers may be regrown
        rc = ensure_buffers(m, (size_t)gi_shard_tiles(w, band, m->n_shards) * GI_TILE * GI_TILE * 3, (size_t)w * band);
        if (rc) return rc;
        const CamDev cd = make_cam(*cam, w);
        auto issue = [&](int i) {
            const int y0 = i * band;
            return issue_band(m, i % kSlots, i < kSlots, cd, light, w, std::min(band, h - y0), y0, *o, want_rgb, want_rgb8);
        };
        // progressive bands, two in flight: band i+1 is issued before band i is delivered, so its
        // renders, gather and reassembly overlap band i's copy to the host and the caller's callback;
        // cancel is polled between bands
        if (cancel && *cancel) rc = error(GI_ERR_CANCELLED, "cancelled");
        else rc = issue(0);
        for (int i = 0; rc == GI_OK && i < n_bands; ++i) {
            if (i + 1 < n_bands) {
                if (cancel && *cancel) { rc = error(GI_ERR_CANCELLED, "cancelled"); break; }
                if ((rc = issue(i + 1)) != GI_OK) break;
            }
            const int j = i % kSlots, y0 = i * band, rows = std::min(band, h - y0);
            const hipError_t e = hipEventSynchronize(m->copied[j]);
            if (e != hipSuccess) { rc = hip_error(e, "band copy-back"); break; }
            const size_t nn = (size_t)w * rows * 3;
            if (rgb) std::memcpy(rgb + (size_t)y0 * w * 3, m->h_rgb[j], nn * sizeof(double));
            if (rgb8) std::memcpy(rgb8 + (size_t)y0 * w * 3, m->h_rgb8[j], nn);
            if (cb) cb(user, y0, rows, rgb8 ? rgb8 + (size_t)y0 * w * 3 : m->h_rgb8[j], rgb ? rgb + (size_t)y0 * w * 3 : m->h_rgb[j]);
        }
        drain(m);
        return rc;
    });
}

}  // extern "C"
