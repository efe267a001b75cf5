// gi_dropin/raytracer.h — drop-in replacement for preon7/2019global include/raytracer.h.
//
// Keeps the reference class's exact interface (raytracer.h:15-101): RayTracer(const Camera&,
// glm::dvec3 light), setScene(const Octree*), run(int w, int h), running()/stop()/start(),
// getImage().  run() renders the frame on the MI355X through the C-ABI (include/gi.h, libgi.so):
// the per-pixel body of raytracer.h:41-84 (primary ray, octree query, last-hit selection,
// texture + Blinn-Phong) executes in the gfx950 kernel, and the finished radiance is stored through
// the reference's own Image::setPixel (image.h:14-16) band by band, so the Viewer's 32 ms repaint
// shows progress exactly as before (viewer.h:18-21) and stop() still ends the frame early.
//
// Put the directory of this header BEFORE the reference's include/ on the include path and link
// libgi.so.  camera.h, entities.h, image.h, material.h, ray.h, viewer.h, gui.h and
// main.cpp stay untouched.
//
// Opt-ins (the defaults are the reference's behaviour, so an unmodified Viewer gets exactly it):
//   * the integrator: setIntegrator(GI_MODE_X, spp, depth, seed), or the environment read once at
//     construction -- GI_MODE=X (or 1), GI_SPP, GI_DEPTH, GI_SEED -- selects the build-defined
//     depth / spp path tracer (DESIGN.md "Mode X": recursive secondary-ray spawn, jittered samples)
//     behind the same run(w, h); default GI_MODE_R, 1 spp, depth 1 (raytracer.h:41-84).
//   * progressive samples (Mode X): setIntegrator(GI_MODE_X, spp, depth, seed, pass) or GI_PASS=n
//     renders the frame's spp in passes of n samples; after each pass the whole frame's running
//     estimate -- exactly the frame of that many samples (for a pass ending at sample 1 the jittered
//     first sample, not the unjittered spp = 1 frame) -- goes through Image::setPixel, so a 64-spp
//     frame shows a first image after the first pass instead of nothing until it is done (the
//     viewer restarts on every resize, viewer.h:41-52), and stop() is honoured between passes (the
//     image keeps the last delivered pass).  The last pass's frame is the one-shot frame bit for
//     bit (gi.h gi_opts sample_begin / sample_end).  One device (not with GI_DEVICES).
//   * several GPUs: GI_DEVICES="0,1,..." or "all" (every gfx950 of the node) renders each frame's
//     8x8 tiles across them (gi_multi, RCCL gather).  Unset: one device, the one current on the
//     thread that uploads the scene (hipSetDevice by the host app is honoured); if the multi-device
//     handle cannot be created (no librccl, no peer access) the frame falls back to that device.
//
// Failures are reported, not just printed: lastStatus() / lastError() (extensions) hold the last
// run()'s gi_status -- GI_OK, GI_ERR_CANCELLED after stop(), or the error that left the Image black:
// a libgi whose ABI differs from this header's (GI_ERR_ABI below), an entity the C-ABI cannot
// describe (GI_ERR_SCENE), a failed upload or render (the gi_status libgi returned).
#pragma once

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include <glm/glm.hpp>

#include "camera.h"
#include "entities.h"
#include "image.h"
#include "octree.h"   // gi_dropin/octree.h (same directory, searched first)
#include "gi.h"
#include "gi_describe.h"

// lastStatus() of a run() refused because the loaded libgi's ABI is not this header's GI_ABI_VERSION
#define GI_ERR_ABI (-100)

class RayTracer {
  public:
    RayTracer() = delete;
    RayTracer(const Camera& camera, glm::dvec3 light)
        : _camera(camera), _light(light), _image(std::make_shared<Image>(0, 0)), _integ(env_integrator()) {}

    /// Extension (not in the reference): the integrator run() uses.  GI_MODE_R (default) is the
    /// reference's per-pixel body; GI_MODE_X is the depth / spp path tracer.  Returns false (and
    /// keeps the current choice) on an invalid combination.
    bool setIntegrator(int mode, int spp, int depth, uint64_t seed = 0, int pass = 0) {
        if (mode != GI_MODE_R && mode != GI_MODE_X) return false;
        if (mode == GI_MODE_X && (spp < 1 || depth < 1 || depth > 0xFFFF || pass < 0)) return false;
        _integ = Integrator{mode, mode == GI_MODE_X ? spp : 1, mode == GI_MODE_X ? depth : 1, seed, mode == GI_MODE_X ? pass : 0};
        return true;
    }
    int integratorMode() const { return _integ.mode; }

    void setScene(const Octree* scene) {
        _scene = scene;
        _gpu.reset();
    }

    void run(int w, int h) {
        _image = std::make_shared<Image>(w, h);   // raytracer.h:25
        _status = GI_OK;
        _error.clear();
        if (!_scene || w <= 0 || h <= 0) return;
        // the reference reads the live octree on every run (raytracer.h:45): the entities are
        // described again and the scene re-uploaded when anything changed (push_back, a material)
        std::vector<gi_entity_desc> ents;
        if (!gi_dropin::describe_all(_scene->entities(), ents)) {
            report(GI_ERR_SCENE, "an entity of the scene has no gi_entity_desc (gi_describe.h)");
            return;
        }
        const double mn[3] = {_scene->min.x, _scene->min.y, _scene->min.z};
        const double mx[3] = {_scene->max.x, _scene->max.y, _scene->max.z};
        const uint64_t hash = gi_dropin::scene_hash(ents, mn, mx);
        if (!_gpu || _gpu->hash != hash) {
            if (!upload(ents, mn, mx, hash)) return;
        }
        gi_camera cam;
        for (int k = 0; k < 3; ++k) {
            cam.pos[k] = _camera.pos[k];
            cam.up[k] = _camera.up[k];
            cam.forward[k] = _camera.forward[k];
        }
        cam.focal = _camera.focalDist;
        const double light[3] = {_light.x, _light.y, _light.z};
        gi_opts o = {};
        o.mode = _integ.mode;
        o.spp = _integ.spp;
        o.depth = _integ.depth;
        o.seed = _integ.seed;
        o.shard_count = 1;
        // progressive bands: 32 rows for the reference's integrator (as cheap per row as the
        // reference's own loop is slow); the path tracer's bands are an eighth of the frame, since
        // each band is a launch that ends on its longest path (C4 in 32-row bands: 8x the frame)
        o.band_rows = _integ.mode == GI_MODE_X ? std::max(32, (h + 63) / 64 * 8) : 32;
        Band band{_image.get(), w, _keep_radiance ? &_radiance : nullptr};
        if (_keep_radiance) _radiance.assign((size_t)w * h * 3, 0.0);
        _passes = 0;
        if (_integ.mode == GI_MODE_X && _integ.pass > 0 && _integ.pass < _integ.spp && !_gpu->multi) {
            // progressive samples: whole-frame passes, each delivered as the running estimate
            o.band_rows = 0;
            int rc = GI_OK;
            for (int s0 = 0; s0 < _integ.spp && rc == GI_OK; s0 += _integ.pass) {
                o.sample_begin = s0;
                o.sample_end = std::min(_integ.spp, s0 + _integ.pass);
                rc = gi_render(_gpu->scene, &cam, light, w, h, &o, nullptr, nullptr, &_cancel, &RayTracer::on_band, &band);
                if (rc == GI_OK) {
                    ++_passes;
                    if (_on_pass) _on_pass(_passes, o.sample_end);   // (may stop() the frame)
                }
            }
            if (rc != GI_OK) report(rc, rc == GI_ERR_CANCELLED ? "cancelled" : gi_last_error());
            return;
        }
        const int rc = _gpu->multi ? gi_multi_render(_gpu->multi, &cam, light, w, h, &o, nullptr, nullptr, &_cancel,
                                                     &RayTracer::on_band, &band)
                                   : gi_render(_gpu->scene, &cam, light, w, h, &o, nullptr, nullptr, &_cancel,
                                               &RayTracer::on_band, &band);
        if (rc != GI_OK) report(rc, rc == GI_ERR_CANCELLED ? "cancelled" : gi_last_error());
    }

    bool running() const { return _cancel == 0; }
    void stop() { _cancel = 1; }
    void start() { _cancel = 0; }

    std::shared_ptr<Image> getImage() const { return _image; }

    /// Extension (tests, tools): keep the last run's fp64 radiance (w*h*3, row-major) beside the
    /// Image, whose RGB888 is its (int)(255*c) quantisation (image.h:14-16).
    void keepRadiance(bool on) { _keep_radiance = on; }
    const std::vector<double>& radiance() const { return _radiance; }
    /// Extension: the last run()'s outcome -- GI_OK, GI_ERR_CANCELLED (stop()), or the error that
    /// left the Image (partly) black: GI_ERR_ABI, GI_ERR_SCENE or the gi_status of the failed libgi
    /// call; lastError() its message.  Errors are also printed to stderr, as before.
    int lastStatus() const { return _status; }
    const std::string& lastError() const { return _error; }
    /// Extension (tests): progressive passes the last run() delivered (0 without passes).
    int passesDelivered() const { return _passes; }
    /// Extension (tools, tests): called on the render thread after each delivered progressive pass
    /// with the passes so far and the samples the image now holds; it may call stop().
    void setPassCallback(std::function<void(int passes, int samples)> f) { _on_pass = std::move(f); }

  private:
    struct Integrator {
        int mode, spp, depth;
        uint64_t seed;
        int pass;   // Mode X progressive passes of this many samples (0: the whole spp at once)
    };
    struct Band {
        Image* image;
        int w;
        std::vector<double>* radiance;
    };

    // GI_MODE / GI_SPP / GI_DEPTH / GI_SEED, read once per process; invalid values keep Mode R
    static Integrator env_integrator() {
        static const Integrator v = [] {
            Integrator r{GI_MODE_R, 1, 1, 0, 0};
            const char* m = std::getenv("GI_MODE");
            if (!m || !(std::strcmp(m, "X") == 0 || std::strcmp(m, "x") == 0 || std::strcmp(m, "1") == 0)) return r;
            const char* sp = std::getenv("GI_SPP");
            const char* dp = std::getenv("GI_DEPTH");
            const char* sd = std::getenv("GI_SEED");
            const char* ps = std::getenv("GI_PASS");
            const long spp = sp ? std::strtol(sp, nullptr, 10) : 1, depth = dp ? std::strtol(dp, nullptr, 10) : 1;
            const long pass = ps ? std::strtol(ps, nullptr, 10) : 0;
            if (spp < 1 || depth < 1 || depth > 0xFFFF || spp > (1L << 30) || pass < 0) return r;
            return Integrator{GI_MODE_X, (int)spp, (int)depth, sd ? (uint64_t)std::strtoull(sd, nullptr, 10) : 0,
                              (int)std::min(pass, spp)};
        }();
        return v;
    }

    // the uploaded scene: the current device (gi_scene) or the devices GI_DEVICES lists (gi_multi)
    struct Gpu {
        gi_scene* scene = nullptr;
        gi_multi* multi = nullptr;
        uint64_t hash = 0;
        ~Gpu() {
            if (scene) gi_scene_destroy(scene);
            if (multi) gi_multi_destroy(multi);
        }
    };

    static void on_band(void* user, int y0, int rows, const uint8_t*, const double* rgb) {
        Band* b = static_cast<Band*>(user);
        for (int j = 0; j < rows; ++j)
            for (int x = 0; x < b->w; ++x) {
                const double* c = rgb + 3 * ((size_t)j * b->w + x);
                b->image->setPixel(x, y0 + j, glm::dvec3{c[0], c[1], c[2]});
            }
        if (b->radiance)
            std::memcpy(b->radiance->data() + (size_t)y0 * b->w * 3, rgb, (size_t)rows * b->w * 3 * sizeof(double));
    }

    // GI_DEVICES: "0,1,..." (those devices) or "all" (every gfx950 of the node, by its device
    // index); unset or empty: none listed, the frame renders on the current device
    static std::vector<int> devices() {
        std::vector<int> d;
        const char* env = std::getenv("GI_DEVICES");
        if (!env || !*env) return d;
        if (std::strcmp(env, "all") == 0) {
            const int n = gi_device_list(nullptr, 0);
            d.resize((size_t)std::max(0, n));
            if (n > 0) gi_device_list(d.data(), n);
            return d;
        }
        for (const char* p = env; *p;) {
            char* end = nullptr;
            const long v = std::strtol(p, &end, 10);
            if (end == p) break;
            d.push_back((int)v);
            p = *end == ',' ? end + 1 : end;
        }
        return d;
    }

    void report(int rc, const char* msg) {
        _status = rc;
        _error = msg ? msg : "";
        if (rc != GI_OK && rc != GI_ERR_CANCELLED) std::fprintf(stderr, "gi: %s (status %d)\n", _error.c_str(), rc);
    }

    bool upload(const std::vector<gi_entity_desc>& ents, const double mn[3], const double mx[3], uint64_t hash) {
        if (gi_abi_version() != GI_ABI_VERSION) {   // gi.h's structs must match the loaded libgi
            char m[96];
            std::snprintf(m, sizeof m, "libgi ABI %d, this header's %d: rebuild against the loaded libgi", gi_abi_version(),
                          GI_ABI_VERSION);
            report(GI_ERR_ABI, m);
            return false;
        }
        gi_scene_desc sd = {};
        for (int k = 0; k < 3; ++k) {
            sd.octree_min[k] = mn[k];
            sd.octree_max[k] = mx[k];
        }
        sd.n_entities = (int32_t)ents.size();
        sd.entities = ents.data();
        auto g = std::make_shared<Gpu>();
        const std::vector<int> devs = devices();
        if (!devs.empty() && gi_multi_create(&sd, (int)devs.size(), devs.data(), &g->multi) != GI_OK) {
            // e.g. no librccl: the frame still renders, on the current device alone
            std::fprintf(stderr, "gi_multi_create: %s (rendering on one device)\n", gi_last_error());
            g->multi = nullptr;
        }
        int rc = GI_OK;
        if (!g->multi && (rc = gi_scene_create(&sd, &g->scene)) != GI_OK) {
            report(rc, gi_last_error());
            return false;
        }
        g->hash = hash;
        _gpu = g;
        return true;
    }

    volatile int _cancel = 1;   // _running = false (raytracer.h:96), polled between bands
    const Octree* _scene = nullptr;
    Camera _camera;
    glm::dvec3 _light;
    std::shared_ptr<Image> _image;
    std::shared_ptr<Gpu> _gpu;   // shared by copies (Gui/Viewer copy the RayTracer by value)
    Integrator _integ;
    bool _keep_radiance = false;
    std::vector<double> _radiance;
    int _passes = 0;
    std::function<void(int, int)> _on_pass;
    int _status = GI_OK;
    std::string _error;
};
