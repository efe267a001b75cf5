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
#pragma once

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include <glm/glm.hpp>

#include "camera.h"
#include "entities.h"
#include "image.h"
#include "octree.h"   // gi_dropin/octree.h (same directory, searched first)
#include "gi.h"
#include "gi_describe.h"

class RayTracer {
  public:
    RayTracer() = delete;
    RayTracer(const Camera& camera, glm::dvec3 light)
        : _camera(camera), _light(light), _image(std::make_shared<Image>(0, 0)) {}

    void setScene(const Octree* scene) {
        _scene = scene;
        _gpu.reset();
    }

    void run(int w, int h) {
        _image = std::make_shared<Image>(w, h);   // raytracer.h:25
        if (!_scene || w <= 0 || h <= 0) return;
        // the reference reads the live octree on every run (raytracer.h:45): the entities are
        // described again and the scene re-uploaded when anything changed (push_back, a material)
        std::vector<gi_entity_desc> ents;
        if (!gi_dropin::describe_all(_scene->entities(), ents)) return;
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
        o.mode = GI_MODE_R;
        o.spp = 1;
        o.depth = 1;
        o.shard_count = 1;
        o.band_rows = 32;
        Band band{_image.get(), w};
        const int rc = _gpu->multi ? gi_multi_render(_gpu->multi, &cam, light, w, h, &o, nullptr, nullptr, &_cancel,
                                                     &RayTracer::on_band, &band)
                                   : gi_render(_gpu->scene, &cam, light, w, h, &o, nullptr, nullptr, &_cancel,
                                               &RayTracer::on_band, &band);
        if (rc != GI_OK && rc != GI_ERR_CANCELLED) std::fprintf(stderr, "gi_render: %s\n", gi_last_error());
    }

    bool running() const { return _cancel == 0; }
    void stop() { _cancel = 1; }
    void start() { _cancel = 0; }

    std::shared_ptr<Image> getImage() const { return _image; }

  private:
    struct Band {
        Image* image;
        int w;
    };

    // the uploaded scene: one device (gi_scene) or several (gi_multi: GI_DEVICES="0,1,..." or
    // "all"; by default every gfx950 of the node when there is more than one)
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
    }

    static std::vector<int> devices() {
        std::vector<int> d;
        const char* env = std::getenv("GI_DEVICES");
        if (env && *env && std::strcmp(env, "all") != 0) {
            for (const char* p = env; *p;) {
                char* end = nullptr;
                const long v = std::strtol(p, &end, 10);
                if (end == p) break;
                d.push_back((int)v);
                p = *end == ',' ? end + 1 : end;
            }
            return d;
        }
        const int n = gi_device_count();
        if (env || n > 1)
            for (int i = 0; i < n; ++i) d.push_back(i);
        return d;
    }

    bool upload(const std::vector<gi_entity_desc>& ents, const double mn[3], const double mx[3], uint64_t hash) {
        if (gi_abi_version() != GI_ABI_VERSION) {   // gi.h's structs must match the loaded libgi
            std::fprintf(stderr, "gi: libgi ABI %d, built against %d\n", gi_abi_version(), GI_ABI_VERSION);
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
        if (devs.size() > 1) {
            if (gi_multi_create(&sd, (int)devs.size(), devs.data(), &g->multi) != GI_OK) {
                std::fprintf(stderr, "gi_multi_create: %s\n", gi_last_error());
                return false;
            }
        } else if (gi_scene_create(&sd, &g->scene) != GI_OK) {
            std::fprintf(stderr, "gi_scene_create: %s\n", gi_last_error());
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
};
