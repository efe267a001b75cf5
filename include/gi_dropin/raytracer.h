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
#include <memory>
#include <vector>

#include <glm/glm.hpp>

#include "camera.h"
#include "entities.h"
#include "image.h"
#include "octree.h"   // gi_dropin/octree.h (same directory, searched first)
#include "gi.h"

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
        if (!_gpu || _gpu_generation != _scene->generation()) {
            if (!upload()) return;
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
        const int rc = gi_render(_gpu.get(), &cam, light, w, h, &o, nullptr, nullptr, &_cancel, &RayTracer::on_band, &band);
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

    static void on_band(void* user, int y0, int rows, const uint8_t*, const double* rgb) {
        Band* b = static_cast<Band*>(user);
        for (int j = 0; j < rows; ++j)
            for (int x = 0; x < b->w; ++x) {
                const double* c = rgb + 3 * ((size_t)j * b->w + x);
                b->image->setPixel(x, y0 + j, glm::dvec3{c[0], c[1], c[2]});
            }
    }

    static void set_material(gi_entity_desc& d, const Material& m) {
        d.has_material = 1;
        for (int k = 0; k < 3; ++k) {
            d.mat_color[k] = m.color[k];
            d.mat_shader[k] = m.shader_parameters[k];
        }
        d.mat_specular_power = m.specular_power;
    }

    // The entity's constructor arguments are recovered from its public members (entities.h) and
    // its current material is passed explicitly (covers `entity->material = ...` after construction).
    static bool describe(const Entity* e, gi_entity_desc& d) {
        d = gi_entity_desc();
        if (auto* s = dynamic_cast<const ImpSphere*>(e)) {
            d.kind = GI_IMP_SPHERE;
            const double a[7] = {s->pos.x, s->pos.y, s->pos.z, (double)s->radius,
                                 s->material.color.x, s->material.color.y, s->material.color.z};
            std::copy(a, a + 7, d.args);
        } else if (auto* t = dynamic_cast<const ImpTriangle*>(e)) {
            d.kind = GI_IMP_TRIANGLE;
            const double a[9] = {t->p1.x, t->p1.y, t->p1.z, t->p2.x, t->p2.y, t->p2.z, t->p3.x, t->p3.y, t->p3.z};
            std::copy(a, a + 9, d.args);
        } else if (auto* q = dynamic_cast<const ExpQuad*>(e)) {
            d.kind = GI_EXP_QUAD;
            const double a[9] = {q->pos.x, q->pos.y, q->pos.z, (double)q->width, (double)q->length, (double)q->alpha,
                                 q->material.color.x, q->material.color.y, q->material.color.z};
            std::copy(a, a + 9, d.args);
        } else if (auto* es = dynamic_cast<const ExpSphere*>(e)) {
            d.kind = GI_EXP_SPHERE;
            const double a[7] = {es->pos.x, es->pos.y, es->pos.z, (double)es->radius,
                                 es->material.color.x, es->material.color.y, es->material.color.z};
            std::copy(a, a + 7, d.args);
        } else if (auto* c = dynamic_cast<const ExpCube*>(e)) {
            d.kind = GI_EXP_CUBE;
            const double a[9] = {c->pos.x, c->pos.y, c->pos.z, (double)c->width, (double)c->length, (double)c->height,
                                 c->material.color.x, c->material.color.y, c->material.color.z};
            std::copy(a, a + 9, d.args);
        } else if (auto* k = dynamic_cast<const ExpCone*>(e)) {
            d.kind = GI_EXP_CONE;   // the member dir holds the constructor argument (entities.h:823)
            const double a[11] = {k->pos.x, k->pos.y, k->pos.z, k->dir.x, k->dir.y, k->dir.z, (double)k->height,
                                  (double)k->radius, k->material.color.x, k->material.color.y, k->material.color.z};
            std::copy(a, a + 11, d.args);
        } else if (auto* r = dynamic_cast<const ExpRectangle*>(e)) {
            d.kind = GI_EXP_RECTANGLE;
            const double a[9] = {r->p1.x, r->p1.y, r->p1.z, r->p2.x, r->p2.y, r->p2.z, r->p3.x, r->p3.y, r->p3.z};
            std::copy(a, a + 9, d.args);
        } else if (auto* b = dynamic_cast<const ExpBox*>(e)) {
            d.kind = GI_EXP_BOX;
            const double a[6] = {b->min.x, b->min.y, b->min.z, b->max.x, b->max.y, b->max.z};
            std::copy(a, a + 6, d.args);
        } else {
            return false;
        }
        set_material(d, e->material);
        return true;
    }

    bool upload() {
        if (gi_abi_version() != GI_ABI_VERSION) {   // gi.h's structs must match the loaded libgi
            std::fprintf(stderr, "gi: libgi ABI %d, built against %d\n", gi_abi_version(), GI_ABI_VERSION);
            return false;
        }
        std::vector<gi_entity_desc> ents;
        for (const Entity* e : _scene->entities()) {
            gi_entity_desc d;
            if (!describe(e, d)) {
                std::fprintf(stderr, "gi: unknown entity type (not one of entities.h's eight)\n");
                return false;
            }
            ents.push_back(d);
        }
        gi_scene_desc sd = {};
        for (int k = 0; k < 3; ++k) {
            sd.octree_min[k] = _scene->min[k];
            sd.octree_max[k] = _scene->max[k];
        }
        sd.n_entities = (int32_t)ents.size();
        sd.entities = ents.data();
        gi_scene* s = nullptr;
        if (gi_scene_create(&sd, &s) != GI_OK) {
            std::fprintf(stderr, "gi_scene_create: %s\n", gi_last_error());
            return false;
        }
        _gpu = std::shared_ptr<gi_scene>(s, gi_scene_destroy);
        _gpu_generation = _scene->generation();
        return true;
    }

    volatile int _cancel = 1;   // _running = false (raytracer.h:96), polled between bands
    const Octree* _scene = nullptr;
    Camera _camera;
    glm::dvec3 _light;
    std::shared_ptr<Image> _image;
    std::shared_ptr<gi_scene> _gpu;   // shared by copies (Gui/Viewer copy the RayTracer by value)
    std::size_t _gpu_generation = 0;
};
