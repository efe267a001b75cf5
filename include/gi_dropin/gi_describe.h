// gi_dropin/gi_describe.h — the reference's entity objects (entities.h) as gi_entity_desc records
// for the C-ABI (include/gi.h), shared by the drop-in Octree and RayTracer headers.  Each entity's
// constructor arguments are recovered from its public members and its current material is passed
// explicitly (so `entity->material = ...` after construction is seen at the next upload).
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

#include "entities.h"
#include "gi.h"

namespace gi_dropin {

inline void set_material(gi_entity_desc& d, const Material& m) {
    d.has_material = 1;
    for (int k = 0; k < 3; ++k) {
        d.mat_color[k] = m.color[k];
        d.mat_shader[k] = m.shader_parameters[k];
    }
    d.mat_specular_power = m.specular_power;
}

inline bool describe(const Entity* e, gi_entity_desc& d) {
    d = gi_entity_desc();
    auto put = [&](std::initializer_list<double> a) {
        int i = 0;
        for (double v : a) d.args[i++] = v;
    };
    if (auto* s = dynamic_cast<const ImpSphere*>(e)) {
        d.kind = GI_IMP_SPHERE;
        put({s->pos.x, s->pos.y, s->pos.z, (double)s->radius, s->material.color.x, s->material.color.y, s->material.color.z});
    } else if (auto* t = dynamic_cast<const ImpTriangle*>(e)) {
        d.kind = GI_IMP_TRIANGLE;
        put({t->p1.x, t->p1.y, t->p1.z, t->p2.x, t->p2.y, t->p2.z, t->p3.x, t->p3.y, t->p3.z});
    } else if (auto* q = dynamic_cast<const ExpQuad*>(e)) {
        d.kind = GI_EXP_QUAD;
        put({q->pos.x, q->pos.y, q->pos.z, (double)q->width, (double)q->length, (double)q->alpha, q->material.color.x,
             q->material.color.y, q->material.color.z});
    } else if (auto* es = dynamic_cast<const ExpSphere*>(e)) {
        d.kind = GI_EXP_SPHERE;
        put({es->pos.x, es->pos.y, es->pos.z, (double)es->radius, es->material.color.x, es->material.color.y,
             es->material.color.z});
    } else if (auto* c = dynamic_cast<const ExpCube*>(e)) {
        d.kind = GI_EXP_CUBE;
        put({c->pos.x, c->pos.y, c->pos.z, (double)c->width, (double)c->length, (double)c->height, c->material.color.x,
             c->material.color.y, c->material.color.z});
    } else if (auto* k = dynamic_cast<const ExpCone*>(e)) {
        d.kind = GI_EXP_CONE;   // the member dir holds the constructor argument (entities.h:823)
        put({k->pos.x, k->pos.y, k->pos.z, k->dir.x, k->dir.y, k->dir.z, (double)k->height, (double)k->radius,
             k->material.color.x, k->material.color.y, k->material.color.z});
    } else if (auto* r = dynamic_cast<const ExpRectangle*>(e)) {
        d.kind = GI_EXP_RECTANGLE;
        put({r->p1.x, r->p1.y, r->p1.z, r->p2.x, r->p2.y, r->p2.z, r->p3.x, r->p3.y, r->p3.z});
    } else if (auto* b = dynamic_cast<const ExpBox*>(e)) {
        d.kind = GI_EXP_BOX;
        put({b->min.x, b->min.y, b->min.z, b->max.x, b->max.y, b->max.z});
    } else {
        return false;
    }
    set_material(d, e->material);
    return true;
}

// Descriptors of a push-ordered entity list; false (and a message on stderr) for an unknown class.
inline bool describe_all(const std::vector<Entity*>& ents, std::vector<gi_entity_desc>& out) {
    out.clear();
    out.reserve(ents.size());
    for (const Entity* e : ents) {
        gi_entity_desc d;
        if (!describe(e, d)) {
            std::fprintf(stderr, "gi: unknown entity type (not one of entities.h's eight)\n");
            return false;
        }
        out.push_back(d);
    }
    return true;
}

// FNV-1a over the descriptors and the root box: a changed entity, material or push order changes it
inline uint64_t scene_hash(const std::vector<gi_entity_desc>& d, const double mn[3], const double mx[3]) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    };
    mix(mn, 3 * sizeof(double));
    mix(mx, 3 * sizeof(double));
    if (!d.empty()) mix(d.data(), d.size() * sizeof(gi_entity_desc));
    const uint64_t n = d.size();
    mix(&n, sizeof n);
    return h;
}

}  // namespace gi_dropin
