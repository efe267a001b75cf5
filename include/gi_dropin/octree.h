// gi_dropin/octree.h — drop-in replacement for preon7/2019global include/octree.h.
//
// Same public surface the reference's callers use: Octree(min, max) (octree.h:14), the public
// min/max members, push_back(Entity*) (octree.h:20-43) and the candidate query
// intersect(const Ray&) (octree.h:46-68).  The tree itself is not built here: push order is
// recorded, and libgi rebuilds the reference octree from it bit for bit (node boxes, lost entities
// A.6, silent drop A.14) -- on the device for RayTracer::run (gi_scene_create), and on the host
// for intersect() (gi_octree_create / gi_octree_intersect: DFS over children 0..7 with the ExpBox
// node test, octree.h:132-155, duplicates kept), rebuilt lazily after push_back.
#pragma once

#include <cstddef>
#include <cstdio>
#include <memory>
#include <vector>

#include <glm/glm.hpp>

#include "entities.h"
#include "gi.h"
#include "gi_describe.h"
#include "ray.h"

class Octree {
  public:
    Octree(glm::dvec3 min, glm::dvec3 max) : min(min), max(max) {}

    glm::dvec3 min;
    glm::dvec3 max;

    /// Store an entity (the reference's push_back; order defines the candidate order, A.1).
    void push_back(Entity* object) {
        _objects.push_back(object);
        ++_generation;
    }

    /// Returns list of entities that have the possibility to be intersected by the ray
    /// (octree.h:45-68): the reference's candidate list, in its order, duplicates included.
    std::vector<Entity*> intersect(const Ray& ray) const {
        std::vector<Entity*> out;
        // The host tree is rebuilt only when push_back has changed the entity list since the last
        // query: the candidate list depends on the entities' geometry and push order alone, and an
        // entity's geometry is fixed by its constructor (entities.h has no setters; materials do
        // not enter Octree::intersect) -- and on a change of the public root box.  So a query costs the tree walk, not a re-description of the
        // whole scene (O(N) per ray before).
        if (!_host || _host_gen != _generation || _host_min != min || _host_max != max) {
            std::vector<gi_entity_desc> d;
            if (!gi_dropin::describe_all(_objects, d)) return out;
            const double mn[3] = {min.x, min.y, min.z}, mx[3] = {max.x, max.y, max.z};
            gi_scene_desc sd = {};
            for (int k = 0; k < 3; ++k) { sd.octree_min[k] = mn[k]; sd.octree_max[k] = mx[k]; }
            sd.n_entities = (int32_t)d.size();
            sd.entities = d.data();
            gi_octree* t = nullptr;
            if (gi_octree_create(&sd, &t) != GI_OK) {
                std::fprintf(stderr, "gi_octree_create: %s\n", gi_last_error());
                return out;
            }
            _host = std::shared_ptr<gi_octree>(t, gi_octree_destroy);
            _host_gen = _generation;
            _host_min = min;
            _host_max = max;
        }
        const double o[3] = {ray.origin.x, ray.origin.y, ray.origin.z}, dir[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
        int64_t n = 0;
        if (gi_octree_intersect(_host.get(), o, dir, nullptr, 0, &n) != GI_OK) return out;
        std::vector<int32_t> idx((size_t)n);
        if (n > 0 && gi_octree_intersect(_host.get(), o, dir, idx.data(), n, &n) != GI_OK) return out;
        out.reserve(idx.size());
        for (int32_t i : idx) out.push_back(_objects[(size_t)i]);
        return out;
    }

    const std::vector<Entity*>& entities() const { return _objects; }
    std::size_t generation() const { return _generation; }

  private:
    std::vector<Entity*> _objects;   // non-owning, as the reference (octree.h:158)
    std::size_t _generation = 0;
    mutable std::shared_ptr<gi_octree> _host;   // host copy of the reference tree for intersect()
    mutable std::size_t _host_gen = 0;   // _generation and root box the host tree was built for
    mutable glm::dvec3 _host_min{0}, _host_max{0};
};
