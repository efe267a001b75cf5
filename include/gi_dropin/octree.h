// gi_dropin/octree.h — drop-in replacement for preon7/2019global include/octree.h.
//
// Same public surface the reference's callers use: Octree(min, max) (octree.h:115), the public
// min/max members (:117-118) and push_back(Entity*) (:121-144).  The tree itself is no longer
// built here: push order is recorded, and libgi (gi_scene_create) rebuilds the reference octree
// from it bit for bit (node boxes, lost entities A.6, silent drop A.14) on the host and uploads it
// to HBM.  Octree::intersect (:147-169) is the per-ray candidate query inside RayTracer::run and
// runs on the GPU; it is not exposed on the host.
#pragma once

#include <cstddef>
#include <vector>

#include <glm/glm.hpp>

#include "entities.h"

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

    const std::vector<Entity*>& entities() const { return _objects; }
    std::size_t generation() const { return _generation; }

  private:
    std::vector<Entity*> _objects;   // non-owning, as the reference (octree.h:259)
    std::size_t _generation = 0;
};
