// gi_dropin/obj.h — OBJ meshes for the reference's scene code (the optional OBJ
// loader).  The reference builds scenes by hand (main.cpp:24-48: octree.push_back(new Entity(...)));
// push_obj does the same for a Wavefront OBJ mesh: one ImpTriangle(p1, p2, p3) (entities.h:138)
// per triangle of each face's fan, in file order, parsed by libgi's gi_obj_parse (gi.h).
#pragma once

#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include <glm/glm.hpp>

#include "entities.h"
#include "gi.h"
#include "octree.h"

namespace gi_dropin {

// Pushes the mesh in `text` onto `octree`; every triangle gets `*material` when it is given (else
// the reference's default ImpTriangle material).  The entities are returned to the caller, who
// keeps them alive while the octree refers to them (main.cpp's `new`ed entities are never freed).
// On a parse error nothing is pushed, the result is empty and *ok (if given) is false;
// gi_last_error() names the line.
inline std::vector<std::unique_ptr<Entity>> push_obj(Octree& octree, const std::string& text,
                                                     const Material* material = nullptr, bool* ok = nullptr) {
    std::vector<std::unique_ptr<Entity>> out;
    int64_t n = 0;
    if (ok) *ok = false;
    if (gi_obj_parse(text.data(), (int64_t)text.size(), nullptr, nullptr, 0, &n) != GI_OK) {
        std::fprintf(stderr, "gi_obj_parse: %s\n", gi_last_error());
        return out;
    }
    std::vector<gi_entity_desc> d((size_t)n);
    if (n > 0 && gi_obj_parse(text.data(), (int64_t)text.size(), nullptr, d.data(), n, &n) != GI_OK) return out;
    out.reserve((size_t)n);
    for (const gi_entity_desc& t : d) {
        const double* a = t.args;
        std::unique_ptr<Entity> e(new ImpTriangle(glm::dvec3(a[0], a[1], a[2]), glm::dvec3(a[3], a[4], a[5]),
                                                  glm::dvec3(a[6], a[7], a[8])));
        if (material) e->material = *material;
        octree.push_back(e.get());
        out.push_back(std::move(e));
    }
    if (ok) *ok = true;
    return out;
}

}  // namespace gi_dropin
