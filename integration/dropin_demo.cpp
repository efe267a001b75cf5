// dropin_demo.cpp — the reference application's render path with the drop-in headers.
//
// Builds the main.cpp scene (main.cpp:24-48) with the reference's own, unmodified Camera /
// ImpSphere / ExpQuad / Image classes, then renders it with gi_dropin/raytracer.h (same class
// name and API as the reference's RayTracer), copying the RayTracer by value as Gui/Viewer do
// (gui.h:19,35).  Writes the RGB888 frame the Viewer would paint.
// With "zoo" it builds the every-entity scene of scenes.zoo_scene() instead (entities.h's eight
// entity classes, constructed by the reference's own constructors).
// With "obj:<path>" it pushes the Wavefront OBJ mesh at <path> instead, through
// gi_dropin/obj.h's push_obj (one ImpTriangle per fan triangle, white Material(color)).
// With "scn:<path>" it builds the scene of a .scn file (scenes.py Scene.to_scn: octree, camera,
// light, imptriangle / impsphere entities with their material lines) with the reference's classes.
// With a 5th argument "cands" it writes, instead of a frame, the length of the drop-in
// Octree::intersect(const Ray&) candidate list (octree.h:46-68) for every pixel's primary ray
// (raytracer.h:26-30, 41-43), as int32 -- compared with the compiled reference's lists; with "rad"
// it writes the frame's fp64 radiance (RayTracer::keepRadiance) instead of its RGB888.
// The integrator is the drop-in's default (the reference's, Mode R) unless the environment opts in
// (GI_MODE=X GI_SPP=.. GI_DEPTH=.. GI_SEED=.. [GI_PASS=..], read by the drop-in RayTracer's
// constructor).  DEMO_STOP_AFTER=k stops the frame after k progressive passes (RayTracer::stop from
// the pass callback, as a Viewer resize would); the demo prints the passes delivered to stderr.
// Exit status: 0 on a delivered frame (or one stopped by DEMO_STOP_AFTER), 3 when the drop-in
// RayTracer reports an error (RayTracer::lastStatus(): a libgi of another ABI, a failed upload or
// render -- the Image would be black), 1/2 on the demo's own input errors.  `dropin_demo --abi`
// prints the GI_ABI_VERSION it was compiled against (tests refuse a stale build).
//   dropin_demo <w> <h> <out> [zoo|main|obj:<path>|scn:<path>] [cands|rad]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>

#include "raytracer.h"   // resolves to include/gi_dropin/raytracer.h (first on the include path)
#include "obj.h"

// The subset of the .scn format the demo needs: octree / camera / light lines, ImpTriangle and
// ImpSphere entities, and the material line that follows an entity (color, shader, specular power;
// an optional Mode X reflectivity has no reference counterpart and must be 0 here).
struct ScnScene {
    glm::dvec3 omin{-20, -20, -20}, omax{20, 20, 20}, cam_pos{-10, 0, 0}, cam_look{1, 0, 0}, light{-10, 10, 10};
    double focal = 0.1;
    std::vector<Entity*> ents;
};
bool read_scn(const std::string& path, ScnScene& sc) {
    std::ifstream in(path);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string kw;
        if (!(ls >> kw) || kw[0] == '#') continue;
        std::vector<double> v;
        for (double x; ls >> x;) v.push_back(x);
        if (kw == "octree" && v.size() == 6) { sc.omin = {v[0], v[1], v[2]}; sc.omax = {v[3], v[4], v[5]}; }
        else if (kw == "camera" && v.size() == 7) { sc.cam_pos = {v[0], v[1], v[2]}; sc.cam_look = {v[3], v[4], v[5]}; sc.focal = v[6]; }
        else if (kw == "light" && v.size() == 3) sc.light = {v[0], v[1], v[2]};
        else if (kw == "imptriangle" && v.size() == 9)
            sc.ents.push_back(new ImpTriangle(glm::dvec3{v[0], v[1], v[2]}, glm::dvec3{v[3], v[4], v[5]}, glm::dvec3{v[6], v[7], v[8]}));
        else if (kw == "impsphere" && v.size() == 7)
            sc.ents.push_back(new ImpSphere(glm::dvec3{v[0], v[1], v[2]}, (float)v[3], glm::dvec3{v[4], v[5], v[6]}));
        else if (kw == "material" && (v.size() == 7 || (v.size() == 8 && v[7] == 0.0)) && !sc.ents.empty()) {
            sc.ents.back()->material = Material(glm::dvec3{v[0], v[1], v[2]}, glm::dvec3{v[3], v[4], v[5]});
            sc.ents.back()->material.specular_power = v[6];
        } else {
            std::fprintf(stderr, "scn: unsupported line: %s\n", line.c_str());
            return false;
        }
    }
    return !sc.ents.empty();
}

int main(int argc, char** argv) {
    if (argc == 2 && std::string(argv[1]) == "--abi") { std::printf("%d\n", GI_ABI_VERSION); return 0; }
    if (argc < 4) { std::fprintf(stderr, "usage: dropin_demo w h out.rgb\n"); return 2; }
    const int w = std::atoi(argv[1]), h = std::atoi(argv[2]);
    ScnScene scn;
    const bool from_scn = argc > 4 && std::string(argv[4]).rfind("scn:", 0) == 0;
    if (from_scn && !read_scn(std::string(argv[4]).substr(4), scn)) return 1;
    Camera camera = from_scn ? Camera(scn.cam_pos, scn.cam_look, scn.focal) : Camera({-10, 0, 0}, {1, 0, 0}, 0.1);
    glm::dvec3 light = from_scn ? scn.light : glm::dvec3{-10, 10, 10};
    RayTracer raytracer(camera, light);
    Octree scene(from_scn ? scn.omin : glm::dvec3{-20, -20, -20}, from_scn ? scn.omax : glm::dvec3{20, 20, 20});
    std::vector<std::unique_ptr<Entity>> mesh;   // push_obj's entities, alive as long as the scene
    if (from_scn) {
        for (Entity* e : scn.ents) scene.push_back(e);
    } else if (argc > 4 && std::string(argv[4]).rfind("obj:", 0) == 0) {
        std::ifstream in(std::string(argv[4]).substr(4), std::ios::binary);
        std::stringstream text;
        text << in.rdbuf();
        const Material white(glm::dvec3{1, 1, 1});
        bool ok = false;
        mesh = gi_dropin::push_obj(scene, text.str(), &white, &ok);
        if (!in || !ok) return 1;
    } else if (argc > 4 && std::string(argv[4]) == "zoo") {
        scene.push_back(new ExpSphere(glm::dvec3{-2, 0, 0}, 2, {0, 1, 0}));
        scene.push_back(new ExpCube(glm::dvec3{0, 0, 0}, 2, 2, 2, {1, 0, 0}));
        scene.push_back(new ExpCone(glm::dvec3{0, 0, 2}, glm::dvec3{-1, 1, -3}, 5, 3, {1, 1, 0}));
        scene.push_back(new ExpQuad(glm::dvec3{0, 0, 0}, 2, 3, (90.0 * M_PI / 180.0), {1, 2, 3}));
        scene.push_back(new ImpSphere(glm::dvec3{3, 4, 4}, 2, {1, 0, 0}));
        ImpTriangle* t = new ImpTriangle(glm::dvec3{0, 3, 2}, glm::dvec3{3, 3, -4}, glm::dvec3{3, -3, -4});
        t->material = Material(glm::dvec3{0, 1, 1}, glm::dvec3{0.1, 0.7, 1.0});
        t->material.specular_power = 5;
        scene.push_back(t);
        scene.push_back(new ExpRectangle(glm::dvec3{1, -6, -3}, glm::dvec3{1, -3, 0}, glm::dvec3{1, -6, 0}));
        scene.push_back(new ExpBox(glm::dvec3{2, 4, -5}, glm::dvec3{4, 6, -3}));
    } else {
        ImpSphere* s2 = new ImpSphere(glm::dvec3{3, 4, 4}, 2, {1, 0, 0});
        ImpSphere* s3 = new ImpSphere(glm::dvec3{4, -4, 4}, 2, {0, 0, 1});
        ExpQuad* q = new ExpQuad(glm::dvec3{0, 0, 0}, 2, 3, (90.0 * M_PI / 180.0), {1, 2, 3});
        scene.push_back(q);
        scene.push_back(s2);
        scene.push_back(s3);
    }
    if (argc > 5 && std::string(argv[5]) == "cands") {
        // raytracer.h:26-30 (vertical offset from w, A.12) and :41-43
        const glm::dvec3 left = glm::normalize(glm::cross(camera.up, camera.forward));
        const glm::dvec2 res{0.0002, 0.0002};
        const glm::dvec3 top_left = ((camera.pos + camera.focalDist * camera.forward) + left * (double)w * 0.5 * res.x +
                                     camera.up * (double)w * 0.5 * res.y) - camera.pos;
        FILE* f = std::fopen(argv[3], "wb");
        if (!f) return 1;
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x) {
                const glm::dvec3 dir = top_left - left * (double)x * res.x - camera.up * (double)y * res.y;
                const int32_t n = (int32_t)scene.intersect(Ray(camera.pos, dir)).size();
                std::fwrite(&n, 4, 1, f);
            }
        std::fclose(f);
        return 0;
    }
    raytracer.setScene(&scene);
    const bool rad = argc > 5 && std::string(argv[5]) == "rad";
    RayTracer viewer_copy = raytracer;
    viewer_copy.keepRadiance(rad);
    if (const char* sa = std::getenv("DEMO_STOP_AFTER")) {
        const int k = std::atoi(sa);
        viewer_copy.setPassCallback([&viewer_copy, k](int passes, int) {
            if (passes >= k) viewer_copy.stop();
        });
    }
    viewer_copy.start();
    viewer_copy.run(w, h);
    std::fprintf(stderr, "passes %d\n", viewer_copy.passesDelivered());
    if (viewer_copy.lastStatus() != GI_OK && viewer_copy.lastStatus() != GI_ERR_CANCELLED) {
        std::fprintf(stderr, "dropin_demo: RayTracer::run failed (status %d): %s\n", viewer_copy.lastStatus(),
                     viewer_copy.lastError().c_str());
        return 3;
    }
    std::shared_ptr<Image> img = viewer_copy.getImage();
    if (img->width() != w || img->height() != h) return 1;
    FILE* f = std::fopen(argv[3], "wb");
    if (!f) return 1;
    if (rad) {
        const std::vector<double>& r = viewer_copy.radiance();
        const bool ok = r.size() == (size_t)w * h * 3 && std::fwrite(r.data(), sizeof(double), r.size(), f) == r.size();
        std::fclose(f);
        return ok ? 0 : 1;
    }
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const glm::dvec3 p = img->getPixel(x, y);
            const unsigned char px[3] = {(unsigned char)(p.x * 255. + 0.5), (unsigned char)(p.y * 255. + 0.5),
                                         (unsigned char)(p.z * 255. + 0.5)};
            std::fwrite(px, 1, 3, f);
        }
    std::fclose(f);
    return 0;
}
