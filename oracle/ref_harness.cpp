// ref_harness.cpp — TEST INFRASTRUCTURE ONLY (oracle).  Never linked into the product.
//
// Drives the *unmodified* reference headers of preon7/2019global (compiled in place from
// /root/reference/include by oracle/Makefile; outputs only into oracle/_ref/) to produce golden
// vectors for the parity tests.  Nothing in this file is reference source: it is a harness that
// builds reference objects from a .scn text file and calls the reference's own functions.
//
//   render  <scene.scn> <w> <h> <out.bin> [x0 y0 x1 y1 [stride]]
//       Per-pixel restatement of RayTracer::run's body (raytracer.h:41-84): Octree::intersect
//       (octree.h:46-68), Entity::intersect (entities.h:26), last-hit-wins selection
//       (raytracer.h:53-74), getTextureCoord (entities.h:32), Material::blinn_phong_texture
//       (material.h:48-62) and Image::setPixel's (int)(255*c) quantisation (image.h:14-16).
//       Records fp64 radiance, hit entity, (u,v), candidate count and node-test count.
//   tree    <scene.scn>                 octree structure dump (octree.h:75-129), DFS order
//   rays    <scene.scn> <rays.bin> <out.bin>   per-entity intersect KAT over a ray list
//   boxes   <boxes.bin> <out.bin>       ExpBox node test (entities.h:379-440) over (box, ray) pairs
//   kat                                 main.cpp:90-133 ad-hoc test functions, printed at %.17g
//   time    <scene.scn> <w> <h> [stride]   wall time of the per-pixel loop (CPU baseline)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <string>
#include <vector>
#include <map>
#include <chrono>
#include <fstream>
#include <sstream>

#include <glm/glm.hpp>
#include "camera.h"
#include "ray.h"
#include "material.h"
#include "bbox.h"
#include "entities.h"
#define private public   // node-level statistics need Octree::Node (octree.h:71-160)
#include "octree.h"
#undef private

struct Scene {
    glm::dvec3 omin{-20, -20, -20}, omax{20, 20, 20};
    glm::dvec3 cam_pos{-10, 0, 0}, cam_look{1, 0, 0};
    double focal = 0.1;
    glm::dvec3 light{-10, 10, 10};
    std::vector<Entity*> ents;   // push_back order
    Octree* tree = nullptr;
    std::map<const Entity*, int> index;
};

static bool load_scene(const char* path, Scene& s) {
    std::ifstream f(path);
    if (!f) { fprintf(stderr, "cannot open %s\n", path); return false; }
    std::string line;
    std::vector<std::string> order;
    while (std::getline(f, line)) {
        size_t h = line.find('#');
        if (h != std::string::npos) line = line.substr(0, h);
        std::istringstream is(line);
        std::string kw;
        if (!(is >> kw)) continue;
        std::vector<double> v;
        double x;
        while (is >> x) v.push_back(x);
        auto need = [&](size_t n) {
            if (v.size() < n) { fprintf(stderr, "bad line: %s\n", line.c_str()); exit(2); }
        };
        if (kw == "octree") { need(6); s.omin = {v[0], v[1], v[2]}; s.omax = {v[3], v[4], v[5]}; }
        else if (kw == "camera") { need(7); s.cam_pos = {v[0], v[1], v[2]}; s.cam_look = {v[3], v[4], v[5]}; s.focal = v[6]; }
        else if (kw == "light") { need(3); s.light = {v[0], v[1], v[2]}; }
        else if (kw == "impsphere") { need(7); s.ents.push_back(new ImpSphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]})); }
        else if (kw == "imptriangle") { need(9); s.ents.push_back(new ImpTriangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]})); }
        else if (kw == "expquad") { need(9); s.ents.push_back(new ExpQuad({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]})); }
        else if (kw == "expsphere") { need(7); s.ents.push_back(new ExpSphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]})); }
        else if (kw == "expcube") { need(9); s.ents.push_back(new ExpCube({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]})); }
        else if (kw == "expcone") { need(11); s.ents.push_back(new ExpCone({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, v[6], v[7], {v[8], v[9], v[10]})); }
        else if (kw == "exprectangle") { need(9); s.ents.push_back(new ExpRectangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]})); }
        else if (kw == "expbox") { need(6); s.ents.push_back(new ExpBox({v[0], v[1], v[2]}, {v[3], v[4], v[5]})); }
        else if (kw == "material") {
            need(3);
            if (s.ents.empty()) { fprintf(stderr, "material before entity\n"); exit(2); }
            Entity* e = s.ents.back();
            if (v.size() >= 6) e->material = Material(glm::dvec3{v[0], v[1], v[2]}, glm::dvec3{v[3], v[4], v[5]});
            else e->material = Material(glm::dvec3{v[0], v[1], v[2]});
            if (v.size() >= 7) e->material.specular_power = v[6];
        } else { fprintf(stderr, "unknown keyword %s\n", kw.c_str()); exit(2); }
    }
    s.tree = new Octree(s.omin, s.omax);
    for (size_t i = 0; i < s.ents.size(); ++i) {
        s.index[s.ents[i]] = (int)i;
        s.tree->push_back(s.ents[i]);
    }
    return true;
}

// Node-test counter: same DFS as Octree::Node::intersect (octree.h:132-155), counting ExpBox tests.
static long g_node_tests = 0;
static std::vector<Entity*> counted_intersect(const Octree::Node& n, const Ray& ray) {
    if (n.is_leaf()) return n._entities;
    std::vector<Entity*> out;
    for (auto i = n._children.begin(); i != n._children.end(); ++i) {
        if (i->get()->_entities.size() == 0) continue;
        ExpBox box = ExpBox(i->get()->_bbox.min, i->get()->_bbox.max);
        glm::dvec3 p{0, 0, 0}, nn{0, 0, 0};
        ++g_node_tests;
        if (box.intersect(ray, p, nn)) {
            auto c = counted_intersect(*i->get(), ray);
            out.insert(out.end(), c.begin(), c.end());
        }
    }
    return out;
}

struct PixelOut {
    double rgb[3];
    int32_t hit, u, v, ncand, nnode;
    uint8_t q[3];
};

// (int)(255*c) then QColor range check: an out-of-range channel makes the QColor invalid, which
// QImage stores as black (image.h:14-16; Qt5 QColor::setRgb).  Verified against RayTracer::run by
// oracle/ref_run.cpp.
static void quantize(const double c[3], uint8_t q[3]) {
    int r = (int)(255 * c[0]), g = (int)(255 * c[1]), b = (int)(255 * c[2]);
    if (r < 0 || r > 255 || g < 0 || g > 255 || b < 0 || b > 255) { q[0] = q[1] = q[2] = 0; return; }
    q[0] = (uint8_t)r; q[1] = (uint8_t)g; q[2] = (uint8_t)b;
}

static void render_pixel(const Scene& s, const Camera& cam, const glm::dvec3& top_left,
                         const glm::dvec3& camrea_left, const glm::dvec2& resolution, int x, int y,
                         bool count_nodes, PixelOut& o) {
    // raytracer.h:41-43
    glm::dvec3 direction = top_left - camrea_left * double(x) * resolution.x - cam.up * double(y) * resolution.y;
    Ray r = Ray(cam.pos, direction);
    std::vector<Entity*> objects;
    if (count_nodes) {
        g_node_tests = 0;
        objects = counted_intersect(s.tree->_root, r);
        o.nnode = (int32_t)g_node_tests;
    } else {
        objects = s.tree->intersect(r);
        o.nnode = -1;
    }
    glm::dvec3 intersect = glm::dvec3{DBL_MAX, DBL_MAX, DBL_MAX};
    glm::dvec3 normal = glm::dvec3{0, 0, 0};
    Entity* front_obj = nullptr;   // A.8: the reference leaves this uninitialised for pixel 0
    for (size_t i = 0; i < objects.size(); i++) {
        glm::dvec3 ci{0, 0, 0}, cn{0, 0, 0};
        double min_dist_square = DBL_MAX;   // re-declared per candidate: last hit wins (A.1)
        if (objects[i]->intersect(r, ci, cn)) {
            auto pt = ci - r.origin;
            double d2 = pow(pt.x, 2) + pow(pt.y, 2) + pow(pt.z, 2);
            if (d2 < min_dist_square) {
                intersect = ci;
                normal = cn;
                front_obj = objects[i];
            }
        }
    }
    o.ncand = (int32_t)objects.size();
    if (front_obj) {
        auto coord = front_obj->getTextureCoord(intersect);
        glm::dvec3 c = front_obj->material.blinn_phong_texture(r, s.light, intersect, normal,
                                                               std::get<0>(coord), std::get<1>(coord));
        o.rgb[0] = c.x; o.rgb[1] = c.y; o.rgb[2] = c.z;
        o.hit = s.index.at(front_obj);
        o.u = std::get<0>(coord);
        o.v = std::get<1>(coord);
    } else {
        o.rgb[0] = o.rgb[1] = o.rgb[2] = 0.0;
        o.hit = -1; o.u = o.v = 0;
    }
    quantize(o.rgb, o.q);
}

struct Frame {
    Camera cam;
    glm::dvec3 top_left, left;
    glm::dvec2 res{0.0002, 0.0002};
    Frame(const Scene& s, int w) : cam(s.cam_pos, s.cam_look, s.focal) {
        // raytracer.h:26-30 (vertical offset uses w, A.12)
        left = glm::normalize(glm::cross(cam.up, cam.forward));
        top_left = (cam.pos + cam.focalDist * cam.forward + left * double(w) * 0.5 * res.x +
                    cam.up * double(w) * 0.5 * res.y) - cam.pos;
    }
};

static int cmd_render(int argc, char** argv) {
    Scene s;
    if (!load_scene(argv[2], s)) return 1;
    int w = atoi(argv[3]), h = atoi(argv[4]);
    const char* out = argv[5];
    int x0 = 0, y0 = 0, x1 = w, y1 = h, stride = 1;
    if (argc >= 10) { x0 = atoi(argv[6]); y0 = atoi(argv[7]); x1 = atoi(argv[8]); y1 = atoi(argv[9]); }
    if (argc >= 11) stride = atoi(argv[10]);
    Frame fr(s, w);
    std::vector<int32_t> xs, ys;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x)
            if (((long)y * w + x) % stride == 0) { xs.push_back(x); ys.push_back(y); }
    size_t n = xs.size();
    std::vector<double> rgb(n * 3);
    std::vector<int32_t> hit(n), uv(n * 2), ncand(n), nnode(n);
    std::vector<uint8_t> q(n * 3);
    for (size_t i = 0; i < n; ++i) {
        PixelOut o;
        render_pixel(s, fr.cam, fr.top_left, fr.left, fr.res, xs[i], ys[i], true, o);
        memcpy(&rgb[i * 3], o.rgb, 24);
        hit[i] = o.hit; uv[2 * i] = o.u; uv[2 * i + 1] = o.v; ncand[i] = o.ncand; nnode[i] = o.nnode;
        memcpy(&q[i * 3], o.q, 3);
    }
    FILE* f = fopen(out, "wb");
    if (!f) return 1;
    const char magic[8] = {'G', 'I', 'R', 'E', 'F', '1', 0, 0};
    int32_t hdr[4] = {w, h, (int32_t)n, 0};
    fwrite(magic, 1, 8, f);
    fwrite(hdr, 4, 4, f);
    fwrite(xs.data(), 4, n, f);
    fwrite(ys.data(), 4, n, f);
    fwrite(rgb.data(), 8, n * 3, f);
    fwrite(hit.data(), 4, n, f);
    fwrite(uv.data(), 4, n * 2, f);
    fwrite(ncand.data(), 4, n, f);
    fwrite(nnode.data(), 4, n, f);
    fwrite(q.data(), 1, n * 3, f);
    fclose(f);
    return 0;
}

static void dump_node(const Scene& s, const Octree::Node& n, int depth, int slot) {
    printf("node %d %d %d %.17g %.17g %.17g %.17g %.17g %.17g %zu", depth, slot, n.is_leaf() ? 1 : 0,
           n._bbox.min.x, n._bbox.min.y, n._bbox.min.z, n._bbox.max.x, n._bbox.max.y, n._bbox.max.z,
           n._entities.size());
    for (auto* e : n._entities) printf(" %d", s.index.at(e));
    printf("\n");
    if (!n.is_leaf())
        for (int c = 0; c < 8; ++c) dump_node(s, *n._children[c], depth + 1, c);
}

static int cmd_tree(char** argv) {
    Scene s;
    if (!load_scene(argv[2], s)) return 1;
    for (size_t i = 0; i < s.ents.size(); ++i) {
        BoundingBox b = s.ents[i]->boundingBox();
        printf("bbox %zu %.17g %.17g %.17g %.17g %.17g %.17g\n", i, b.min.x, b.min.y, b.min.z, b.max.x, b.max.y, b.max.z);
    }
    dump_node(s, s.tree->_root, 0, -1);
    return 0;
}

// rays.bin: int32 n, then n × (origin[3], dir[3]) doubles; dir is passed through Ray's ctor
// (ray.h:6, normalises).  Output per (ray, entity): int32 hit, double P[3], N[3], int32 u, v.
static int cmd_rays(char** argv) {
    Scene s;
    if (!load_scene(argv[2], s)) return 1;
    FILE* f = fopen(argv[3], "rb");
    if (!f) return 1;
    int32_t n = 0;
    if (fread(&n, 4, 1, f) != 1) return 1;
    std::vector<double> rr((size_t)n * 6);
    if (fread(rr.data(), 8, rr.size(), f) != rr.size()) return 1;
    fclose(f);
    FILE* o = fopen(argv[4], "wb");
    for (int i = 0; i < n; ++i) {
        Ray r({rr[6 * i], rr[6 * i + 1], rr[6 * i + 2]}, {rr[6 * i + 3], rr[6 * i + 4], rr[6 * i + 5]});
        for (auto* e : s.ents) {
            glm::dvec3 p{0, 0, 0}, nn{0, 0, 0};
            int32_t hit = e->intersect(r, p, nn) ? 1 : 0;
            int32_t uv[2] = {0, 0};
            if (hit) { auto c = e->getTextureCoord(p); uv[0] = std::get<0>(c); uv[1] = std::get<1>(c); }
            double pn[6] = {p.x, p.y, p.z, nn.x, nn.y, nn.z};
            fwrite(&hit, 4, 1, o);
            fwrite(pn, 8, 6, o);
            fwrite(uv, 4, 2, o);
        }
    }
    fclose(o);
    return 0;
}

// boxes.bin: int32 n, then n × (min[3], max[3], origin[3], dir[3]).  Output: int32 hit per record.
static int cmd_boxes(char** argv) {
    FILE* f = fopen(argv[2], "rb");
    if (!f) return 1;
    int32_t n = 0;
    if (fread(&n, 4, 1, f) != 1) return 1;
    std::vector<double> b((size_t)n * 12);
    if (fread(b.data(), 8, b.size(), f) != b.size()) return 1;
    fclose(f);
    std::vector<int32_t> out(n);
    for (int i = 0; i < n; ++i) {
        const double* q = &b[12 * (size_t)i];
        ExpBox box({q[0], q[1], q[2]}, {q[3], q[4], q[5]});
        Ray r({q[6], q[7], q[8]}, {q[9], q[10], q[11]});
        glm::dvec3 p{0, 0, 0}, nn{0, 0, 0};
        out[i] = box.intersect(r, p, nn) ? 1 : 0;
    }
    FILE* o = fopen(argv[3], "wb");
    fwrite(out.data(), 4, n, o);
    fclose(o);
    return 0;
}

static void pv(const char* name, glm::dvec3 v) { printf("%s %.17g %.17g %.17g\n", name, v.x, v.y, v.z); }

static int cmd_kat() {
    {   // main.cpp:90-104 entity_test
        ImpSphere s = ImpSphere(glm::dvec3{2, 0, 0}, 10, {0, 1, 0});
        Ray r = Ray(glm::dvec3{-10, 0, 0}, glm::dvec3{1, 0.5, 0.5});
        glm::dvec3 p{0, 0, 0}, n{0, 0, 0};
        printf("entity_test.hit %d\n", s.intersect(r, p, n) ? 1 : 0);
        pv("entity_test.point", p);
        pv("entity_test.normal", n);
    }
    {   // main.cpp:126-133 bbox_test
        BoundingBox b1 = BoundingBox(glm::dvec3{0, 0, 0}, glm::dvec3{2, 2, 2});
        BoundingBox b2 = BoundingBox(glm::dvec3{-2, -2, 0}, glm::dvec3{1, 1, 2});
        printf("bbox_test.intersect %d\n", b1.intersect(b2) ? 1 : 0);
        printf("bbox_test.contains %d\n", b1.contains(glm::dvec3{1, 1, 1}) ? 1 : 0);
    }
    {   // main.cpp:106-124 matrix_test
        glm::dvec3 a{1, 0, 1}, b{0, 2.5, 0}, c{3, 3, 3};
        glm::mat3 m = glm::transpose(glm::mat3(a, b, c));
        for (int i = 0; i < 3; ++i) printf("matrix_test.col%d %.9g %.9g %.9g\n", i, m[i][0], m[i][1], m[i][2]);
        printf("matrix_test.dot %.17g\n", glm::dot(a, b));
    }
    return 0;
}

static int cmd_time(int argc, char** argv) {
    Scene s;
    if (!load_scene(argv[2], s)) return 1;
    int w = atoi(argv[3]), h = atoi(argv[4]);
    int stride = argc >= 6 ? atoi(argv[5]) : 1;
    Frame fr(s, w);
    auto t0 = std::chrono::steady_clock::now();
    long n = 0;
    double sum = 0;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            if (((long)y * w + x) % stride) continue;
            PixelOut o;
            render_pixel(s, fr.cam, fr.top_left, fr.left, fr.res, x, y, false, o);
            sum += o.q[0] + o.q[1] + o.q[2];
            ++n;
        }
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    printf("{\"rays\": %ld, \"seconds\": %.6f, \"mray_s\": %.6f, \"checksum\": %.0f}\n", n, sec, n / sec * 1e-6, sum);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ref_harness render|tree|rays|boxes|kat|time ...\n"); return 2; }
    std::string c = argv[1];
    if (c == "render" && argc >= 6) return cmd_render(argc, argv);
    if (c == "tree" && argc >= 3) return cmd_tree(argv);
    if (c == "rays" && argc >= 5) return cmd_rays(argv);
    if (c == "boxes" && argc >= 4) return cmd_boxes(argv);
    if (c == "kat") return cmd_kat();
    if (c == "time" && argc >= 5) return cmd_time(argc, argv);
    fprintf(stderr, "bad arguments\n");
    return 2;
}
