// ref_run.cpp — TEST INFRASTRUCTURE ONLY (oracle).  Runs the reference's own RayTracer::run
// (raytracer.h:23-87) end to end, including its QImage-backed Image (image.h:7-29), and writes the
// 8-bit RGB888 frame.  Used once per scene to confirm that ref_harness's per-pixel restatement of
// raytracer.h:41-84 reproduces RayTracer::run exactly (tests/test_oracle_golden.py).
//
//   ref_run <scene.scn> <w> <h> <out.rgb>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <glm/glm.hpp>
#include "raytracer.h"

int main(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: ref_run scene.scn w h out.rgb\n"); return 2; }
    std::ifstream f(argv[1]);
    if (!f) return 1;
    glm::dvec3 omin{-20, -20, -20}, omax{20, 20, 20}, cpos{-10, 0, 0}, clook{1, 0, 0}, light{-10, 10, 10};
    double focal = 0.1;
    std::vector<Entity*> ents;
    std::string line;
    while (std::getline(f, line)) {
        size_t h = line.find('#');
        if (h != std::string::npos) line = line.substr(0, h);
        std::istringstream is(line);
        std::string kw;
        if (!(is >> kw)) continue;
        std::vector<double> v;
        double x;
        while (is >> x) v.push_back(x);
        if (kw == "octree") { omin = {v[0], v[1], v[2]}; omax = {v[3], v[4], v[5]}; }
        else if (kw == "camera") { cpos = {v[0], v[1], v[2]}; clook = {v[3], v[4], v[5]}; focal = v[6]; }
        else if (kw == "light") light = {v[0], v[1], v[2]};
        else if (kw == "impsphere") ents.push_back(new ImpSphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}));
        else if (kw == "imptriangle") ents.push_back(new ImpTriangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]}));
        else if (kw == "expquad") ents.push_back(new ExpQuad({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]}));
        else if (kw == "expsphere") ents.push_back(new ExpSphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}));
        else if (kw == "expcube") ents.push_back(new ExpCube({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]}));
        else if (kw == "expcone") ents.push_back(new ExpCone({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, v[6], v[7], {v[8], v[9], v[10]}));
        else if (kw == "exprectangle") ents.push_back(new ExpRectangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]}));
        else if (kw == "expbox") ents.push_back(new ExpBox({v[0], v[1], v[2]}, {v[3], v[4], v[5]}));
        else if (kw == "material") {
            Entity* e = ents.back();
            if (v.size() >= 6) e->material = Material(glm::dvec3{v[0], v[1], v[2]}, glm::dvec3{v[3], v[4], v[5]});
            else e->material = Material(glm::dvec3{v[0], v[1], v[2]});
            if (v.size() >= 7) e->material.specular_power = v[6];
        }
    }
    Octree scene(omin, omax);
    for (auto* e : ents) scene.push_back(e);
    Camera camera(cpos, clook, focal);
    RayTracer rt(camera, light);
    rt.setScene(&scene);
    rt.start();
    int w = atoi(argv[2]), hh = atoi(argv[3]);
    rt.run(w, hh);
    std::shared_ptr<Image> img = rt.getImage();
    FILE* o = fopen(argv[4], "wb");
    for (int y = 0; y < hh; ++y)
        for (int x = 0; x < w; ++x) {
            glm::dvec3 p = img->getPixel(x, y);   // qRed/255. etc. (image.h:18-21)
            unsigned char px[3] = {(unsigned char)(p.x * 255. + 0.5), (unsigned char)(p.y * 255. + 0.5),
                                   (unsigned char)(p.z * 255. + 0.5)};
            fwrite(px, 1, 3, o);
        }
    fclose(o);
    return 0;
}
