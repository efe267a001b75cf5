// gi_build.cpp — host-side scene construction for libgi (compiled by g++ -ffp-contract=off).
//
// Entities are built exactly as the reference constructors build them (own restatement):
//   ImpSphere   entities.h:45-47, bbox :98-99 (member-init while pos == {0,0,0})
//   ImpTriangle entities.h:138-148, bbox :251-275 (+0.01 on max.z, +1e-5 on flat axes, A.13)
//   ExpQuad     entities.h:581-590 (float trig on the float alpha), bbox :623-624 (A.5)
//   ExpSphere   entities.h:461-506 (fp32 stack/sector trig, vertices offset by -pos; intersect()
//               skips triangle 0, :520), bbox origin-centred (A.5)
//   ExpCube     entities.h:652-727 (12 triangles, texture frame vertices[0])
//   ExpCone     entities.h:823-899 (fixed axis (-1,0,-10), fp32 glm::mat3 rotations, 50 sectors)
//   ExpRectangle entities.h:310-340 (t1 = (p1,p2,p3), t2 = (p1,p2,-p3): p4 = -p3, A.4)
//   ExpBox      entities.h:381-446 (6 faces x (t1, t2 with the third corner negated))
// then pushed into the reference octree with Octree::push_back semantics (octree.h:20-129,
// bbox.h:25-39), including the silent drop (A.14) and entities kept only at the split node (A.6).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gi.h"
#include "gi_scene.h"

namespace gi {

namespace {

struct BEnt {
    REnt rec;
    V3 bmin, bmax;
    std::vector<TriRec> tris;
};

REnt blank_rec(int kind) {
    REnt r;
    memset(&r, 0, sizeof r);
    r.kind = kind;
    r.color[0] = 1; r.color[1] = 0; r.color[2] = 0;   // Entity() : Material(dvec3(1,0,0)) (entities.h:21)
    r.shader[0] = 0.1; r.shader[1] = 0.7; r.shader[2] = 1.0;   // material.h:27
    r.spec_pow = 5.0;                                          // material.h:29
    return r;
}

void set_color(REnt& r, const double* c) { r.color[0] = c[0]; r.color[1] = c[1]; r.color[2] = c[2]; }

bool build_entity(const gi_entity_desc& d, BEnt& e, std::string& err) {
    const double* a = d.args;
    switch (d.kind) {
    case GI_IMP_SPHERE: {
        e.rec = blank_rec(K_IMP_SPHERE);
        set_color(e.rec, a + 4);
        e.rec.radius = (float)a[3];
        e.rec.pos[0] = a[0]; e.rec.pos[1] = a[1]; e.rec.pos[2] = a[2];
        const double r = e.rec.radius;
        e.bmin = v3((float)(0.0 - r), (float)(0.0 - r), (float)(0.0 - r));
        e.bmax = v3((float)(0.0 + r), (float)(0.0 + r), (float)(0.0 + r));
        break;
    }
    case GI_IMP_TRIANGLE: {
        e.rec = blank_rec(K_IMP_TRIANGLE);
        TriRec t;
        const V3 p1 = v3(a[0], a[1], a[2]), p2 = v3(a[3], a[4], a[5]), p3 = v3(a[6], a[7], a[8]);
        make_tri(p1, p2, p3, t);
        e.tris.push_back(t);
        e.rec.pos[0] = t.pos[0]; e.rec.pos[1] = t.pos[1]; e.rec.pos[2] = t.pos[2];
        {   // getTextureCoord's per-triangle constants (entities.h:277-303), same fp64 ops as per hit
            const V3 p21 = p2 - p1, p31 = p3 - p1, p32 = p3 - p2;
            st3(e.rec.qv0, p1);
            st3(e.rec.qv1, p21);
            e.rec.qv2[0] = gsqrt(sq3(p21));                            // |p2 - p1|
            e.rec.qv2[1] = gsqrt(sq3(0.5 * (p21 + p31))) / 160.0;      // unit_v
            e.rec.qv2[2] = gsqrt(sq3(0.5 * ((-p32) + (-p31)))) / 160.0;   // unit_h
        }
        e.bmin = v3(smin(smin(p1.x, p2.x), p3.x), smin(smin(p1.y, p2.y), p3.y), smin(smin(p1.z, p2.z), p3.z));
        e.bmax = v3(smax(smax(p1.x, p2.x), p3.x), smax(smax(p1.y, p2.y), p3.y), smax(smax(p1.z, p2.z), p3.z) + 0.01);
        if (e.bmax.x == e.bmin.x) e.bmax.x += 1e-5;
        if (e.bmax.y == e.bmin.y) e.bmax.y += 1e-5;
        if (e.bmax.z == e.bmin.z) e.bmax.z += 1e-5;
        break;
    }
    case GI_EXP_QUAD: {
        e.rec = blank_rec(K_EXP_QUAD);
        set_color(e.rec, a + 6);
        const V3 pos = v3(a[0], a[1], a[2]);
        e.rec.pos[0] = pos.x; e.rec.pos[1] = pos.y; e.rec.pos[2] = pos.z;
        const float w = (float)a[3], l = (float)a[4], al = (float)a[5];
        e.rec.width = w; e.rec.length = l; e.rec.alpha = al;
        const float hw = w / 2, hl = l / 2;
        const double ca = (double)std::cos(al), sa = (double)std::sin(al);   // float overloads (cosf/sinf)
        V3 q[4];
        q[0] = v3((pos.x + hw) * ca, pos.y + hl, pos.z + (pos.x + hw) * sa);
        q[1] = v3((pos.x - hw) * ca, pos.y + hl, pos.z + (pos.x - hw) * sa);
        q[2] = v3((pos.x + hw) * ca, pos.y - hl, pos.z + (pos.x + hw) * sa);
        q[3] = v3((pos.x - hw) * ca, pos.y - hl, pos.z + pos.z + (pos.x - hw) * sa);   // entities.h:586
        TriRec t0, t1;
        make_tri(q[1], q[2], q[0], t0);   // entities.h:588
        make_tri(q[1], q[3], q[2], t1);   // entities.h:589
        e.tris.push_back(t0);
        e.tris.push_back(t1);
        st3(e.rec.qv0, q[0]);
        st3(e.rec.qv1, q[1]);
        e.bmin = v3((float)(0.0 - hw), (float)(0.0 - hl), (float)0.0);
        e.bmax = v3((float)(0.0 + hw), (float)(0.0 + hl), (float)(0.0 + (0.0 + hw) * sa));
        break;
    }
    case GI_EXP_SPHERE: {
        e.rec = blank_rec(K_EXP_SPHERE);
        set_color(e.rec, a + 4);
        const V3 pos = v3(a[0], a[1], a[2]);
        st3(e.rec.pos, pos);
        const float rad = (float)a[3];
        e.rec.radius = rad;
        const int nsec = 10, nstk = 10;
        const float sec_step = (float)(2 * REF_PI / nsec), stk_step = (float)(REF_PI / nstk);
        std::vector<V3> vert;
        for (int i = 0; i <= nstk; ++i) {
            const float stk = (float)(REF_PI / 2 - (double)(i * stk_step));
            const float xy = rad * cosf(stk);
            const float z = (float)((double)(rad * sinf(stk)) - pos.z);
            for (int j = 0; j <= nsec; ++j) {
                const float sec = j * sec_step;
                vert.push_back(v3((float)((double)(xy * cosf(sec)) - pos.x), (float)((double)(xy * sinf(sec)) - pos.y), z));
            }
        }
        bool first = true;   // intersect() starts at triangle 1 (entities.h:520)
        for (int i = 0; i < nstk; ++i) {
            int k1 = i * (nsec + 1), k2 = k1 + nsec + 1;
            for (int j = 0; j < nsec; ++j, ++k1, ++k2) {
                TriRec t;
                if (i != 0) {
                    make_tri(vert[k1], vert[k2], vert[k1 + 1], t);
                    if (!first) e.tris.push_back(t);
                    first = false;
                }
                if (i != nstk - 1) {
                    make_tri(vert[k1 + 1], vert[k2], vert[k2 + 1], t);
                    if (!first) e.tris.push_back(t);
                    first = false;
                }
            }
        }
        const double r = rad;
        e.bmin = v3((float)(0.0 - r), (float)(0.0 - r), (float)(0.0 - r));
        e.bmax = v3((float)(0.0 + r), (float)(0.0 + r), (float)(0.0 + r));
        break;
    }
    case GI_EXP_CUBE: {
        e.rec = blank_rec(K_EXP_CUBE);
        set_color(e.rec, a + 6);
        const V3 pos = v3(a[0], a[1], a[2]);
        st3(e.rec.pos, pos);
        const float w = (float)a[3], l = (float)a[4], h = (float)a[5];
        e.rec.width = w; e.rec.length = l; e.rec.height = h;
        const float hw = w / 2, hl = l / 2, hh = h / 2;
        const V3 c[8] = {v3(pos.x - hw, pos.y - hl, pos.z - hh), v3(pos.x - hw, pos.y - hl, pos.z + hh),
                         v3(pos.x + hw, pos.y - hl, pos.z - hh), v3(pos.x + hw, pos.y - hl, pos.z + hh),
                         v3(pos.x - hw, pos.y + hl, pos.z + hh), v3(pos.x - hw, pos.y + hl, pos.z - hh),
                         v3(pos.x + hw, pos.y + hl, pos.z - hh), v3(pos.x + hw, pos.y + hl, pos.z + hh)};
        static const int F[12][3] = {{0, 1, 2}, {3, 1, 2}, {4, 5, 7}, {7, 5, 6}, {1, 0, 4}, {4, 0, 5},
                                     {3, 7, 2}, {7, 6, 2}, {1, 4, 3}, {3, 4, 7}, {0, 5, 2}, {2, 5, 6}};
        for (const auto& f : F) {
            TriRec t;
            make_tri(c[f[0]], c[f[1]], c[f[2]], t);
            e.tris.push_back(t);
        }
        st3(e.rec.qv0, c[0]);
        e.bmin = v3((float)(0.0 - hw), (float)(0.0 - hl), (float)(0.0 - hh));
        e.bmax = v3((float)(0.0 + hw), (float)(0.0 + hl), (float)(0.0 + hh));
        break;
    }
    case GI_EXP_CONE: {
        e.rec = blank_rec(K_EXP_CONE);
        set_color(e.rec, a + 8);
        const V3 pos = v3(a[0], a[1], a[2]);
        st3(e.rec.pos, pos);
        const float h = (float)a[6], rad = (float)a[7];
        e.rec.height = h; e.rec.radius = rad;
        const V3 axis = normalize(v3(-1, 0, -10));   // entities.h:825 overrides the argument
        // glm::mat3 (fp32, column-major m[col][row]) rotations about x then y, applied to a vec3
        float rx[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, ry[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        const V3 xd = v3(0, axis.y, axis.z);
        if (!(xd.x == 0 && xd.y == 0 && xd.z == 0)) {
            const double ang = (axis.y < 0 ? 1.0 : -1.0) * std::acos(dot(normalize(xd), v3(0, 0, -1)));
            rx[1][1] = (float)std::cos(ang); rx[1][2] = (float)(-std::sin(ang));
            rx[2][1] = (float)std::sin(ang); rx[2][2] = (float)std::cos(ang);
        }
        const V3 yd = v3(axis.x, 0, -std::sqrt(axis.z * axis.z + axis.y * axis.y));
        if (!(yd.x == 0 && yd.y == 0 && yd.z == 0)) {
            const double ang = (axis.x > 0 ? 1.0 : -1.0) * std::acos(dot(normalize(yd), v3(0, 0, -1)));
            ry[0][0] = (float)std::cos(ang); ry[0][2] = (float)std::sin(ang);
            ry[2][0] = (float)(-std::sin(ang)); ry[2][2] = (float)std::cos(ang);
        }
        auto rot = [](const float m[3][3], V3 v) {
            const float x = (float)v.x, y = (float)v.y, z = (float)v.z;
            return v3(m[0][0] * x + m[1][0] * y + m[2][0] * z, m[0][1] * x + m[1][1] * y + m[2][1] * z,
                      m[0][2] * x + m[1][2] * y + m[2][2] * z);
        };
        std::vector<V3> rim;
        const double nsub = 50.0;
        for (int i = 0; i <= nsub; ++i) {
            const float deg = (float)(i * 360.0 / nsub);
            V3 p = v3(pos.x + (double)rad * std::cos((double)deg * REF_PI / 180.0),
                      pos.y + (double)rad * std::sin((double)deg * REF_PI / 180.0), pos.z - (double)h);
            p = rot(ry, rot(rx, p - pos)) + pos;
            rim.push_back(p);
        }
        const V3 base = pos + normalize(axis) * (double)h;
        for (size_t i = 0; i + 1 < rim.size(); ++i) {
            TriRec t;
            make_tri(pos, rim[i], rim[i + 1], t);
            e.tris.push_back(t);
            make_tri(base, rim[i], rim[i + 1], t);
            e.tris.push_back(t);
        }
        const double theta = (double)std::atan(rad / h);   // float atan (entities.h:950)
        e.rec.sin_theta = std::sin(theta);
        e.bmin = v3((float)(0.0 - (double)rad), (float)(0.0 - (double)rad), (float)(0.0 - (double)h));
        e.bmax = v3((float)(0.0 + (double)rad), (float)(0.0 + (double)rad), (float)0.0);
        break;
    }
    case GI_EXP_RECTANGLE: {
        e.rec = blank_rec(K_EXP_RECTANGLE);
        const V3 p1 = v3(a[0], a[1], a[2]), p2 = v3(a[3], a[4], a[5]), p3 = v3(a[6], a[7], a[8]);
        if (dot(p1 - p3, p2 - p3) != 0.0) {   // the reference asserts a right angle at p3 (entities.h:312)
            err = "ExpRectangle: (p1-p3).(p2-p3) != 0";
            return false;
        }
        const V3 p4 = -p3;
        TriRec t;
        make_tri(p1, p2, p3, t);
        e.tris.push_back(t);
        make_tri(p1, p2, p4, t);
        e.tris.push_back(t);
        st3(e.rec.qv0, p1); st3(e.rec.qv1, p3); st3(e.rec.qv2, p4);
        st3(e.rec.pos, 0.5 * (p1 + p2));
        e.bmin = v3(smin(p1.x, p2.x), smin(p1.y, p2.y), smin(p1.z, p2.z));
        e.bmax = v3(smax(p1.x, p2.x), smax(p1.y, p2.y), smax(p1.z, p2.z));
        break;
    }
    case GI_EXP_BOX: {
        e.rec = blank_rec(K_EXP_BOX);
        const V3 mn = v3(a[0], a[1], a[2]), mx = v3(a[3], a[4], a[5]);
        const V3 dlb = mn, drb = v3(mx.x, mn.y, mn.z), dlt = v3(mn.x, mx.y, mn.z), drt = v3(mx.x, mx.y, mn.z);
        const V3 ulb = v3(mn.x, mn.y, mx.z), urb = v3(mx.x, mn.y, mx.z), ult = v3(mn.x, mx.y, mx.z), urt = mx;
        const V3 face[6][3] = {{dlb, urb, ulb}, {dlb, ult, dlt}, {dlb, drt, dlt},
                               {urt, ulb, ult}, {urt, drb, drt}, {urt, dlt, drt}};   // ExpBox::faces (:389-406)
        for (const auto& f : face) {
            TriRec t;
            make_tri(f[0], f[1], f[2], t);
            e.tris.push_back(t);
            make_tri(f[0], f[1], -f[2], t);
            e.tris.push_back(t);
        }
        e.bmin = mn;
        e.bmax = mx;
        break;
    }
    default:
        err = "unsupported entity kind " + std::to_string(d.kind);
        return false;
    }
    if (d.has_material) {
        set_color(e.rec, d.mat_color);
        e.rec.shader[0] = d.mat_shader[0]; e.rec.shader[1] = d.mat_shader[1]; e.rec.shader[2] = d.mat_shader[2];
        e.rec.spec_pow = d.mat_specular_power;
        if (!(d.mat_reflectivity >= 0.0 && d.mat_reflectivity <= 1.0)) {   // NaN fails too
            err = "mat_reflectivity must lie in [0, 1]";
            return false;
        }
        e.rec.refl = d.mat_reflectivity;
    }
    return true;
}

// ---- reference octree ------------------------------------------------------------------------
bool bb_overlap(V3 amin, V3 amax, V3 bmin, V3 bmax) {   // BoundingBox::intersect (bbox.h:25-39)
    const V3 p1 = 0.5 * (amin + amax), p2 = 0.5 * (bmin + bmax);
    const V3 d = p1 - p2;
    const bool xo = std::fabs(d.x) < (0.5 * (amax.x - amin.x) + 0.5 * (bmax.x - bmin.x));
    const bool yo = std::fabs(d.y) < (0.5 * (amax.y - amin.y) + 0.5 * (bmax.y - bmin.y));
    const bool zo = std::fabs(d.z) < (0.5 * (amax.z - amin.z) + 0.5 * (bmax.z - bmin.z));
    return xo && yo && zo;
}
bool le3(V3 a, V3 b) { return a.x <= b.x && a.y <= b.y && a.z <= b.z; }

struct RBuild {
    struct N {
        V3 mn, mx;
        std::vector<int32_t> ents;
        int32_t child0 = -1;
    };
    std::vector<N> nodes;
    const std::vector<BEnt>* ents;

    void partition(int ni) {   // octree.h:75-110
        if (nodes[ni].child0 >= 0) return;
        const V3 mn = nodes[ni].mn, mx = nodes[ni].mx;
        const V3 mid = (mn + mx) * 0.5;
        bool all_in = true;
        for (int32_t e : nodes[ni].ents) all_in = all_in && le3((*ents)[e].bmin, mid) && le3(mid, (*ents)[e].bmax);
        if (all_in) return;
        const V3 bx[8][2] = {
            {mn, mid},
            {v3(mn.x, mid.y, mn.z), v3(mid.x, mx.y, mid.z)},
            {v3(mid.x, mn.y, mn.z), v3(mx.x, mid.y, mid.z)},
            {v3(mid.x, mid.y, mn.z), v3(mx.x, mx.y, mid.z)},
            {mid, mx},
            {v3(mn.x, mid.y, mid.z), v3(mid.x, mx.y, mx.z)},
            {v3(mid.x, mn.y, mid.z), v3(mx.x, mid.y, mx.z)},
            {v3(mn.x, mn.y, mid.z), v3(mid.x, mid.y, mx.z)},
        };
        const int32_t c0 = (int32_t)nodes.size();
        for (int c = 0; c < 8; ++c) {
            N n;
            n.mn = bx[c][0];
            n.mx = bx[c][1];
            nodes.push_back(n);
        }
        nodes[ni].child0 = c0;
    }
    void push_obj(int ni, int32_t e) {   // octree.h:115-129
        nodes[ni].ents.push_back(e);
        partition(ni);
        if (nodes[ni].child0 < 0) return;
        const BEnt& E = (*ents)[e];
        for (int c = 0; c < 8; ++c) {
            const int ci = nodes[ni].child0 + c;
            if (le3(nodes[ci].mn, E.bmin) && le3(E.bmax, nodes[ci].mx)) push_obj(ci, e);
            else if (bb_overlap(nodes[ci].mn, nodes[ci].mx, E.bmin, E.bmax)) nodes[ci].ents.push_back(e);
        }
    }
};

// ---- Mode X octree (build-defined: tight cells, every overlapping leaf holds the primitive) ---
struct Box {
    double mn[3], mx[3];
};
const int XLEAF_MAX = 4;
const int XMAX_DEPTH = 12;

// Separating-axis triangle/box overlap (Akenine-Moller 2001): 3 box normals, the triangle plane
// and the 9 edge x axis products.  Conservative: callers pass a padded box.
bool tri_box_overlap(const double* c, const double* hs, const XPrim& p) {
    double v[3][3];
    for (int k = 0; k < 3; ++k) {
        v[0][k] = p.a[k] - c[k];
        v[1][k] = p.a[k] + p.b[k] - c[k];
        v[2][k] = p.a[k] + p.c[k] - c[k];
    }
    for (int k = 0; k < 3; ++k) {   // box normals
        const double mn = std::min(std::min(v[0][k], v[1][k]), v[2][k]);
        const double mx = std::max(std::max(v[0][k], v[1][k]), v[2][k]);
        if (mn > hs[k] || mx < -hs[k]) return false;
    }
    double e[3][3];
    for (int k = 0; k < 3; ++k) {
        e[0][k] = v[1][k] - v[0][k];
        e[1][k] = v[2][k] - v[1][k];
        e[2][k] = v[0][k] - v[2][k];
    }
    for (int i = 0; i < 3; ++i)        // edge i x box axis j
        for (int j = 0; j < 3; ++j) {
            double a[3] = {0, 0, 0};
            const int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            a[j1] = -e[i][j2];
            a[j2] = e[i][j1];
            const double p0 = a[0] * v[0][0] + a[1] * v[0][1] + a[2] * v[0][2];
            const double p1 = a[0] * v[1][0] + a[1] * v[1][1] + a[2] * v[1][2];
            const double p2 = a[0] * v[2][0] + a[1] * v[2][1] + a[2] * v[2][2];
            const double r = hs[0] * std::fabs(a[0]) + hs[1] * std::fabs(a[1]) + hs[2] * std::fabs(a[2]);
            const double mn = std::min(std::min(p0, p1), p2), mx = std::max(std::max(p0, p1), p2);
            if (mn > r * (1 + 1e-12) || mx < -r * (1 + 1e-12)) return false;
        }
    // triangle plane
    const double n[3] = {e[0][1] * e[1][2] - e[0][2] * e[1][1], e[0][2] * e[1][0] - e[0][0] * e[1][2],
                         e[0][0] * e[1][1] - e[0][1] * e[1][0]};
    const double d = n[0] * v[0][0] + n[1] * v[0][1] + n[2] * v[0][2];
    const double r = hs[0] * std::fabs(n[0]) + hs[1] * std::fabs(n[1]) + hs[2] * std::fabs(n[2]);
    return std::fabs(d) <= r * (1 + 1e-12);
}

bool prim_box_overlap(const XPrim& p, const double* mn, const double* mx) {
    double c[3], hs[3];
    for (int k = 0; k < 3; ++k) { c[k] = 0.5 * (mn[k] + mx[k]); hs[k] = 0.5 * (mx[k] - mn[k]); }
    if (p.kind == 0) return tri_box_overlap(c, hs, p);
    double d2 = 0;   // sphere: squared distance from the centre to the box
    for (int k = 0; k < 3; ++k) {
        const double q = std::max(mn[k] - p.a[k], std::max(0.0, p.a[k] - mx[k]));
        d2 += q * q;
    }
    return d2 <= p.b[0] * p.b[0] * (1 + 1e-12);
}

struct XBuild {
    const std::vector<Box>* pb;
    const std::vector<XPrim>* prims;
    std::vector<XNode>* out;
    std::vector<int32_t>* idx;
    double pad;
    int max_depth = 0;
    int leaf_max = XLEAF_MAX;

    static bool overlap(const Box& a, const Box& b) {
        for (int k = 0; k < 3; ++k)
            if (a.mx[k] < b.mn[k] || b.mx[k] < a.mn[k]) return false;
        return true;
    }
    Box tight(const Box& cell, const std::vector<int32_t>& prims) const {
        Box u;
        for (int k = 0; k < 3; ++k) { u.mn[k] = INFINITY; u.mx[k] = -INFINITY; }
        for (int32_t p : prims)
            for (int k = 0; k < 3; ++k) {
                u.mn[k] = std::min(u.mn[k], (*pb)[p].mn[k]);
                u.mx[k] = std::max(u.mx[k], (*pb)[p].mx[k]);
            }
        Box t;
        for (int k = 0; k < 3; ++k) {
            t.mn[k] = std::max(cell.mn[k], u.mn[k]) - pad;
            t.mx[k] = std::min(cell.mx[k], u.mx[k]) + pad;
        }
        return t;
    }
    // builds node `ni` (already allocated) for `cell` holding `prims`
    void build(int ni, const Box& cell, std::vector<int32_t>& prims, int depth) {
        max_depth = std::max(max_depth, depth);
        const Box tb = tight(cell, prims);
        XNode& n0 = (*out)[ni];
        for (int k = 0; k < 3; ++k) { n0.mn[k] = tb.mn[k]; n0.mx[k] = tb.mx[k]; }
        n0.child_base = -1; n0.child_mask = 0; n0.prim_off = 0; n0.prim_cnt = 0;
        std::vector<int32_t> kids[8];
        Box cb[8];
        bool split = (int)prims.size() > leaf_max && depth < XMAX_DEPTH;
        if (split) {
            double mid[3];
            for (int k = 0; k < 3; ++k) mid[k] = 0.5 * (cell.mn[k] + cell.mx[k]);
            bool progress = false;
            for (int c = 0; c < 8; ++c) {
                for (int k = 0; k < 3; ++k) {
                    const bool hi = (c >> k) & 1;
                    cb[c].mn[k] = hi ? mid[k] : cell.mn[k];
                    cb[c].mx[k] = hi ? cell.mx[k] : mid[k];
                }
                Box test = cb[c];
                for (int k = 0; k < 3; ++k) { test.mn[k] -= pad; test.mx[k] += pad; }
                for (int32_t p : prims)
                    if (overlap(test, (*pb)[p]) && prim_box_overlap((*this->prims)[p], test.mn, test.mx)) kids[c].push_back(p);
                if (!kids[c].empty() && kids[c].size() < prims.size()) progress = true;
            }
            split = progress;
        }
        if (!split) {
            XNode& n = (*out)[ni];
            n.prim_off = (int32_t)idx->size();
            n.prim_cnt = (int32_t)prims.size();
            idx->insert(idx->end(), prims.begin(), prims.end());
            return;
        }
        int mask = 0, cnt = 0;
        for (int c = 0; c < 8; ++c)
            if (!kids[c].empty()) { mask |= 1 << c; ++cnt; }
        const int base = (int)out->size();
        out->resize(out->size() + cnt);
        (*out)[ni].child_base = base;
        (*out)[ni].child_mask = mask;
        std::vector<int32_t>().swap(prims);   // release before recursing
        int k = 0;
        for (int c = 0; c < 8; ++c)
            if (!kids[c].empty()) build(base + k++, cb[c], kids[c], depth + 1);
    }
};

// Plane groups (Mode X; DESIGN.md §5 "own-plane leaves"): triangles that lie in one plane share a
// group id (XPrim::pad[0], 0..253; kXNoPlane otherwise), and a wide-node leaf child all of whose
// records are one group carries its id (byte c of XWNode::pad; kXNoPlane otherwise).  A ray leaving
// a surface point of group g can skip g's leaves outright: its origin lies on g's plane to within
// rounding, so the exact test of any triangle in that plane finds t within a few ulps of 0 -- below
// MX_TMIN -- unless the ray is nearly parallel to the plane.  The kernels skip only when
// |d . n| >= x_skip_a * max|cam| + x_skip_b, K = 2000 times the worst rounding:
//   * the origin P = o + t d of a hit on X is off X's plane by ~u (|o| + |P| + |o - v0| / s): the
//     rounding of P and of the exact test's t (whose error along the ray, ~u |o - v0| / (s |d . n|),
//     shrinks with the incidence), s the sine of the triangle's smallest angle;
//   * a triangle Y of the group lies within tau of X's plane (measured here), and its own test's t
//     error is ~u |P - v0_Y| / (s_Y |d . n|);
// so |t_Y| <= (u (|cam| + 4 E) / s_min + tau) / |d . n| up to small constants, and |d . n| >=
// K (u (|cam| + 4 E) / s_min + tau) / MX_TMIN keeps it below MX_TMIN / K.  Triangles with s < 1e-3
// join no group.  The CPU checker (tests/cpp/xaccel_check.cpp) runs the skip against brute force on
// rays from surface points, down to incidences just above the bound.
constexpr int kXNoPlane = 255;
void assign_plane_groups(HostScene& hs) {
    const size_t np = hs.xprims.size();
    hs.x_skip_a = 0.0;
    hs.x_skip_b = 2.0;   // > 1 >= |d . n|: no skip
    for (XPrim& p : hs.xprims) p.pad[0] = kXNoPlane;
    for (XWNode& w : hs.xwnodes) memset(w.pad, 0xFF, sizeof w.pad);
    double E = 0.0;
    for (const XPrim& p : hs.xprims)
        for (int k = 0; k < 3; ++k) {
            if (p.kind == 1) {
                E = std::max(E, std::fabs(p.a[k]) + std::fabs(p.b[0]));
            } else {
                E = std::max(E, std::fabs(p.a[k]));
                E = std::max(E, std::fabs(p.a[k] + p.b[k]));
                E = std::max(E, std::fabs(p.a[k] + p.c[k]));
            }
        }
    struct G {
        V3 n;
        double off;
    };
    std::vector<G> groups;
    double s_min = 1.0, tau = 0.0;
    const double tol = 1e-12 * std::max(E, 1.0);
    for (size_t i = 0; i < np; ++i) {
        XPrim& p = hs.xprims[i];
        if (p.kind != 0) continue;
        const V3 v0 = ld3(p.a), e1 = ld3(p.b), e2 = ld3(p.c), e3 = e2 - e1;
        const V3 cr = cross(e1, e2);
        const double area2 = std::sqrt(dot(cr, cr)), l1 = std::sqrt(dot(e1, e1)), l2 = std::sqrt(dot(e2, e2)),
                     l3 = std::sqrt(dot(e3, e3));
        if (!(area2 > 0.0) || !std::isfinite(area2)) continue;
        const double s = std::min(std::min(area2 / (l1 * l2), area2 / (l1 * l3)), area2 / (l2 * l3));
        if (!(s >= 1e-3)) continue;
        V3 n = cr * (1.0 / area2);
        if (n.x < 0 || (n.x == 0 && (n.y < 0 || (n.y == 0 && n.z < 0)))) n = -n;
        const V3 vs[3] = {v0, v0 + e1, v0 + e2};
        int g = -1;
        double dev = 0.0;
        for (size_t k = 0; k < groups.size() && g < 0; ++k) {
            const V3 dn = n - groups[k].n;
            if (std::max(std::fabs(dn.x), std::max(std::fabs(dn.y), std::fabs(dn.z))) > 1e-12) continue;
            double m = 0.0;
            for (const V3& v : vs) m = std::max(m, std::fabs(dot(groups[k].n, v) - groups[k].off));
            if (m <= tol) {
                g = (int)k;
                dev = m;
            }
        }
        if (g < 0) {
            if (groups.size() >= 254) continue;
            groups.push_back(G{n, dot(n, v0)});
            g = (int)groups.size() - 1;
            for (const V3& v : vs) dev = std::max(dev, std::fabs(dot(n, v) - groups[g].off));
        }
        p.pad[0] = g;
        tau = std::max(tau, dev);
        s_min = std::min(s_min, s);
    }
    if (groups.empty()) return;
    for (XWNode& w : hs.xwnodes) {
        uint8_t* b = reinterpret_cast<uint8_t*>(w.pad);
        for (int c = 0; c < 8; ++c) {
            if (w.child[c] >= 0 || w.child[c] == XEMPTY || w.cnt[c] == 0) continue;
            int g = hs.xprims[hs.xhot[~w.child[c]].prim].pad[0];
            for (int j = 1; j < w.cnt[c] && g != kXNoPlane; ++j)
                if (hs.xprims[hs.xhot[~w.child[c] + j].prim].pad[0] != g) g = kXNoPlane;
            b[c] = (uint8_t)g;
        }
    }
    const double K = 2000.0, u = 0x1.0p-53, tmin = 1e-7;
    hs.x_skip_a = K * u / (s_min * tmin);
    hs.x_skip_b = K * (4.0 * u * E / s_min + tau + 4.0 * u * E) / tmin;
}

}  // namespace

bool build_host_scene(const gi_scene_desc& desc, HostScene& hs, std::string& err) {
    std::vector<BEnt> ents((size_t)desc.n_entities);
    for (int i = 0; i < desc.n_entities; ++i)
        if (!build_entity(desc.entities[i], ents[i], err)) return false;

    // entity + triangle records
    hs.ents.clear();
    hs.tris.clear();
    for (BEnt& e : ents) {
        e.rec.tri_first = (int32_t)hs.tris.size();
        e.rec.tri_count = (int32_t)e.tris.size();
        hs.tris.insert(hs.tris.end(), e.tris.begin(), e.tris.end());
        hs.ents.push_back(e.rec);
    }

    // reference octree
    RBuild rb;
    rb.ents = &ents;
    RBuild::N root;
    root.mn = v3(desc.octree_min[0], desc.octree_min[1], desc.octree_min[2]);
    root.mx = v3(desc.octree_max[0], desc.octree_max[1], desc.octree_max[2]);
    rb.nodes.push_back(root);
    hs.n_dropped = 0;
    for (int32_t i = 0; i < desc.n_entities; ++i) {
        if (!bb_overlap(rb.nodes[0].mn, rb.nodes[0].mx, ents[i].bmin, ents[i].bmax)) { ++hs.n_dropped; continue; }   // octree.h:22-24
        rb.push_obj(0, i);
    }
    const size_t nn = rb.nodes.size();
    hs.rnodes.assign(nn, RNode());
    hs.leaf_ents.clear();
    std::vector<int32_t> depth(nn, 0);
    std::vector<char> reach((size_t)desc.n_entities, 0);
    hs.n_leaves = 0;
    hs.max_depth = 0;
    for (size_t i = 0; i < nn; ++i) {
        const RBuild::N& s = rb.nodes[i];
        RNode& d = hs.rnodes[i];
        st3(d.mn, s.mn);
        st3(d.mx, s.mx);
        d.child0 = s.child0;
        if (i == 0) d.parent = -1;
        d.ent_cnt = (int32_t)s.ents.size();
        d.ent_off = -1;
        if (s.child0 < 0) {
            d.ent_off = (int32_t)hs.leaf_ents.size();
            hs.leaf_ents.insert(hs.leaf_ents.end(), s.ents.begin(), s.ents.end());
            for (int32_t e : s.ents) reach[e] = 1;
            ++hs.n_leaves;
        } else {
            for (int c = 0; c < 8; ++c) {
                hs.rnodes[s.child0 + c].parent = (int32_t)i;
                depth[s.child0 + c] = depth[i] + 1;
            }
        }
        hs.max_depth = std::max(hs.max_depth, depth[i]);
    }
    hs.n_reachable = 0;
    for (char r : reach) hs.n_reachable += r;
    build_rcand(hs);   // Mode R candidate reconstruction (gi_bvh.cpp)

    // Mode X primitives (every entity, in push order; ExpQuad contributes its 2 triangles)
    hs.xprims.clear();
    std::vector<Box> pb;
    for (int32_t i = 0; i < desc.n_entities; ++i) {
        const REnt& r = hs.ents[i];
        if (r.kind == K_IMP_SPHERE) {
            XPrim p;
            memset(&p, 0, sizeof p);
            p.kind = 1; p.ent = i;
            p.a[0] = r.pos[0]; p.a[1] = r.pos[1]; p.a[2] = r.pos[2];
            p.b[0] = (double)r.radius;
            hs.xprims.push_back(p);
            Box b;
            for (int k = 0; k < 3; ++k) { b.mn[k] = r.pos[k] - (double)r.radius; b.mx[k] = r.pos[k] + (double)r.radius; }
            pb.push_back(b);
        } else {
            for (int t = 0; t < r.tri_count; ++t) {
                const TriRec& tr = hs.tris[r.tri_first + t];
                XPrim p;
                memset(&p, 0, sizeof p);
                p.kind = 0; p.ent = i;
                const V3 p1 = ld3(tr.p1), e1 = ld3(tr.p2) - p1, e2 = ld3(tr.p3) - p1;
                st3(p.a, p1); st3(p.b, e1); st3(p.c, e2);
                for (int k = 0; k < 3; ++k) p.n[k] = tr.n[k];
                hs.xprims.push_back(p);
                Box b;
                for (int k = 0; k < 3; ++k) {
                    b.mn[k] = std::min(std::min(tr.p1[k], tr.p2[k]), tr.p3[k]);
                    b.mx[k] = std::max(std::max(tr.p1[k], tr.p2[k]), tr.p3[k]);
                }
                pb.push_back(b);
            }
        }
    }
    hs.xnodes.clear();
    hs.xprim_idx.clear();
    // GI_XACCEL=octree (a test hook: the frame does not depend on the acceleration structure) builds
    // the round-1 SAT octree instead of the SAH BVH; GI_XLEAF_MAX (test hook) caps leaf sizes
    const char* accel = std::getenv("GI_XACCEL");
    if (!(accel && std::string(accel) == "octree")) {
        std::vector<double> bounds(6 * pb.size());
        for (size_t i = 0; i < pb.size(); ++i)
            for (int k = 0; k < 3; ++k) { bounds[6 * i + k] = pb[i].mn[k]; bounds[6 * i + 3 + k] = pb[i].mx[k]; }
        int leaf_max = 4;
        if (const char* lm = std::getenv("GI_XLEAF_MAX")) leaf_max = std::max(1, std::atoi(lm));
        build_xbvh(hs.xprims, bounds, leaf_max, hs, true);
        assign_plane_groups(hs);
        return true;
    }
    hs.xnodes.resize(1);
    Box rootb;
    for (int k = 0; k < 3; ++k) { rootb.mn[k] = INFINITY; rootb.mx[k] = -INFINITY; }
    for (const Box& b : pb)
        for (int k = 0; k < 3; ++k) { rootb.mn[k] = std::min(rootb.mn[k], b.mn[k]); rootb.mx[k] = std::max(rootb.mx[k], b.mx[k]); }
    if (pb.empty()) {
        for (int k = 0; k < 3; ++k) { rootb.mn[k] = 0; rootb.mx[k] = 0; }
    }
    double ext = 1.0;
    for (int k = 0; k < 3; ++k) ext = std::max(ext, std::max(std::fabs(rootb.mn[k]), std::fabs(rootb.mx[k])));
    XBuild xb;
    xb.pb = &pb;
    xb.prims = &hs.xprims;
    xb.out = &hs.xnodes;
    xb.idx = &hs.xprim_idx;
    xb.pad = 1e-9 * ext;
    if (const char* lm = std::getenv("GI_XLEAF_MAX")) xb.leaf_max = std::max(1, std::atoi(lm));
    std::vector<int32_t> all(pb.size());
    for (size_t i = 0; i < pb.size(); ++i) all[i] = (int32_t)i;
    if (pb.empty()) {
        XNode& n = hs.xnodes[0];
        memset(&n, 0, sizeof n);
        n.mn[0] = n.mn[1] = n.mn[2] = 1.0;   // empty box: no ray enters
        n.mx[0] = n.mx[1] = n.mx[2] = -1.0;
        n.child_base = -1;
    } else {
        xb.build(0, rootb, all, 0);
    }
    hs.x_max_depth = xb.max_depth;

    // wide traversal nodes: one XWNode per interior cell holding its children's boxes in fp32
    double pad32 = 1e-5 * ext;
    auto lo32 = [&](double v) {
        float f = (float)(v - pad32);
        if ((double)f > v - pad32) f = std::nextafter(f, -INFINITY);
        return f;
    };
    auto hi32 = [&](double v) {
        float f = (float)(v + pad32);
        if ((double)f < v + pad32) f = std::nextafter(f, INFINITY);
        return f;
    };
    const size_t nx = hs.xnodes.size();
    std::vector<int32_t> ref(nx, 0);
    int32_t nwide = 0, nleaf = 0;
    for (size_t i = 0; i < nx; ++i) {
        if (hs.xnodes[i].child_mask != 0) ref[i] = nwide++;
        else ref[i] = ~(nleaf++);
    }
    hs.xleaves.assign((size_t)nleaf, XLeaf{0, 0});
    hs.xhot.clear();
    hs.xbox.clear();
    for (size_t i = 0; i < nx; ++i)
        if (hs.xnodes[i].child_mask == 0) {
            const XNode& n = hs.xnodes[i];
            hs.xleaves[~ref[i]] = XLeaf{(int32_t)hs.xhot.size(), n.prim_cnt};   // range in xhot
            for (int k = 0; k < n.prim_cnt; ++k) {
                const int32_t pi = hs.xprim_idx[n.prim_off + k];
                const XPrim& p = hs.xprims[pi];
                XHot h;
                memcpy(h.a, p.a, sizeof h.a);
                memcpy(h.b, p.b, sizeof h.b);
                memcpy(h.c, p.c, sizeof h.c);
                h.prim = pi;
                h.kind = p.kind;
                hs.xhot.push_back(h);
                XBox bx;
                for (int a = 0; a < 3; ++a) { bx.lo[a] = lo32(pb[pi].mn[a]); bx.hi[a] = hi32(pb[pi].mx[a]); }
                bx.pad[0] = pi;
                bx.pad[1] = p.kind;
                hs.xbox.push_back(bx);
            }
        }
    const bool root_leaf = hs.xnodes[0].child_mask == 0;
    hs.xwnodes.assign(root_leaf ? 1 : (size_t)nwide, XWNode());
    auto empty_slot = [](XWNode& w, int c) {
        for (int k = 0; k < 3; ++k) { w.lo[k][c] = INFINITY; w.hi[k][c] = -INFINITY; }
        w.child[c] = XEMPTY;
    };
    for (XWNode& w : hs.xwnodes) {
        for (int c = 0; c < 8; ++c) empty_slot(w, c);
        w.parent = -1;
        for (int c = 0; c < 8; ++c) w.cnt[c] = 0;
        w.exists = 0;
        w.pad[0] = w.pad[1] = 0;
    }
    auto fill_slot = [&](XWNode& w, int c, const XNode& n, int32_t r) {
        for (int k = 0; k < 3; ++k) { w.lo[k][c] = lo32(n.mn[k]); w.hi[k][c] = hi32(n.mx[k]); }
        if (r >= 0) {
            w.child[c] = r;
        } else {   // leaf: offset of its records in xhot + count
            const XLeaf& lf = hs.xleaves[~r];
            w.child[c] = ~lf.off;
            w.cnt[c] = (uint16_t)std::min(lf.cnt, 65535);
        }
    };
    if (root_leaf) {
        fill_slot(hs.xwnodes[0], 0, hs.xnodes[0], ref[0]);
    } else {
        for (size_t i = 0; i < nx; ++i) {
            const XNode& n = hs.xnodes[i];
            if (n.child_mask == 0) continue;
            XWNode& w = hs.xwnodes[ref[i]];
            int rank = 0;
            for (int c = 0; c < 8; ++c)
                if ((n.child_mask >> c) & 1) {
                    const int ci = n.child_base + rank++;
                    fill_slot(w, c, hs.xnodes[ci], ref[ci]);
                    if (ref[ci] >= 0) hs.xwnodes[ref[ci]].parent = ref[i];
                }
        }
    }
    finalize_xwnodes(hs.xwnodes);
    assign_plane_groups(hs);
    return true;
}

}  // namespace gi
