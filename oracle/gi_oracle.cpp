// gi_oracle.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference per-pixel radiance
// loop (preon7/2019global) and of the build-defined Mode X integrator.  Own code; it
// restates glm 0.9.8.2's operation order explicitly instead of including glm.  Compiled with
// -ffp-contract=off (no FMA contraction) so every fp op rounds exactly as the reference's does.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library.
#include "gi_oracle.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

thread_local std::string g_err;

// ---------------------------------------------------------------------------------------------
// glm 0.9.8.2 arithmetic, restated (3rd_party/glm/detail/func_geometric.inl:54-96,
// func_exponential.inl:128-133, type_vec3.inl operators): dot = (x*x'+y*y')+z*z';
// cross = (y*z'-y'*z, z*x'-z'*x, x*y'-x'*y); normalize(v) = v * (1/sqrt(dot(v,v))).
// ---------------------------------------------------------------------------------------------
struct V3 { double x, y, z; };
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 x, V3 y) { return {x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
inline V3 normalize(V3 v) { return v * (1.0 / std::sqrt(dot(v, v))); }
inline double length(V3 v) { return std::sqrt(dot(v, v)); }
// pow(a.x,2)+pow(a.y,2)+pow(a.z,2): g++ folds pow(x,2) to x*x (identical at -O0)
inline double sq3(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
inline double smin(double a, double b) { return (b < a) ? b : a; }   // std::min
inline double smax(double a, double b) { return (a < b) ? b : a; }   // std::max
inline float sminf(float a, float b) { return (b < a) ? b : a; }

// x86-64 cvttsd2si: NaN / out-of-range -> INT_MIN; the reference's int() casts.
inline int32_t x86_trunc(double d) {
    if (!(d > -2147483649.0 && d < 2147483648.0)) return INT32_MIN;
    return (int32_t)d;
}

const double REF_PI = 3.1415926535;   // entities.h:16

struct Mat {
    V3 color{1, 0, 0};
    V3 shader{0.1, 0.7, 1.0};   // material.h:27
    double spec_pow = 5.0;      // material.h:29
    double refl = 0.0;          // Mode X only: mirror-reflection probability (no reference counterpart)
};

// ImpTriangle (entities.h:136-306): members initialised in declaration order.
struct Tri {
    V3 p1, p2, p3, e1, e2, n, pos;
    float e1f[3], e2f[3];
};
Tri make_tri(V3 p1, V3 p2, V3 p3) {
    Tri t;
    t.p1 = p1; t.p2 = p2; t.p3 = p3;
    t.e1 = p2 - p1;                  // :146
    t.e2 = p3 - p1;                  // :147
    t.n = normalize(cross(t.e1, t.e2));   // :148
    t.pos = 0.5 * (0.5 * (p1 + p2) + p3); // :139
    t.e1f[0] = (float)t.e1.x; t.e1f[1] = (float)t.e1.y; t.e1f[2] = (float)t.e1.z;
    t.e2f[0] = (float)t.e2.x; t.e2f[1] = (float)t.e2.y; t.e2f[2] = (float)t.e2.z;
    return t;
}

// ImpTriangle::intersect (entities.h:150-249).  The 3x3 solve runs in fp32: glm::mat3 of the
// dvec3 columns (type_mat3x3.inl:99-109, float casts), transpose, glm's cofactor inverse
// (func_matrix.inl:272-294), then vec3(right) * A_i (type_mat3x3.inl:437-443).  Only sol.z is used.
bool tri_intersect(const Tri& t, V3 o, V3 d, V3& P, V3& N) {
    if (dot(t.n, d) == 0) return false;   // :151
    // m = transpose(mat3(e1, e2, -dir)): m[c][r]
    const float m00 = t.e1f[0], m01 = t.e2f[0], m02 = (float)(-d.x);
    const float m10 = t.e1f[1], m11 = t.e2f[1], m12 = (float)(-d.y);
    const float m20 = t.e1f[2], m21 = t.e2f[2], m22 = (float)(-d.z);
    const float det = m00 * (m11 * m22 - m21 * m12) - m10 * (m01 * m22 - m21 * m02) + m20 * (m01 * m12 - m11 * m02);
    const float ood = 1.0f / det;
    const float i20 = (m10 * m21 - m20 * m11) * ood;
    const float i21 = (-(m00 * m21 - m20 * m01)) * ood;
    const float i22 = (m00 * m11 - m10 * m01) * ood;
    const V3 right = o - t.pos;   // :156
    const float vx = (float)right.x, vy = (float)right.y, vz = (float)right.z;
    const float solz = i20 * vx + i21 * vy + i22 * vz;
    const V3 point = o + (double)solz * d;   // :166
    const V3 d1 = normalize(cross(t.p1 - point, t.p2 - point));
    const V3 d2 = normalize(cross(t.p2 - point, t.p3 - point));
    const V3 d3 = normalize(cross(t.p3 - point, t.p1 - point));
    const double eps = 1.0e-3;
    const V3 nn = dot(d, t.n) < 0 ? t.n : -t.n;
    if (length(d1) < eps || length(d2) < eps || length(d3) < eps) {   // :201-230 (dead for finite input)
        P = point; N = nn; return true;
    }
    const V3 f1 = d1 - d2, f2 = d2 - d3;
    const bool cp1 = sq3(f1) < eps, cp2 = sq3(f2) < eps;   // :232-235
    if (cp1 && cp2) { P = point; N = nn; return true; }
    return false;
}

// ImpSphere::intersect (entities.h:53-96): fp32/fp64 mix exactly as written.
bool sphere_intersect(V3 pos, float radius, V3 o, V3 d, V3& P, V3& N) {
    const V3 np = pos - o;
    float a1 = 1, a2 = 1, a3 = 1;
    if (d.x != 0) { a2 = (float)(d.y / d.x); a3 = (float)(d.z / d.x); }
    else if (d.y != 0) { a1 = (float)(d.x / d.y); a3 = (float)(d.z / d.y); }
    else if (d.z != 0) { a2 = (float)(d.y / d.z); a1 = (float)(d.x / d.z); }
    else return false;
    const double A1 = a1, A2 = a2, A3 = a3;
    const float a = (float)(A1 * A1 + A2 * A2 + A3 * A3);
    const float b = (float)(-2.0 * (np.x * A1 + np.y * A2 + np.z * A3));
    const double R = radius;
    const float c = (float)(np.x * np.x + np.y * np.y + np.z * np.z - R * R);
    const double B = b;
    const float ac4 = (4.0f * a) * c;
    const double disc = B * B - (double)ac4;
    if (disc < 0) return false;
    const double s = std::sqrt(disc);
    const float a2f = 2.0f * a;
    const float v1 = (float)((-(double)b + s) / (double)a2f);   // -b is exact in float
    const float v2 = (float)((-(double)b - s) / (double)a2f);
    const float base = sminf(std::fabs(v1), std::fabs(v2));
    V3 ip{(double)(base * a1), (double)(base * a2), (double)(base * a3)};
    ip = ip + o;
    P = ip;
    N = normalize(ip - pos);
    return true;
}

enum Kind { IMP_SPHERE = 1, IMP_TRIANGLE = 2, EXP_QUAD = 3, EXP_SPHERE = 4, EXP_CUBE = 5, EXP_CONE = 6,
            EXP_RECTANGLE = 7, EXP_BOX = 8 };

struct Ent {
    int kind = 0;
    Mat mat;
    V3 pos{0, 0, 0};
    float radius = 0, width = 0, length_ = 0, alpha = 0;
    Tri tri;
    std::vector<Tri> tris;   // group triangles (ExpQuad/Sphere/Cube/Cone; Rectangle t1,t2; Box 6x(t1,t2))
    V3 qv[4];                // ExpQuad vertices; ExpCube vertices[0]; ExpRectangle p1, p3, p4
    float height = 0;        // ExpCube / ExpCone
    double cone_theta = 0;   // ExpCone: atan(radius/height) evaluated in float (entities.h:950)
    V3 bmin, bmax;           // boundingBox() as the reference reports it (A.5, A.13)
};

// ---- constructors ----------------------------------------------------------------------------
Ent make_imp_sphere(V3 pos, double radius_arg, V3 color) {
    Ent e;
    e.kind = IMP_SPHERE;
    e.mat.color = color;
    e.radius = (float)radius_arg;
    e.pos = pos;
    // bbox member initialised while pos is still {0,0,0} (entities.h:98-99, A.5); glm::vec3
    const double r = e.radius;
    e.bmin = {(double)(float)(0.0 - r), (double)(float)(0.0 - r), (double)(float)(0.0 - r)};
    e.bmax = {(double)(float)(0.0 + r), (double)(float)(0.0 + r), (double)(float)(0.0 + r)};
    return e;
}

void tri_bbox(const Tri& t, V3& mn, V3& mx) {   // entities.h:251-275 (A.13)
    mn = {smin(smin(t.p1.x, t.p2.x), t.p3.x), smin(smin(t.p1.y, t.p2.y), t.p3.y), smin(smin(t.p1.z, t.p2.z), t.p3.z)};
    mx = {smax(smax(t.p1.x, t.p2.x), t.p3.x), smax(smax(t.p1.y, t.p2.y), t.p3.y), smax(smax(t.p1.z, t.p2.z), t.p3.z) + 0.01};
    if (mx.x == mn.x) mx.x += 1e-5;
    if (mx.y == mn.y) mx.y += 1e-5;
    if (mx.z == mn.z) mx.z += 1e-5;
}

Ent make_imp_triangle(V3 p1, V3 p2, V3 p3) {
    Ent e;
    e.kind = IMP_TRIANGLE;   // Entity() default material: red (entities.h:21)
    e.tri = make_tri(p1, p2, p3);
    e.pos = e.tri.pos;
    tri_bbox(e.tri, e.bmin, e.bmax);
    return e;
}

Ent make_exp_quad(V3 pos, double w_arg, double l_arg, double a_arg, V3 color) {   // entities.h:581-590
    Ent e;
    e.kind = EXP_QUAD;
    e.mat.color = color;
    e.width = (float)w_arg; e.length_ = (float)l_arg; e.alpha = (float)a_arg;
    e.pos = pos;
    const float hw = e.width / 2, hl = e.length_ / 2;
    const double ca = (double)std::cos(e.alpha), sa = (double)std::sin(e.alpha);   // float overloads
    e.qv[0] = {(pos.x + hw) * ca, pos.y + hl, pos.z + (pos.x + hw) * sa};
    e.qv[1] = {(pos.x - hw) * ca, pos.y + hl, pos.z + (pos.x - hw) * sa};
    e.qv[2] = {(pos.x + hw) * ca, pos.y - hl, pos.z + (pos.x + hw) * sa};
    e.qv[3] = {(pos.x - hw) * ca, pos.y - hl, pos.z + pos.z + (pos.x - hw) * sa};   // :586 typo
    e.tris.push_back(make_tri(e.qv[1], e.qv[2], e.qv[0]));
    e.tris.push_back(make_tri(e.qv[1], e.qv[3], e.qv[2]));
    // bbox with pos = {0,0,0} (entities.h:623-624, A.5), through glm::vec3
    e.bmin = {(double)(float)(0.0 - hw), (double)(float)(0.0 - hl), (double)(float)0.0};
    e.bmax = {(double)(float)(0.0 + hw), (double)(float)(0.0 + hl), (double)(float)(0.0 + (0.0 + hw) * sa)};
    return e;
}

// glm::mat3 (float) * dvec3: the vector is narrowed to vec3, product in fp32 (type_mat3x3.inl:429-435)
struct M3f { float c[3][3]; };   // c[col][row]
V3 m3_mul(const M3f& m, V3 v) {
    const float x = (float)v.x, y = (float)v.y, z = (float)v.z;
    return {(double)(m.c[0][0] * x + m.c[1][0] * y + m.c[2][0] * z), (double)(m.c[0][1] * x + m.c[1][1] * y + m.c[2][1] * z),
            (double)(m.c[0][2] * x + m.c[1][2] * y + m.c[2][2] * z)};
}

Ent make_exp_sphere(V3 pos, double radius_arg, V3 color) {   // entities.h:461-506
    Ent e;
    e.kind = EXP_SPHERE;
    e.mat.color = color;
    e.radius = (float)radius_arg;
    e.pos = pos;
    const int sectornum = 10, stacknum = 10;
    const float sectorStep = (float)(2 * REF_PI / sectornum);
    const float stackStep = (float)(REF_PI / stacknum);
    std::vector<V3> vert;
    for (int i = 0; i <= stacknum; ++i) {
        const float stackAngle = (float)(REF_PI / 2 - (double)(i * stackStep));
        const float tmp = e.radius * cosf(stackAngle);
        const float z = (float)((double)(e.radius * sinf(stackAngle)) - pos.z);   // vertices offset by -pos
        for (int j = 0; j <= sectornum; ++j) {
            const float sectorAngle = j * sectorStep;
            const float x = (float)((double)(tmp * cosf(sectorAngle)) - pos.x);
            const float y = (float)((double)(tmp * sinf(sectorAngle)) - pos.y);
            vert.push_back({(double)x, (double)y, (double)z});
        }
    }
    std::vector<Tri> all;
    for (int i = 0; i < stacknum; ++i) {
        int k1 = i * (sectornum + 1), k2 = k1 + sectornum + 1;
        for (int j = 0; j < sectornum; ++j, ++k1, ++k2) {
            if (i != 0) all.push_back(make_tri(vert[k1], vert[k2], vert[k1 + 1]));
            if (i != stacknum - 1) all.push_back(make_tri(vert[k1 + 1], vert[k2], vert[k2 + 1]));
        }
    }
    e.tris.assign(all.begin() + 1, all.end());   // intersect() starts at triangle 1 (entities.h:520)
    const double r = e.radius;
    e.bmin = {(double)(float)(0.0 - r), (double)(float)(0.0 - r), (double)(float)(0.0 - r)};
    e.bmax = {(double)(float)(0.0 + r), (double)(float)(0.0 + r), (double)(float)(0.0 + r)};
    return e;
}

Ent make_exp_cube(V3 pos, double w_arg, double l_arg, double h_arg, V3 color) {   // entities.h:652-727
    Ent e;
    e.kind = EXP_CUBE;
    e.mat.color = color;
    e.width = (float)w_arg; e.length_ = (float)l_arg; e.height = (float)h_arg;
    e.pos = pos;
    const float hw = e.width / 2, hl = e.length_ / 2, hh = e.height / 2;
    const V3 v[8] = {{pos.x - hw, pos.y - hl, pos.z - hh}, {pos.x - hw, pos.y - hl, pos.z + hh},
                     {pos.x + hw, pos.y - hl, pos.z - hh}, {pos.x + hw, pos.y - hl, pos.z + hh},
                     {pos.x - hw, pos.y + hl, pos.z + hh}, {pos.x - hw, pos.y + hl, pos.z - hh},
                     {pos.x + hw, pos.y + hl, pos.z - hh}, {pos.x + hw, pos.y + hl, pos.z + hh}};
    const int T[12][3] = {{0, 1, 2}, {3, 1, 2}, {4, 5, 7}, {7, 5, 6}, {1, 0, 4}, {4, 0, 5},
                          {3, 7, 2}, {7, 6, 2}, {1, 4, 3}, {3, 4, 7}, {0, 5, 2}, {2, 5, 6}};
    for (auto& t : T) e.tris.push_back(make_tri(v[t[0]], v[t[1]], v[t[2]]));
    e.qv[0] = v[0];
    e.bmin = {(double)(float)(0.0 - hw), (double)(float)(0.0 - hl), (double)(float)(0.0 - hh)};
    e.bmax = {(double)(float)(0.0 + hw), (double)(float)(0.0 + hl), (double)(float)(0.0 + hh)};
    return e;
}

Ent make_exp_cone(V3 pos, V3 dir_arg, double h_arg, double r_arg, V3 color) {   // entities.h:823-899
    Ent e;
    e.kind = EXP_CONE;
    e.mat.color = color;
    e.height = (float)h_arg;
    e.radius = (float)r_arg;
    e.pos = pos;
    const V3 dir = normalize(V3{-1, 0, -10});   // assigns the shadowing ctor parameter (:825)
    M3f I = {{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}}, rx = I, ry = I;
    const double x_sign = dir.y < 0 ? 1.0 : -1.0;
    const V3 x_dir{0, dir.y, dir.z};
    if (!(x_dir.x == 0 && x_dir.y == 0 && x_dir.z == 0)) {
        const double a = x_sign * std::acos(dot(normalize(x_dir), V3{0, 0, -1}));
        rx = {{{1, 0, 0}, {0, (float)std::cos(a), (float)(-std::sin(a))}, {0, (float)std::sin(a), (float)std::cos(a)}}};
    }
    const double y_sign = dir.x > 0 ? 1.0 : -1.0;
    const V3 y_dir{dir.x, 0, -std::sqrt(dir.z * dir.z + dir.y * dir.y)};
    if (!(y_dir.x == 0 && y_dir.y == 0 && y_dir.z == 0)) {
        const double a = y_sign * std::acos(dot(normalize(y_dir), V3{0, 0, -1}));
        ry = {{{(float)std::cos(a), 0, (float)std::sin(a)}, {0, 1, 0}, {(float)(-std::sin(a)), 0, (float)std::cos(a)}}};
    }
    std::vector<V3> vert{pos};
    const double nsub = 50.0;
    for (int i = 0; i <= nsub; ++i) {
        const float alpha = (float)(i * 360.0 / nsub);
        V3 loc{pos.x + (double)e.radius * std::cos((double)alpha * REF_PI / 180.0),
               pos.y + (double)e.radius * std::sin((double)alpha * REF_PI / 180.0), pos.z - (double)e.height};
        loc = loc - pos;
        loc = m3_mul(rx, loc);
        loc = m3_mul(ry, loc);
        loc = loc + pos;
        vert.push_back(loc);
    }
    const V3 bottom = pos + normalize(dir) * (double)e.height;
    for (size_t i = 1; i < vert.size() - 1; ++i) {
        e.tris.push_back(make_tri(pos, vert[i], vert[i + 1]));
        e.tris.push_back(make_tri(bottom, vert[i], vert[i + 1]));
    }
    e.cone_theta = (double)std::atan(e.radius / e.height);   // float atan (:950)
    (void)dir_arg;   // the member dir keeps the argument but nothing reads it
    e.bmin = {(double)(float)(0.0 - (double)e.radius), (double)(float)(0.0 - (double)e.radius), (double)(float)(0.0 - (double)e.height)};
    e.bmax = {(double)(float)(0.0 + (double)e.radius), (double)(float)(0.0 + (double)e.radius), (double)(float)0.0};
    return e;
}

Ent make_exp_rectangle(V3 p1, V3 p2, V3 p3) {   // entities.h:310-340 (p4 = -p3, A.4)
    Ent e;
    e.kind = EXP_RECTANGLE;   // Entity(): red
    const V3 p4 = -p3;
    e.tris.push_back(make_tri(p1, p2, p3));
    e.tris.push_back(make_tri(p1, p2, p4));
    e.qv[0] = p1; e.qv[1] = p3; e.qv[2] = p4;
    e.pos = 0.5 * (p1 + p2);
    e.bmin = {smin(p1.x, p2.x), smin(p1.y, p2.y), smin(p1.z, p2.z)};
    e.bmax = {smax(p1.x, p2.x), smax(p1.y, p2.y), smax(p1.z, p2.z)};
    return e;
}

void box_faces(V3 mn, V3 mx, V3 F[6][3]) {   // ExpBox::faces (entities.h:389-406)
    const V3 dlb = mn, drb{mx.x, mn.y, mn.z}, dlt{mn.x, mx.y, mn.z}, drt{mx.x, mx.y, mn.z};
    const V3 ulb{mn.x, mn.y, mx.z}, urb{mx.x, mn.y, mx.z}, ult{mn.x, mx.y, mx.z}, urt = mx;
    const V3 G[6][3] = {{dlb, urb, ulb}, {dlb, ult, dlt}, {dlb, drt, dlt}, {urt, ulb, ult}, {urt, drb, drt}, {urt, dlt, drt}};
    for (int f = 0; f < 6; ++f) for (int k = 0; k < 3; ++k) F[f][k] = G[f][k];
}

Ent make_exp_box(V3 mn, V3 mx) {   // entities.h:381-446
    Ent e;
    e.kind = EXP_BOX;
    V3 F[6][3];
    box_faces(mn, mx, F);
    for (int f = 0; f < 6; ++f) {
        e.tris.push_back(make_tri(F[f][0], F[f][1], F[f][2]));
        e.tris.push_back(make_tri(F[f][0], F[f][1], -F[f][2]));
    }
    e.bmin = mn;
    e.bmax = mx;
    return e;
}

// Entity::intersect dispatch (Mode R)
bool ent_intersect(const Ent& e, V3 o, V3 d, V3& P, V3& N) {
    switch (e.kind) {
    case IMP_SPHERE: return sphere_intersect(e.pos, e.radius, o, d, P, N);
    case IMP_TRIANGLE: return tri_intersect(e.tri, o, d, P, N);
    case EXP_RECTANGLE: {   // entities.h:326-336: t1, else t2
        if (tri_intersect(e.tris[0], o, d, P, N)) return true;
        return tri_intersect(e.tris[1], o, d, P, N);
    }
    case EXP_BOX: {   // entities.h:415-440: every face tested; the LAST hitting face's point wins
        bool any = false;
        for (int f = 0; f < 6; ++f) {
            V3 p, n;
            bool h = tri_intersect(e.tris[2 * f], o, d, p, n);
            if (!h) h = tri_intersect(e.tris[2 * f + 1], o, d, p, n);
            if (h) {
                if (sq3(p - o) < DBL_MAX) { P = p; N = n; }
                any = true;
            }
        }
        return any;
    }
    case EXP_QUAD: case EXP_SPHERE: case EXP_CUBE: case EXP_CONE: {
        // entities.h:596-620 / 514-536 / 736-760 / 906-930: nearest by <= (ties -> later);
        // the outputs are overwritten even on a miss (:616-617)
        bool flag = false;
        double md = DBL_MAX;
        V3 mi{DBL_MAX, DBL_MAX, DBL_MAX}, cn{0, 0, 0};
        for (const Tri& t : e.tris) {
            V3 p, n;
            if (tri_intersect(t, o, d, p, n)) {
                const double dd = sq3(p - o);
                if (dd <= md) { mi = p; cn = n; md = dd; }
                flag = true;
            }
        }
        P = mi; N = cn;
        return flag;
    }
    }
    return false;
}

// ---- texture coordinates (entities.h:108-130, 277-303, 630-641) --------------------------
void tex_imp_sphere(const Ent& e, V3 ip, int32_t& x, int32_t& y) {
    const double r = e.radius;
    const double unit_v = 2.0 * REF_PI * r / 320.0;
    const V3 to = ip - e.pos;
    const V3 up{0, 0, r};
    const double cos_vert = dot(to, up) / (r * r);
    const double ang = std::acos(cos_vert);
    y = x86_trunc((r * ang) / unit_v);
    const double small_r = r * std::sin(ang);
    const V3 lm{0, small_r, 0};
    const double cos_hori = dot(V3{to.x, to.y, 0}, lm) / (small_r * small_r);
    const double unit_h = 2.0 * REF_PI * small_r / 320.0;
    x = x86_trunc(small_r * std::acos(cos_hori) / unit_h);
}

void tex_imp_triangle(const Tri& t, V3 ip, int32_t& x, int32_t& y) {
    const V3 p21 = t.p2 - t.p1, p31 = t.p3 - t.p1, p32 = t.p3 - t.p2, i1 = ip - t.p1;
    const double p21l = std::sqrt(sq3(p21));
    const double i1l = std::sqrt(sq3(i1));
    const double theta = std::acos(dot(p21, i1) / (p21l * i1l));
    const double ixl = i1l * std::sin(theta);
    const V3 v = 0.5 * (p21 + p31);
    const double vl = std::sqrt(sq3(v));
    const V3 h = 0.5 * ((-p32) + (-p31));
    const double hl = std::sqrt(sq3(h));
    const double uv = vl / 160.0, uh = hl / 160.0;
    y = x86_trunc(i1l / uh);
    x = x86_trunc(ixl / uv);
}

void tex_exp_quad(const Ent& e, V3 ip, int32_t& x, int32_t& y) {
    const double uv = (double)e.width / 160.0, uh = (double)e.length_ / 160.0;
    const V3 rv = e.qv[0] - e.qv[1];
    const V3 i1 = ip - e.qv[1];
    const double i1l = std::sqrt(sq3(i1));
    const double theta = std::acos(dot(i1, rv) / ((double)e.width * i1l));
    y = x86_trunc(i1l * std::sin(theta) / uh);
    x = x86_trunc(i1l * std::cos(theta) / uv);
}

void tex_exp_sphere(const Ent& e, V3 ip, int32_t& x, int32_t& y) {   // entities.h:549-571
    const double r = e.radius;
    const double unit_v = 2.0 * REF_PI * r / 320.0;
    const V3 to = ip - e.pos;
    const double cos_vert = dot(to, V3{0, 0, r}) / (r * r);
    const double ang = std::acos(cos_vert);
    y = x86_trunc((0.5 * REF_PI * r - r * ang) / unit_v);
    const double small_r = r * std::sin(ang);
    const double cos_hori = dot(V3{to.x, to.y, 0}, V3{0, small_r, 0}) / (small_r * small_r);
    const double unit_h = 2.0 * REF_PI * small_r / 320.0;
    x = x86_trunc(small_r * std::acos(cos_hori) / unit_h);
}

void tex_exp_cube(const Ent& e, V3 ip, int32_t& x, int32_t& y) {   // entities.h:769-811
    const double uv = (double)e.width / 160.0, uh = (double)e.length_ / 160.0;
    const V3 rv{0, (double)e.width, 0};
    const V3 i1 = ip - e.qv[0];
    const double l = std::sqrt(sq3(i1));
    const double theta = std::acos(dot(i1, rv) / ((double)e.width * l));
    y = x86_trunc(l * std::sin(theta) / uh);
    x = x86_trunc(l * std::cos(theta) / uv);
}

void tex_exp_cone(const Ent& e, V3 ip, int32_t& x, int32_t& y) {   // entities.h:942-961
    const double R = e.radius, H = e.height;
    const double unit_h = std::sqrt(R * R + H * H) / 320.0;
    const V3 ipos = ip - e.pos;
    const double ylen = std::sqrt(sq3(ipos));
    y = x86_trunc(ylen / unit_h);
    const V3 center{(double)(float)e.pos.x, (double)(float)e.pos.y, (double)(float)ip.z};   // glm::vec3
    const double rp = ylen * std::sin(e.cone_theta);
    const V3 left{0, (double)(float)rp, 0};                                               // glm::vec3
    const V3 ic = ip - center;
    const double unit_v = 2.0 * REF_PI * rp / 320.0;
    double alpha = std::acos(dot(ic, left) / (rp * rp));
    if (alpha > REF_PI / 4.0) alpha = std::acos(dot(ic, -left) / (rp * rp));
    x = x86_trunc(rp * alpha / unit_v);
}

void tex_exp_rectangle(const Ent& e, V3 ip, int32_t& x, int32_t& y) {   // entities.h:346-365
    const V3 p1 = e.qv[0], p3 = e.qv[1], p4 = e.qv[2];
    const V3 p31 = p3 - p1, p41 = p4 - p1;
    const double width = std::sqrt(sq3(p41)), length = std::sqrt(sq3(p31));
    const double uv = width / 64.0, uh = length / 64.0;
    const V3 i1 = ip - p1;
    const double l = std::sqrt(sq3(i1));
    const double ct = std::acos(dot(i1, p31) / (length * l));   // an angle named cos_theta
    x = x86_trunc(l * std::sin(std::acos(ct)) / uh);
    y = x86_trunc(l * ct / uv);
}

void tex_coord(const Ent& e, V3 ip, int32_t& x, int32_t& y) {
    switch (e.kind) {
    case IMP_SPHERE: tex_imp_sphere(e, ip, x, y); return;
    case IMP_TRIANGLE: tex_imp_triangle(e.tri, ip, x, y); return;
    case EXP_QUAD: tex_exp_quad(e, ip, x, y); return;
    case EXP_SPHERE: tex_exp_sphere(e, ip, x, y); return;
    case EXP_CUBE: tex_exp_cube(e, ip, x, y); return;
    case EXP_CONE: tex_exp_cone(e, ip, x, y); return;
    case EXP_RECTANGLE: tex_exp_rectangle(e, ip, x, y); return;
    }
    x = y = 0;   // ExpBox (entities.h:448-451)
}

// Texture (material.h:65-106): 32x32 int checker; colours truncated to int (A.7).  A negative
// remainder indexes pattern[i][j] out of its row (A.9): the compiled reference reads the flat
// element i*32+j, which stays inside the array when 0 <= i*32+j < 1024; outside the array it
// reads stack memory (UB) -- this restatement then wraps the flat index into [0,1024).
V3 texel(V3 color, int32_t u, int32_t v) {
    int f = (u % 32) * 32 + (v % 32);
    if (f < 0 || f >= 1024) f = ((f % 1024) + 1024) % 1024;
    const int i = f / 32, j = f % 32;
    if ((i <= 16 && j <= 16) || (i > 16 && j > 16)) return {1, 1, 1};
    return {(double)x86_trunc(color.x), (double)x86_trunc(color.y), (double)x86_trunc(color.z)};
}

// Material::blinn_phong_texture (material.h:48-62)
V3 shade_ref(const Mat& m, V3 dir, V3 light, V3 ip, V3 n, int32_t u, int32_t v) {
    const V3 tc = texel(m.color, u, v);
    const V3 tdc = tc * 0.5;
    const V3 la = tc * m.shader.x;
    const V3 ld = (smax(0.0, dot(n, normalize(light - ip))) * tdc) * m.shader.y;
    const V3 bis = normalize(normalize(-dir) + normalize(light - ip));
    const V3 ls = (std::pow(smax(0.0, dot(n, bis)), m.spec_pow) * V3{1, 1, 1}) * m.shader.z;
    const V3 out = (la + ld) + ls;
    return {smin(out.x, 1.0), smin(out.y, 1.0), smin(out.z, 1.0)};
}

// Image::setPixel (image.h:14-16) + QColor range check
void quantize(const double* c, uint8_t* q) {
    int32_t r = x86_trunc(255 * c[0]), g = x86_trunc(255 * c[1]), b = x86_trunc(255 * c[2]);
    if (r < 0 || r > 255 || g < 0 || g > 255 || b < 0 || b > 255) { q[0] = q[1] = q[2] = 0; return; }
    q[0] = (uint8_t)r; q[1] = (uint8_t)g; q[2] = (uint8_t)b;
}

// ---- octree (octree.h:12-163, bbox.h:25-39) ------------------------------------------------
bool bb_intersect(V3 amin, V3 amax, V3 bmin, V3 bmax) {
    const V3 p1 = 0.5 * (amin + amax), p2 = 0.5 * (bmin + bmax);
    const V3 d = p1 - p2;
    const bool xo = std::fabs(d.x) < (0.5 * (amax.x - amin.x) + 0.5 * (bmax.x - bmin.x));
    const bool yo = std::fabs(d.y) < (0.5 * (amax.y - amin.y) + 0.5 * (bmax.y - bmin.y));
    const bool zo = std::fabs(d.z) < (0.5 * (amax.z - amin.z) + 0.5 * (bmax.z - bmin.z));
    return xo && yo && zo;
}
inline bool le3(V3 a, V3 b) { return a.x <= b.x && a.y <= b.y && a.z <= b.z; }

struct Node {
    V3 mn, mx;
    std::vector<int> ents;
    int child0 = -1;
};

struct Octree {
    std::vector<Node> nodes;
    const std::vector<Ent>* ents = nullptr;

    void init(V3 mn, V3 mx) { nodes.clear(); nodes.push_back(Node{mn, mx, {}, -1}); }

    void partition(int ni) {   // octree.h:75-110
        if (nodes[ni].child0 >= 0) return;
        const V3 mn = nodes[ni].mn, mx = nodes[ni].mx;
        const V3 mid = (mn + mx) * 0.5;
        bool all_in = true;
        for (int e : nodes[ni].ents) {
            const Ent& E = (*ents)[e];
            all_in = all_in && le3(E.bmin, mid) && le3(mid, E.bmax);
        }
        if (all_in) return;
        const int c0 = (int)nodes.size();
        const V3 bx[8][2] = {
            {mn, mid},
            {{mn.x, mid.y, mn.z}, {mid.x, mx.y, mid.z}},
            {{mid.x, mn.y, mn.z}, {mx.x, mid.y, mid.z}},
            {{mid.x, mid.y, mn.z}, {mx.x, mx.y, mid.z}},
            {mid, mx},
            {{mn.x, mid.y, mid.z}, {mid.x, mx.y, mx.z}},
            {{mid.x, mn.y, mid.z}, {mx.x, mid.y, mx.z}},
            {{mn.x, mn.y, mid.z}, {mid.x, mid.y, mx.z}},
        };
        for (int c = 0; c < 8; ++c) nodes.push_back(Node{bx[c][0], bx[c][1], {}, -1});
        nodes[ni].child0 = c0;
    }

    void push_obj(int ni, int e) {   // octree.h:115-129
        nodes[ni].ents.push_back(e);
        partition(ni);
        if (nodes[ni].child0 < 0) return;
        const Ent& E = (*ents)[e];
        for (int c = 0; c < 8; ++c) {
            const int ci = nodes[ni].child0 + c;
            if (le3(nodes[ci].mn, E.bmin) && le3(E.bmax, nodes[ci].mx)) push_obj(ci, e);
            else if (bb_intersect(nodes[ci].mn, nodes[ci].mx, E.bmin, E.bmax)) nodes[ci].ents.push_back(e);
        }
    }

    void push_back(int e) {   // octree.h:20-43
        const Ent& E = (*ents)[e];
        if (!bb_intersect(nodes[0].mn, nodes[0].mx, E.bmin, E.bmax)) return;   // A.14
        push_obj(0, e);
    }
};

// ExpBox node test (entities.h:379-440): OR over 6 ExpRectangle faces, each t1=(p1,p2,p3) or
// t2=(p1,p2,p4) with p4 = -p3 (A.4).  Only the bool is used by Octree::Node::intersect.
bool rect_hit(V3 p1, V3 p2, V3 p3, V3 o, V3 d) {
    V3 P, N;
    if (tri_intersect(make_tri(p1, p2, p3), o, d, P, N)) return true;
    return tri_intersect(make_tri(p1, p2, -p3), o, d, P, N);
}
bool box_hit(V3 mn, V3 mx, V3 o, V3 d) {
    const V3 dlb = mn, drb{mx.x, mn.y, mn.z}, dlt{mn.x, mx.y, mn.z}, drt{mx.x, mx.y, mn.z};
    const V3 ulb{mn.x, mn.y, mx.z}, urb{mx.x, mn.y, mx.z}, ult{mn.x, mx.y, mx.z}, urt = mx;
    bool hit = false;
    hit = rect_hit(dlb, urb, ulb, o, d) || hit;
    hit = rect_hit(dlb, ult, dlt, o, d) || hit;
    hit = rect_hit(dlb, drt, dlt, o, d) || hit;
    hit = rect_hit(urt, ulb, ult, o, d) || hit;
    hit = rect_hit(urt, drb, drt, o, d) || hit;
    hit = rect_hit(urt, dlt, drt, o, d) || hit;
    return hit;
}

void query(const Octree& t, int ni, V3 o, V3 d, std::vector<int>& out, int& ntests) {   // octree.h:132-155
    const Node& n = t.nodes[ni];
    if (n.child0 < 0) { out.insert(out.end(), n.ents.begin(), n.ents.end()); return; }
    for (int c = 0; c < 8; ++c) {
        const int ci = n.child0 + c;
        if (t.nodes[ci].ents.empty()) continue;
        ++ntests;
        if (box_hit(t.nodes[ci].mn, t.nodes[ci].mx, o, d)) query(t, ci, o, d, out, ntests);
    }
}

// ---- scene -----------------------------------------------------------------------------------
struct Scene {
    V3 omin{-20, -20, -20}, omax{20, 20, 20};
    V3 cpos{-10, 0, 0}, clook{1, 0, 0};
    double focal = 0.1;
    V3 light{-10, 10, 10};
    std::vector<Ent> ents;
    Octree tree;
};

bool parse(const char* text, Scene& s, bool build_tree = true) {
    std::istringstream in(text);
    std::string line;
    while (std::getline(in, line)) {
        size_t h = line.find('#');
        if (h != std::string::npos) line = line.substr(0, h);
        std::istringstream is(line);
        std::string kw;
        if (!(is >> kw)) continue;
        std::vector<double> v;
        double x;
        while (is >> x) v.push_back(x);
        auto need = [&](size_t n) { return v.size() >= n; };
        if (kw == "octree" && need(6)) { s.omin = {v[0], v[1], v[2]}; s.omax = {v[3], v[4], v[5]}; }
        else if (kw == "camera" && need(7)) { s.cpos = {v[0], v[1], v[2]}; s.clook = {v[3], v[4], v[5]}; s.focal = v[6]; }
        else if (kw == "light" && need(3)) s.light = {v[0], v[1], v[2]};
        else if (kw == "impsphere" && need(7)) s.ents.push_back(make_imp_sphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}));
        else if (kw == "imptriangle" && need(9)) s.ents.push_back(make_imp_triangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]}));
        else if (kw == "expquad" && need(9)) s.ents.push_back(make_exp_quad({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]}));
        else if (kw == "expsphere" && need(7)) s.ents.push_back(make_exp_sphere({v[0], v[1], v[2]}, v[3], {v[4], v[5], v[6]}));
        else if (kw == "expcube" && need(9)) s.ents.push_back(make_exp_cube({v[0], v[1], v[2]}, v[3], v[4], v[5], {v[6], v[7], v[8]}));
        else if (kw == "expcone" && need(11)) s.ents.push_back(make_exp_cone({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, v[6], v[7], {v[8], v[9], v[10]}));
        else if (kw == "exprectangle" && need(9)) s.ents.push_back(make_exp_rectangle({v[0], v[1], v[2]}, {v[3], v[4], v[5]}, {v[6], v[7], v[8]}));
        else if (kw == "expbox" && need(6)) s.ents.push_back(make_exp_box({v[0], v[1], v[2]}, {v[3], v[4], v[5]}));
        else if (kw == "material" && need(3)) {
            if (s.ents.empty()) { g_err = "material before entity"; return false; }
            Mat m;
            m.color = {v[0], v[1], v[2]};
            if (v.size() >= 6) m.shader = {v[3], v[4], v[5]};
            if (v.size() >= 7) m.spec_pow = v[6];
            if (v.size() >= 8) m.refl = v[7];
            s.ents.back().mat = m;
        } else { g_err = "unsupported scene line: " + line; return false; }
    }
    s.tree.ents = &s.ents;
    s.tree.init(s.omin, s.omax);
    if (build_tree)   // Mode X does not use the reference octree
        for (int i = 0; i < (int)s.ents.size(); ++i) s.tree.push_back(i);
    return true;
}

struct Cam {
    V3 pos, up{0, 0, 1}, fwd, left, top_left;
    double focal, rx = 0.0002, ry = 0.0002;
};
Cam make_cam(const Scene& s, int w) {   // camera.h:8-10, raytracer.h:26-30
    Cam c;
    c.pos = s.cpos;
    c.fwd = normalize(s.clook - s.cpos);
    c.focal = s.focal;
    c.left = normalize(cross(c.up, c.fwd));
    c.top_left = (((c.pos + c.focal * c.fwd) + ((c.left * (double)w) * 0.5) * c.rx) + ((c.up * (double)w) * 0.5) * c.ry) - c.pos;
    return c;
}

// ---- Mode R pixel (raytracer.h:41-84) -------------------------------------------------------
void pixel_mode_r(const Scene& s, const Cam& c, int x, int y, double* rgb, int32_t& hit, int32_t& u,
                  int32_t& v, int32_t& ncand, int32_t& nnode) {
    const V3 dir0 = (c.top_left - (c.left * (double)x) * c.rx) - (c.up * (double)y) * c.ry;
    const V3 o = c.pos, d = normalize(dir0);   // Ray ctor (ray.h:6)
    std::vector<int> cand;
    int nt = 0;
    query(s.tree, 0, o, d, cand, nt);
    ncand = (int32_t)cand.size();
    nnode = nt;
    int front = -1;
    V3 ip{DBL_MAX, DBL_MAX, DBL_MAX}, nrm{0, 0, 0};
    for (int e : cand) {   // last hitting candidate wins (A.1)
        V3 P, N;
        if (ent_intersect(s.ents[e], o, d, P, N)) {
            const double d2 = sq3(P - o);
            if (d2 < DBL_MAX) { ip = P; nrm = N; front = e; }
        }
    }
    hit = front;
    if (front < 0) { rgb[0] = rgb[1] = rgb[2] = 0; u = v = 0; return; }
    tex_coord(s.ents[front], ip, u, v);
    const V3 col = shade_ref(s.ents[front].mat, d, s.light, ip, nrm, u, v);
    rgb[0] = col.x; rgb[1] = col.y; rgb[2] = col.z;
}

// ============================================================================================
// Mode X — build-defined integrator (DESIGN.md "Mode X").  Only +,-,*,/,sqrt and comparisons
// (all correctly rounded, no contraction), so the GPU kernel can match it bit for bit.
// ============================================================================================
const double MX_TMIN = 1e-7;
const double MX_PI = 0x1.921fb54442d18p+1, MX_PIO2 = 0x1.921fb54442d18p+0;
const double ASIN_C[30] = {
    0x1.0000000000000p+0, 0x1.5555555555555p-3, 0x1.3333333333333p-4, 0x1.6db6db6db6db7p-5,
    0x1.f1c71c71c71c7p-6, 0x1.6e8ba2e8ba2e9p-6, 0x1.1c4ec4ec4ec4fp-6, 0x1.c99999999999ap-7,
    0x1.7a87878787878p-7, 0x1.3fde50d79435ep-7, 0x1.12ef3cf3cf3cfp-7, 0x1.df3bd37a6f4dfp-8,
    0x1.a6863d70a3d71p-8, 0x1.782dda12f684cp-8, 0x1.51ba308d3dcb1p-8, 0x1.31683bdef7bdfp-8,
    0x1.15ee9d45d1746p-8, 0x1.fcaf8fb6db6dbp-9, 0x1.d3d2a8e0dd67dp-9, 0x1.b026f57b13b14p-9,
    0x1.90cb77f60c7cep-9, 0x1.750de64d7d05fp-9, 0x1.5c5f56efaaaabp-9, 0x1.464c0950f7d47p-9,
    0x1.3275586c5f2f0p-9, 0x1.208d3570ae5a6p-9, 0x1.1052bc5fa960ap-9, 0x1.018f963c229bfp-9,
    0x1.e82be60d9127ep-10, 0x1.cf7dea5b6e830p-10};

double mx_asin_small(double y) {   // |y| <= 0.5: Taylor series, Horner, 30 terms
    const double z = y * y;
    double p = ASIN_C[29];
    for (int k = 28; k >= 0; --k) p = p * z + ASIN_C[k];
    return y * p;
}
double mx_acos(double x) {
    if (!(x >= -1.0 && x <= 1.0)) return NAN;
    if (x >= -0.5 && x <= 0.5) return MX_PIO2 - mx_asin_small(x);
    if (x > 0.5) return 2.0 * mx_asin_small(std::sqrt((1.0 - x) * 0.5));
    return MX_PI - 2.0 * mx_asin_small(std::sqrt((1.0 + x) * 0.5));
}
double mx_sin_acos(double c) { return std::sqrt(1.0 - c * c); }            // NaN for |c| > 1
double mx_cos_acos(double c) { return (c >= -1.0 && c <= 1.0) ? c : NAN; }

double mx_powi(double x, int p) {
    double r = 1.0, b = x;
    while (p) {
        if (p & 1) r = r * b;
        b = b * b;
        p >>= 1;
    }
    return r;
}

// Any specular power (material.h:29 is a double): integer p in [0, 64] by square-and-multiply,
// otherwise exp(p * ln x) -- ln from the atanh series of the mantissa in [sqrt(1/2), sqrt(2)],
// exp by a degree-17 Taylor polynomial after n = round(y / ln 2), 2^n through the exponent bits.
// Only +, -, *, / and exact bit operations: the same doubles on any IEEE machine.
double mx_ln(double x) {
    int e = 0;
    if (x < 0x1.0p-1022) { x = x * 0x1.0p+54; e = -54; }
    uint64_t b;
    memcpy(&b, &x, 8);
    e += (int)((b >> 52) & 0x7FF) - 1023;
    const uint64_t mb = (b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    memcpy(&m, &mb, 8);
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }
    const double s = (m - 1.0) / (m + 1.0), z = s * s;
    static const double inv_odd[13] = {1.0 / 25.0, 1.0 / 23.0, 1.0 / 21.0, 1.0 / 19.0, 1.0 / 17.0, 1.0 / 15.0, 1.0 / 13.0,
                                       1.0 / 11.0, 1.0 / 9.0, 1.0 / 7.0, 1.0 / 5.0, 1.0 / 3.0, 1.0};
    double q = inv_odd[0];
    for (int k = 1; k < 13; ++k) q = q * z + inv_odd[k];
    const double de = (double)e;
    return de * 0x1.62e42fee00000p-1 + (de * 0x1.a39ef35793c76p-33 + 2.0 * s * q);
}
double mx_exp(double y) {
    if (!(y > -746.0)) return std::isnan(y) ? y : 0.0;
    if (y > 710.0) return INFINITY;
    const int n = (int)(y * 0x1.71547652b82fep+0 + (y >= 0.0 ? 0.5 : -0.5));
    const double dn = (double)n;
    const double r = (y - dn * 0x1.62e42fee00000p-1) - dn * 0x1.a39ef35793c76p-33;
    static const double inv_fact[18] = {1.0 / 355687428096000.0, 1.0 / 20922789888000.0, 1.0 / 1307674368000.0,
                                        1.0 / 87178291200.0, 1.0 / 6227020800.0, 1.0 / 479001600.0, 1.0 / 39916800.0,
                                        1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0, 1.0 / 5040.0, 1.0 / 720.0,
                                        1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5, 1.0, 1.0};
    double q = inv_fact[0];
    for (int k = 1; k < 18; ++k) q = q * r + inv_fact[k];
    uint64_t sb;
    double sc;
    if (n >= -1022) {
        sb = (uint64_t)(n + 1023) << 52;
        memcpy(&sc, &sb, 8);
        return q * sc;
    }
    sb = (uint64_t)(n + 1023 + 54) << 52;
    memcpy(&sc, &sb, 8);
    return (q * sc) * 0x1.0p-54;
}
double mx_pow(double x, double p) {
    if (p >= 0.0 && p <= 64.0 && p == (double)(int)p) return mx_powi(x, (int)p);
    if (std::isnan(p) || std::isnan(x)) return NAN;
    if (x == 0.0) return p > 0.0 ? 0.0 : INFINITY;
    if (x < 0.0) return NAN;
    if (std::isinf(x)) return p > 0.0 ? x : 0.0;
    return mx_exp(p * mx_ln(x));
}

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
inline double mx_u01(uint64_t seed, uint64_t pixel, uint32_t sample, uint32_t bounce, uint32_t dim) {
    uint64_t k = mix64(seed + 0x9E3779B97F4A7C15ULL * (pixel + 1));
    k = mix64(k ^ (((uint64_t)sample << 32) | ((uint64_t)(bounce & 0xFFFF) << 16) | (uint64_t)(dim & 0xFFFF)));
    return (double)(k >> 11) * 0x1.0p-53;
}

// Shirley-Chiu concentric map of (u1,u2) to the unit disk; sin/cos on [-pi/4, pi/4] by Taylor
// polynomials (degree 17 / 16, Horner), fp64 +,-,* only.
void mx_sincos_q(double p, double& sn, double& cs) {
    static const double S[8] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
    -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49};
    static const double C[8] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
    -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45};
    const double z = p * p;
    double ps = S[7], pc = C[7];
    for (int k = 6; k >= 0; --k) {
        ps = ps * z + S[k];
        pc = pc * z + C[k];
    }
    sn = p + p * (z * ps);
    cs = 1.0 + z * pc;
}
void mx_disk(double u1, double u2, double& dx, double& dy, double& r2) {
    const double a = 2.0 * u1 - 1.0, b = 2.0 * u2 - 1.0;
    const double QPI = 0x1.921fb54442d18p-1;
    if (a == 0.0 && b == 0.0) { dx = dy = r2 = 0.0; return; }
    double r, sn, cs;
    if (std::fabs(a) > std::fabs(b)) {
        r = a;
        mx_sincos_q(QPI * (b / a), sn, cs);
        dx = r * cs;
        dy = r * sn;
    } else {
        r = b;
        mx_sincos_q(QPI * (a / b), sn, cs);
        dx = r * sn;
        dy = r * cs;
    }
    r2 = r * r;
}

struct Prim {
    int kind;     // 0 = triangle, 1 = sphere
    int ent;
    V3 v0, e1, e2, n;   // triangle: p1, p2-p1, p3-p1, normalize(cross(e1,e2))
    V3 c;               // sphere centre
    double r;           // sphere radius (the float radius widened)
};

void build_prims(const Scene& s, std::vector<Prim>& prims) {
    for (int i = 0; i < (int)s.ents.size(); ++i) {
        const Ent& e = s.ents[i];
        auto add_tri = [&](const Tri& t) {
            Prim p{};
            p.kind = 0; p.ent = i; p.v0 = t.p1; p.e1 = t.e1; p.e2 = t.e2; p.n = t.n;
            prims.push_back(p);
        };
        if (e.kind == IMP_SPHERE) {
            Prim p{};
            p.kind = 1; p.ent = i; p.c = e.pos; p.r = (double)e.radius;
            prims.push_back(p);
        } else if (e.kind == IMP_TRIANGLE) add_tri(e.tri);
        else for (const Tri& t : e.tris) add_tri(t);
    }
}

// Möller–Trumbore, two-sided, with the barycentric tests on the numerators (u = un/det in [0,1],
// v = vn/det >= 0, u + v <= 1 compared as un, vn, un+vn against 0 and det, by the sign of det);
// t = tn/det is the only division.  Returns t or +inf.
// Mode X arithmetic with fused multiply-adds (std::fma: correctly rounded, as the device's
// v_fma_f64): dot = fma(z, z', fma(y, y', x*x')), cross components fma(a, b, -(c*d)).
inline double fdot(V3 a, V3 b) { return std::fma(a.z, b.z, std::fma(a.y, b.y, a.x * b.x)); }
inline V3 fcross(V3 x, V3 y) {
    return {std::fma(x.y, y.z, -(y.y * x.z)), std::fma(x.z, y.x, -(y.z * x.x)), std::fma(x.x, y.y, -(y.x * x.y))};
}
double mx_tri_t(const Prim& p, V3 o, V3 d, double tmin) {
    const V3 pv = fcross(d, p.e2);
    const double det = fdot(p.e1, pv);
    if (det == 0.0) return INFINITY;
    const V3 tv = o - p.v0;
    const double un = fdot(tv, pv);
    if (det > 0.0 ? (un < 0.0 || un > det) : (un > 0.0 || un < det)) return INFINITY;
    const V3 qv = fcross(tv, p.e1);
    const double vn = fdot(d, qv);
    const double uvn = un + vn;
    if (det > 0.0 ? (vn < 0.0 || uvn > det) : (vn > 0.0 || uvn < det)) return INFINITY;
    const double t = fdot(p.e2, qv) / det;
    return (t > tmin) ? t : INFINITY;
}
double mx_sph_t(const Prim& p, V3 o, V3 d, double tmin) {
    const V3 oc = o - p.c;
    const double b = fdot(oc, d);
    const double c2 = std::fma(-p.r, p.r, fdot(oc, oc));
    const double disc = std::fma(b, b, -c2);
    if (disc < 0.0) return INFINITY;
    const double sq = std::sqrt(disc);
    double t = -b - sq;
    if (t > tmin) return t;
    t = -b + sq;
    return (t > tmin) ? t : INFINITY;
}
inline double mx_prim_t(const Prim& p, V3 o, V3 d, double tmin) {
    return p.kind == 0 ? mx_tri_t(p, o, d, tmin) : mx_sph_t(p, o, d, tmin);
}

// Closest hit over ALL primitives: min t > MX_TMIN, ties to the lower primitive index; shadow
// query: any t in (MX_TMIN, tmax).  Two equivalent evaluations (same answer for every ray):
//  * brute force over the primitive list (structure independent; small scenes, cross-checks);
//  * this oracle's own binary BVH (median split, fp64 boxes padded far above rounding), used for
//    large scenes so the C4/C5 workloads can be checked in seconds.  It only skips primitives
//    whose padded box the ray cannot reach before the current best t, so it returns exactly what
//    the brute force returns (CPU test: tests/test_oracle_golden.py, bvh vs brute force).
struct OAccel {
    struct Node { double lo[3], hi[3]; int left, right, first, count; };   // leaf: left < 0
    std::vector<Node> nodes;
    std::vector<int> idx;
    bool brute = true;
};

int g_no_shadow = 0;     // gio_set_no_shadow (tests): Mode X without shadow rays (GI_FLAG_X_NO_SHADOW)
int g_accel_mode = -1;   // -1: BVH above 256 primitives; 0: always brute force; 1: always BVH

void prim_bounds(const Prim& p, double lo[3], double hi[3]) {
    if (p.kind == 0) {
        const V3 a = p.v0, b = p.v0 + p.e1, c = p.v0 + p.e2;
        const double va[3] = {a.x, a.y, a.z}, vb[3] = {b.x, b.y, b.z}, vc[3] = {c.x, c.y, c.z};
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::fmin(va[k], std::fmin(vb[k], vc[k]));
            hi[k] = std::fmax(va[k], std::fmax(vb[k], vc[k]));
        }
    } else {
        const double cc[3] = {p.c.x, p.c.y, p.c.z};
        for (int k = 0; k < 3; ++k) { lo[k] = cc[k] - p.r; hi[k] = cc[k] + p.r; }
    }
    for (int k = 0; k < 3; ++k) {   // padding: 1e-7 of the coordinates' magnitude plus the extent
        const double pad = 1e-7 * (std::fabs(lo[k]) + std::fabs(hi[k]) + (hi[k] - lo[k])) + 1e-12;
        lo[k] -= pad;
        hi[k] += pad;
    }
}

int build_node(OAccel& A, std::vector<double>& blo, std::vector<double>& bhi, std::vector<double>& cen, int first,
               int count) {
    OAccel::Node nd;
    for (int k = 0; k < 3; ++k) { nd.lo[k] = INFINITY; nd.hi[k] = -INFINITY; }
    double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = first; i < first + count; ++i) {
        const int q = A.idx[i];
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = std::fmin(nd.lo[k], blo[3 * q + k]);
            nd.hi[k] = std::fmax(nd.hi[k], bhi[3 * q + k]);
            clo[k] = std::fmin(clo[k], cen[3 * q + k]);
            chi[k] = std::fmax(chi[k], cen[3 * q + k]);
        }
    }
    nd.left = nd.right = -1;
    nd.first = first;
    nd.count = count;
    const int me = (int)A.nodes.size();
    A.nodes.push_back(nd);
    if (count <= 4) return me;
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[ax] - clo[ax]) ax = k;
    const int mid = first + count / 2;
    std::nth_element(A.idx.begin() + first, A.idx.begin() + mid, A.idx.begin() + first + count, [&](int a, int b) {
        const double ca = cen[3 * a + ax], cb = cen[3 * b + ax];
        return ca < cb || (ca == cb && a < b);
    });
    const int l = build_node(A, blo, bhi, cen, first, mid - first);
    const int r = build_node(A, blo, bhi, cen, mid, first + count - mid);
    A.nodes[me].left = l;
    A.nodes[me].right = r;
    return me;
}

void build_accel(const std::vector<Prim>& prims, OAccel& A) {
    A.brute = g_accel_mode == 0 || (g_accel_mode < 0 && prims.size() <= 256);
    A.nodes.clear();
    A.idx.clear();
    if (A.brute || prims.empty()) { A.brute = true; return; }
    const int n = (int)prims.size();
    std::vector<double> blo(3 * (size_t)n), bhi(3 * (size_t)n), cen(3 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        prim_bounds(prims[i], &blo[3 * (size_t)i], &bhi[3 * (size_t)i]);
        for (int k = 0; k < 3; ++k) cen[3 * (size_t)i + k] = 0.5 * (blo[3 * (size_t)i + k] + bhi[3 * (size_t)i + k]);
    }
    A.idx.resize((size_t)n);
    for (int i = 0; i < n; ++i) A.idx[(size_t)i] = i;
    A.nodes.reserve(2 * (size_t)n / 2 + 8);
    build_node(A, blo, bhi, cen, 0, n);
}

// fp64 slab test of a padded box against the ray segment t in [0, tlim]
bool node_reach(const OAccel::Node& nd, V3 o, V3 d, double tlim) {
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    double tn = 0.0, tf = tlim;
    for (int k = 0; k < 3; ++k) {
        if (dd[k] == 0.0) {
            if (oo[k] < nd.lo[k] || oo[k] > nd.hi[k]) return false;
            continue;
        }
        double t0 = (nd.lo[k] - oo[k]) / dd[k], t1 = (nd.hi[k] - oo[k]) / dd[k];
        if (t0 > t1) std::swap(t0, t1);
        tn = std::fmax(tn, t0);
        tf = std::fmin(tf, t1);
    }
    return tn <= tf;
}
inline double t_slack(double t) { return std::isinf(t) ? t : t * (1.0 + 1e-9) + 1e-9; }

int mx_closest(const std::vector<Prim>& prims, const OAccel& A, V3 o, V3 d, double& tbest) {
    int best = -1;
    tbest = INFINITY;
    if (A.brute) {
        for (int i = 0; i < (int)prims.size(); ++i) {
            const double t = mx_prim_t(prims[i], o, d, MX_TMIN);
            if (t < tbest) { tbest = t; best = i; }   // strict: ties keep the lower index
        }
        return best;
    }
    int stack[128], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const OAccel::Node& nd = A.nodes[stack[--sp]];
        if (!node_reach(nd, o, d, t_slack(tbest))) continue;
        if (nd.left < 0) {
            for (int j = nd.first; j < nd.first + nd.count; ++j) {
                const int i = A.idx[j];
                const double t = mx_prim_t(prims[i], o, d, MX_TMIN);
                if (t < tbest || (t == tbest && i < best)) { tbest = t; best = i; }
            }
        } else {
            stack[sp++] = nd.right;
            stack[sp++] = nd.left;
        }
    }
    return best;
}
bool mx_occluded(const std::vector<Prim>& prims, const OAccel& A, V3 o, V3 d, double tmax) {
    if (A.brute) {
        for (const Prim& p : prims)
            if (mx_prim_t(p, o, d, MX_TMIN) < tmax) return true;
        return false;
    }
    int stack[128], sp = 0;
    stack[sp++] = 0;
    const double tl = t_slack(tmax);
    while (sp) {
        const OAccel::Node& nd = A.nodes[stack[--sp]];
        if (!node_reach(nd, o, d, tl)) continue;
        if (nd.left < 0) {
            for (int j = nd.first; j < nd.first + nd.count; ++j)
                if (mx_prim_t(prims[A.idx[j]], o, d, MX_TMIN) < tmax) return true;
        } else {
            stack[sp++] = nd.right;
            stack[sp++] = nd.left;
        }
    }
    return false;
}

void mx_texcoord(const Ent& e, V3 ip, int32_t& x, int32_t& y) {
    if (e.kind == IMP_SPHERE) {
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - e.pos;
        const double cv = dot(to, V3{0, 0, r}) / (r * r);
        y = x86_trunc((r * mx_acos(cv)) / unit_v);
        const double small_r = r * mx_sin_acos(cv);
        const double ch = dot(V3{to.x, to.y, 0}, V3{0, small_r, 0}) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * mx_acos(ch) / unit_h);
    } else if (e.kind == IMP_TRIANGLE) {
        const Tri& t = e.tri;
        const V3 p21 = t.p2 - t.p1, p31 = t.p3 - t.p1, p32 = t.p3 - t.p2, i1 = ip - t.p1;
        const double p21l = std::sqrt(sq3(p21)), i1l = std::sqrt(sq3(i1));
        const double c = dot(p21, i1) / (p21l * i1l);
        const double ixl = i1l * mx_sin_acos(c);
        const double vl = std::sqrt(sq3(0.5 * (p21 + p31)));
        const double hl = std::sqrt(sq3(0.5 * ((-p32) + (-p31))));
        y = x86_trunc(i1l / (hl / 160.0));
        x = x86_trunc(ixl / (vl / 160.0));
    } else if (e.kind == EXP_QUAD) {
        const double uv = (double)e.width / 160.0, uh = (double)e.length_ / 160.0;
        const V3 rv = e.qv[0] - e.qv[1], i1 = ip - e.qv[1];
        const double i1l = std::sqrt(sq3(i1));
        const double c = dot(i1, rv) / ((double)e.width * i1l);
        y = x86_trunc(i1l * mx_sin_acos(c) / uh);
        x = x86_trunc(i1l * mx_cos_acos(c) / uv);
    } else if (e.kind == EXP_SPHERE) {   // tex_exp_sphere with the Mode X acos
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - e.pos;
        const double cv = dot(to, V3{0, 0, r}) / (r * r);
        y = x86_trunc((0.5 * REF_PI * r - r * mx_acos(cv)) / unit_v);
        const double small_r = r * mx_sin_acos(cv);
        const double ch = dot(V3{to.x, to.y, 0}, V3{0, small_r, 0}) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * mx_acos(ch) / unit_h);
    } else if (e.kind == EXP_CUBE) {
        const double uv = (double)e.width / 160.0, uh = (double)e.length_ / 160.0;
        const V3 i1 = ip - e.qv[0];
        const double l = std::sqrt(sq3(i1));
        const double c = dot(i1, V3{0, (double)e.width, 0}) / ((double)e.width * l);
        y = x86_trunc(l * mx_sin_acos(c) / uh);
        x = x86_trunc(l * mx_cos_acos(c) / uv);
    } else if (e.kind == EXP_CONE) {   // sin(cone_theta) is a build-time constant (host libm)
        const double R = e.radius, H = e.height;
        const double unit_h = std::sqrt(R * R + H * H) / 320.0;
        const double ylen = std::sqrt(sq3(ip - e.pos));
        y = x86_trunc(ylen / unit_h);
        const V3 center{(double)(float)e.pos.x, (double)(float)e.pos.y, (double)(float)ip.z};
        const double rp = ylen * std::sin(e.cone_theta);
        const V3 left{0, (double)(float)rp, 0};
        const V3 ic = ip - center;
        const double unit_v = 2.0 * REF_PI * rp / 320.0;
        double alpha = mx_acos(dot(ic, left) / (rp * rp));
        if (alpha > REF_PI / 4.0) alpha = mx_acos(dot(ic, -left) / (rp * rp));
        x = x86_trunc(rp * alpha / unit_v);
    } else if (e.kind == EXP_RECTANGLE) {
        const V3 p1 = e.qv[0], p31 = e.qv[1] - p1, p41 = e.qv[2] - p1;
        const double width = std::sqrt(sq3(p41)), length = std::sqrt(sq3(p31));
        const V3 i1 = ip - p1;
        const double l = std::sqrt(sq3(i1));
        const double ct = mx_acos(dot(i1, p31) / (length * l));
        x = x86_trunc(l * mx_sin_acos(ct) / (length / 64.0));
        y = x86_trunc(l * ct / (width / 64.0));
    } else x = y = 0;   // ExpBox
}

// One sample of pixel (x, y): its radiance L (before the pixel mean) and the rays it traced.
void sample_mode_x(const Scene& s, const std::vector<Prim>& prims, const OAccel& A, const Cam& c, int w, int x, int y,
                   int smp, int spp, int depth, uint64_t seed, V3& Lout, int32_t& hit0, int32_t& u0, int32_t& v0,
                   long& rays) {
    const uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
    double jx = 0.0, jy = 0.0;
    if (spp > 1) { jx = mx_u01(seed, pix, smp, 0xFFFF, 0); jy = mx_u01(seed, pix, smp, 0xFFFF, 1); }
    const V3 dir0 = (c.top_left - (c.left * ((double)x + jx)) * c.rx) - (c.up * ((double)y + jy)) * c.ry;
    V3 o = c.pos, d = normalize(dir0);
    V3 L{0, 0, 0}, T{1, 1, 1};
    for (int b = 0; b < depth; ++b) {
        double t;
        const int pi = mx_closest(prims, A, o, d, t);
        ++rays;
        if (pi < 0) break;
        const Prim& p = prims[pi];
        const Ent& e = s.ents[p.ent];
        const V3 P = o + t * d;
        V3 N = p.kind == 0 ? p.n : normalize(P - p.c);
        if (!(dot(d, N) < 0)) N = -N;
        int32_t tu, tv;
        mx_texcoord(e, P, tu, tv);
        if (smp == 0 && b == 0) { hit0 = p.ent; u0 = tu; v0 = tv; }
        const V3 tc = texel(e.mat.color, tu, tv);
        // local Blinn-Phong with a shadow ray toward the point light
        const V3 lv = s.light - P;
        const double ldist = std::sqrt(dot(lv, lv));
        const V3 Ld = normalize(lv);
        const bool vis = g_no_shadow || !mx_occluded(prims, A, P, Ld, ldist);
        ++rays;
        const V3 la = tc * e.mat.shader.x;
        V3 loc = la;
        if (vis) {
            const V3 ld = (smax(0.0, dot(N, Ld)) * (tc * 0.5)) * e.mat.shader.y;
            const V3 bis = normalize(normalize(-d) + Ld);
            const double sp = mx_pow(smax(0.0, dot(N, bis)), e.mat.spec_pow);
            const V3 ls = V3{sp, sp, sp} * e.mat.shader.z;
            loc = (la + ld) + ls;
        }
        loc = {smin(loc.x, 1.0), smin(loc.y, 1.0), smin(loc.z, 1.0)};
        L = L + mul(T, loc);
        if (b == depth - 1) break;
        // mirror bounce with probability refl (uniform dim 4): T unchanged, d reflected about N
        if (e.mat.refl > 0.0 && mx_u01(seed, pix, smp, b, 4) < e.mat.refl) {
            d = normalize(d - N * (2.0 * dot(d, N)));
            o = P;
            continue;
        }
        T = mul(T, tc * 0.5);
        if (T.x == 0.0 && T.y == 0.0 && T.z == 0.0) break;
        // cosine-weighted direction: concentric disk point + Malley's projection
        double sx, sy, r2;
        mx_disk(mx_u01(seed, pix, smp, b, 2), mx_u01(seed, pix, smp, b, 3), sx, sy, r2);
        const double sz = std::sqrt(1.0 - r2);
        const double sg = N.z >= 0.0 ? 1.0 : -1.0;   // Duff et al. 2017 orthonormal basis
        const double aa = -1.0 / (sg + N.z);
        const double bb = N.x * N.y * aa;
        const V3 t1{1.0 + sg * N.x * N.x * aa, sg * bb, -sg * N.x};
        const V3 t2{bb, sg + N.y * N.y * aa, -N.y};
        d = normalize((t1 * sx + t2 * sy) + N * sz);
        o = P;
    }
    Lout = L;
}

// pixel = min(sum_s L_s / spp, 1), samples added in order s = 0..spp-1 from +0.  Ls (optional):
// the samples' radiance, already computed (parallel over samples for small windows).
void pixel_mode_x(const Scene& s, const std::vector<Prim>& prims, const OAccel& A, const Cam& c, int w, int x, int y,
                  int spp, int depth, uint64_t seed, double* rgb, int32_t& hit0, int32_t& u0, int32_t& v0,
                  int32_t& nrays, const V3* Ls = nullptr, long pre_rays = 0) {
    double sum[3] = {0, 0, 0};
    hit0 = -1; u0 = v0 = 0;
    long rays = pre_rays;
    for (int smp = 0; smp < spp; ++smp) {
        V3 L;
        if (Ls) L = Ls[smp];
        else sample_mode_x(s, prims, A, c, w, x, y, smp, spp, depth, seed, L, hit0, u0, v0, rays);
        sum[0] = sum[0] + L.x; sum[1] = sum[1] + L.y; sum[2] = sum[2] + L.z;
    }
    for (int k = 0; k < 3; ++k) rgb[k] = smin(sum[k] / (double)spp, 1.0);
    nrays = (int32_t)rays;
}

}  // namespace

extern "C" {

const char* gio_last_error(void) { return g_err.c_str(); }

void gio_set_accel(int mode) { g_accel_mode = mode < 0 ? -1 : (mode ? 1 : 0); }

void gio_set_no_shadow(int on) { g_no_shadow = on ? 1 : 0; }

int gio_render(const char* scn, int w, int h, int mode, int spp, int depth, uint64_t seed, int x0, int y0,
               int x1, int y1, int threads, double* rgb, int32_t* hit, int32_t* uv, int32_t* ncand,
               int32_t* nnode, uint8_t* q) {
    Scene s;
    if (!parse(scn, s, mode != 1)) return -1;
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x1 > w || y1 > h || x0 > x1 || y0 > y1) { g_err = "bad window"; return -2; }
    if (mode == 1) {
        if (spp < 1 || depth < 1) { g_err = "mode X needs spp >= 1 and depth >= 1"; return -3; }
        for (const Ent& e : s.ents)
            if (!(e.mat.refl >= 0.0 && e.mat.refl <= 1.0)) { g_err = "reflectivity must lie in [0, 1]"; return -3; }
    }
    std::vector<Prim> prims;
    OAccel A;
    if (mode == 1) { build_prims(s, prims); build_accel(prims, A); }
    const Cam c = make_cam(s, w);
    const int ww = x1 - x0;
    const long npx = (long)ww * (y1 - y0);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    // few pixels with many samples: the samples of each pixel in parallel, summed in order after
    if (mode == 1 && spp > 1 && npx < 64) {
        std::vector<V3> Ls((size_t)spp);
        std::vector<long> nr((size_t)spp);
        std::vector<int32_t> h0((size_t)spp), uu((size_t)spp), vv((size_t)spp);
        for (long i = 0; i < npx; ++i) {
            const int x = x0 + (int)(i % ww), y = y0 + (int)(i / ww);
#pragma omp parallel for schedule(dynamic, 1)
            for (int smp = 0; smp < spp; ++smp) {
                nr[(size_t)smp] = 0;
                h0[(size_t)smp] = -1; uu[(size_t)smp] = vv[(size_t)smp] = 0;
                sample_mode_x(s, prims, A, c, w, x, y, smp, spp, depth, seed, Ls[(size_t)smp], h0[(size_t)smp],
                              uu[(size_t)smp], vv[(size_t)smp], nr[(size_t)smp]);
            }
            long rays = 0;
            for (int smp = 0; smp < spp; ++smp) rays += nr[(size_t)smp];
            double col[3];
            int32_t hh, u, v, nc;
            pixel_mode_x(s, prims, A, c, w, x, y, spp, depth, seed, col, hh, u, v, nc, Ls.data(), rays);
            hh = h0[0]; u = uu[0]; v = vv[0];
            if (rgb) { rgb[3 * i] = col[0]; rgb[3 * i + 1] = col[1]; rgb[3 * i + 2] = col[2]; }
            if (hit) hit[i] = hh;
            if (uv) { uv[2 * i] = u; uv[2 * i + 1] = v; }
            if (ncand) ncand[i] = nc;
            if (nnode) nnode[i] = 0;
            if (q) quantize(col, q + 3 * i);
        }
        return 0;
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (long i = 0; i < npx; ++i) {
        const int x = x0 + (int)(i % ww), y = y0 + (int)(i / ww);
        double col[3];
        int32_t hh, u, v, nc = 0, nn = 0;
        if (mode == 0) pixel_mode_r(s, c, x, y, col, hh, u, v, nc, nn);
        else { pixel_mode_x(s, prims, A, c, w, x, y, spp, depth, seed, col, hh, u, v, nc); nn = 0; }
        if (rgb) { rgb[3 * i] = col[0]; rgb[3 * i + 1] = col[1]; rgb[3 * i + 2] = col[2]; }
        if (hit) hit[i] = hh;
        if (uv) { uv[2 * i] = u; uv[2 * i + 1] = v; }
        if (ncand) ncand[i] = nc;
        if (nnode) nnode[i] = nn;
        if (q) quantize(col, q + 3 * i);
    }
    return 0;
}

// bench.py's cpu_baseline leg: Mode X over the full-width rows y = row0 + k * stride (k < n_rows),
// timed by the caller.  A primary sample whose ray misses the scene's bounding box (the union of the
// primitives' padded boxes, prim_bounds) adds exactly +0 and reaches no geometry: it is counted apart
// (out[1]) and not traced, as the GPU's classify pass / root-box pretest resolve such samples apart
// from its `value`.  out: [0] rays (primary + bounce + shadow, resolved ones included), [1] resolved
// primary samples, [2] pixels, [3] the sum of the pixels' radiance (keeps the work observable).
// rgb / q (optional, 3 per pixel of the rows, row by row): the pixels as gio_render writes them
// (fp64 radiance and RGB888) -- the whole-frame / strided-row parity tests and bench.py's check of
// its own GPU frame.
int gio_time_rows(const char* scn, int w, int h, int spp, int depth, uint64_t seed, int row0, int stride, int n_rows,
                  int threads, double* out, double* rgb, uint8_t* q) {
    Scene s;
    if (!parse(scn, s, false)) return -1;
    if (w <= 0 || h <= 0 || spp < 1 || depth < 1 || stride < 1 || n_rows < 0 || row0 < 0) { g_err = "bad arguments"; return -2; }
    std::vector<Prim> prims;
    OAccel A;
    build_prims(s, prims);
    build_accel(prims, A);
    double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (const Prim& p : prims) {
        double lo[3], hi[3];
        prim_bounds(p, lo, hi);
        for (int k = 0; k < 3; ++k) { blo[k] = std::fmin(blo[k], lo[k]); bhi[k] = std::fmax(bhi[k], hi[k]); }
    }
    const Cam c = make_cam(s, w);
    std::vector<int> rows;
    for (int k = 0; k < n_rows && row0 + (long)k * stride < h; ++k) rows.push_back(row0 + k * stride);
    const long npx = (long)rows.size() * w;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    long rays = 0, res = 0;
    double sum = 0.0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : rays, res, sum)
    for (long i = 0; i < npx; ++i) {
        const int x = (int)(i % w), y = rows[(size_t)(i / w)];
        const uint64_t pix = (uint64_t)y * (uint64_t)w + (uint64_t)x;
        double acc[3] = {0, 0, 0};
        for (int smp = 0; smp < spp; ++smp) {
            double jx = 0.0, jy = 0.0;
            if (spp > 1) { jx = mx_u01(seed, pix, smp, 0xFFFF, 0); jy = mx_u01(seed, pix, smp, 0xFFFF, 1); }
            const V3 d0 = normalize((c.top_left - (c.left * ((double)x + jx)) * c.rx) - (c.up * ((double)y + jy)) * c.ry);
            const double o3[3] = {c.pos.x, c.pos.y, c.pos.z}, d3[3] = {d0.x, d0.y, d0.z};
            double tn = 0.0, tf = INFINITY;
            for (int k = 0; k < 3; ++k) {
                const double t0 = (blo[k] - o3[k]) / d3[k], t1 = (bhi[k] - o3[k]) / d3[k];
                tn = std::fmax(tn, std::fmin(t0, t1));
                tf = std::fmin(tf, std::fmax(t0, t1));
            }
            if (prims.empty() || !(tn <= tf)) { ++rays; ++res; continue; }   // L = 0
            V3 L;
            int32_t h0 = -1, u0 = 0, v0 = 0;
            sample_mode_x(s, prims, A, c, w, x, y, smp, spp, depth, seed, L, h0, u0, v0, rays);
            acc[0] = acc[0] + L.x; acc[1] = acc[1] + L.y; acc[2] = acc[2] + L.z;
        }
        sum += acc[0] + acc[1] + acc[2];
        // the pixel as pixel_mode_x forms it (a resolved sample's +0 left out of acc changes no sum:
        // acc >= +0 throughout)
        double col[3];
        for (int k = 0; k < 3; ++k) col[k] = smin(acc[k] / (double)spp, 1.0);
        if (rgb) { rgb[3 * i] = col[0]; rgb[3 * i + 1] = col[1]; rgb[3 * i + 2] = col[2]; }
        if (q) quantize(col, q + 3 * i);
    }
    out[0] = (double)rays;
    out[1] = (double)res;
    out[2] = (double)npx;
    out[3] = sum;
    return 0;
}

long gio_tree(const char* scn, char* buf, long cap) {
    Scene s;
    if (!parse(scn, s)) return -1;
    std::string out;
    char tmp[512];
    for (size_t i = 0; i < s.ents.size(); ++i) {
        const Ent& e = s.ents[i];
        snprintf(tmp, sizeof tmp, "bbox %zu %.17g %.17g %.17g %.17g %.17g %.17g\n", i, e.bmin.x, e.bmin.y, e.bmin.z,
                 e.bmax.x, e.bmax.y, e.bmax.z);
        out += tmp;
    }
    struct R {
        static void dump(const Octree& t, int ni, int depth, int slot, std::string& out) {
            const Node& n = t.nodes[ni];
            char b[512];
            snprintf(b, sizeof b, "node %d %d %d %.17g %.17g %.17g %.17g %.17g %.17g %zu", depth, slot, n.child0 < 0 ? 1 : 0,
                     n.mn.x, n.mn.y, n.mn.z, n.mx.x, n.mx.y, n.mx.z, n.ents.size());
            out += b;
            for (int e : n.ents) { snprintf(b, sizeof b, " %d", e); out += b; }
            out += "\n";
            if (n.child0 >= 0)
                for (int c = 0; c < 8; ++c) dump(t, n.child0 + c, depth + 1, c, out);
        }
    };
    R::dump(s.tree, 0, 0, -1, out);
    if (buf && cap > 0) {
        long n = (long)out.size() < cap - 1 ? (long)out.size() : cap - 1;
        memcpy(buf, out.data(), (size_t)n);
        buf[n] = 0;
    }
    return (long)out.size();
}

int gio_rays(const char* scn, int n, const double* rays, int32_t* out_hit, double* out_pn, int32_t* out_uv) {
    Scene s;
    if (!parse(scn, s)) return -1;
    const size_t E = s.ents.size();
    for (int i = 0; i < n; ++i) {
        const V3 o{rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]};
        const V3 d = normalize(V3{rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]});
        for (size_t k = 0; k < E; ++k) {
            V3 P{0, 0, 0}, N{0, 0, 0};
            const size_t j = (size_t)i * E + k;
            const bool h = ent_intersect(s.ents[k], o, d, P, N);
            int32_t u = 0, v = 0;
            if (h) tex_coord(s.ents[k], P, u, v);
            else if (s.ents[k].kind >= EXP_QUAD && s.ents[k].kind <= EXP_CONE) { /* overwritten on miss too (:616-617) */ }
            else { P = {0, 0, 0}; N = {0, 0, 0}; }
            out_hit[j] = h ? 1 : 0;
            double* pn = out_pn + 6 * j;
            pn[0] = P.x; pn[1] = P.y; pn[2] = P.z; pn[3] = N.x; pn[4] = N.y; pn[5] = N.z;
            out_uv[2 * j] = u; out_uv[2 * j + 1] = v;
        }
    }
    return 0;
}

int gio_boxes(int n, const double* recs, int32_t* out) {
    for (int i = 0; i < n; ++i) {
        const double* q = recs + 12 * (size_t)i;
        out[i] = box_hit({q[0], q[1], q[2]}, {q[3], q[4], q[5]}, {q[6], q[7], q[8]},
                         normalize(V3{q[9], q[10], q[11]})) ? 1 : 0;
    }
    return 0;
}

}  // extern "C"
