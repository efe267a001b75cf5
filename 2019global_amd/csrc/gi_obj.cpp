// gi_obj.cpp — Wavefront OBJ text -> ImpTriangle entity descriptors (the optional
// OBJ loader for real meshes).  The reference has no scene files: main.cpp:24-48 pushes hand-built
// entities, and a mesh is a run of ImpTriangle(p1, p2, p3) (entities.h:138) pushes.  This turns an
// OBJ's faces into exactly such a run, so a loaded mesh goes through gi_scene_create (and the
// drop-in Octree::push_back) like any other entities.
//
// Accepted: `v x y z [...]` (a w or vertex colour after xyz is ignored), `f` with 3 or more vertex
// references in any of the forms i, i/t, i//n, i/t/n (1-based; negative = relative to the last
// vertex), fan-triangulated in face order (v0, v_k, v_k+1); `#` comments; blank lines; `\` line
// continuations.  Ignored (no reference counterpart): vt, vn, vp, o, g, s, usemtl, mtllib, l, p and
// unknown keywords.  Numbers follow one ASCII grammar (is_real below), parsed independently of the
// C locale.  scenes.load_obj restates these rules in Python (tests compare the two).
#include <charconv>
#include <cmath>
#include <system_error>
#include <cstring>
#include <string>
#include <vector>

#include "gi.h"
#include "gi_internal.h"

namespace {

// one logical line (continuations joined) split into whitespace-separated tokens
struct Tok {
    const char* p;
    size_t n;
};

// The one number grammar both parsers accept (scenes.load_obj restates it as a regex):
//   real    [+-]? ( D+ ( '.' D* )? | '.' D+ ) ( [eE] [+-]? D+ )?     D = ASCII 0-9
//   integer [+-]? D+
// Hex floats, inf / nan, digit separators and non-ASCII digits are malformed on both sides.
size_t scan_digits(const char* p, size_t i, size_t n) {
    while (i < n && p[i] >= '0' && p[i] <= '9') ++i;
    return i;
}
bool is_real(const char* p, size_t n) {
    size_t i = (n > 0 && (p[0] == '+' || p[0] == '-')) ? 1 : 0;
    const size_t d0 = i;
    i = scan_digits(p, i, n);
    const bool int_part = i > d0;
    bool frac_part = false;
    if (i < n && p[i] == '.') {
        const size_t f0 = ++i;
        i = scan_digits(p, i, n);
        frac_part = i > f0;
    }
    if (!int_part && !frac_part) return false;
    if (i < n && (p[i] == 'e' || p[i] == 'E')) {
        ++i;
        if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
        const size_t e0 = i;
        i = scan_digits(p, i, n);
        if (i == e0) return false;
    }
    return i == n;
}

// std::from_chars: correctly rounded like Python's float(), and independent of the C locale (the
// reference host is a Qt app: QApplication calls setlocale(LC_ALL, ""), so strtod would stop at
// the '.' of "1.5" under a comma-decimal locale such as de_DE)
// decimal exponent of the leading non-zero digit of a real token accepted by is_real (the value is
// in [10^e, 10^(e+1))); a large sentinel when every digit is zero
long long decimal_magnitude(const char* p, size_t n) {
    size_t i = (n > 0 && (p[0] == '+' || p[0] == '-')) ? 1 : 0;
    long long pos = 0;   // position of the leading non-zero digit relative to the point (0: units)
    bool found = false;
    long long int_digits = 0;
    for (; i < n && p[i] >= '0' && p[i] <= '9'; ++i) {
        if (!found && p[i] != '0') found = true;
        if (found) ++int_digits;
    }
    if (found) pos = int_digits - 1;
    if (i < n && p[i] == '.') {
        ++i;
        for (long long k = 1; i < n && p[i] >= '0' && p[i] <= '9'; ++i, ++k)
            if (!found && p[i] != '0') { found = true; pos = -k; }
    }
    if (!found) return 1ll << 40;
    long long e = 0;
    if (i < n && (p[i] == 'e' || p[i] == 'E')) {
        ++i;
        const bool neg = i < n && p[i] == '-';
        if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
        for (; i < n && p[i] >= '0' && p[i] <= '9'; ++i) e = std::min(e * 10 + (p[i] - '0'), 1ll << 40);
        if (neg) e = -e;
    }
    return pos + e;
}

bool parse_double(const Tok& t, double& v) {
    if (!is_real(t.p, t.n)) return false;
    const char* b = t.p + (t.p[0] == '+' ? 1 : 0);   // from_chars takes no leading '+'
    const std::from_chars_result r = std::from_chars(b, t.p + t.n, v);
    if (r.ec == std::errc::result_out_of_range && r.ptr == t.p + t.n && decimal_magnitude(t.p, t.n) < 0) {
        // underflow: the value rounds to a signed zero (from_chars reports it as out of range and
        // leaves v alone; Python's float() -- scenes.load_obj -- returns the zero)
        v = t.p[0] == '-' ? -0.0 : 0.0;
        return true;
    }
    return r.ec == std::errc() && r.ptr == t.p + t.n && std::isfinite(v);
}

bool parse_index(const Tok& t, long long& v) {
    size_t k = 0;
    while (k < t.n && t.p[k] != '/') ++k;   // the vertex index is the part before the first '/'
    size_t i = (k > 0 && (t.p[0] == '+' || t.p[0] == '-')) ? 1 : 0;
    if (scan_digits(t.p, i, k) != k || k == i) return false;
    const char* b = t.p + (t.p[0] == '+' ? 1 : 0);
    const std::from_chars_result r = std::from_chars(b, t.p + k, v, 10);
    return r.ec == std::errc() && r.ptr == t.p + k && v != 0;
}

}  // namespace

extern "C" int gi_obj_parse(const char* text, int64_t len, const gi_entity_desc* tmpl, gi_entity_desc* out, int64_t cap,
                            int64_t* n) {
    return gi::guard([&]() -> int {
        if (!text || len < 0 || !n || cap < 0 || (cap > 0 && !out)) return gi::error(GI_ERR_ARG, "bad arguments");
        std::vector<double> verts;   // xyz per vertex
        int64_t count = 0;
        std::vector<Tok> tok;
        std::string joined;          // a line with continuations, when there is one
        int64_t i = 0, lineno = 0;
        while (i < len) {
            // gather one logical line [a, b); a line ending in '\' continues on the next one
            joined.clear();
            bool cont = true, used_join = false;
            int64_t a = i, b = i;
            while (cont && i < len) {
                ++lineno;
                int64_t s = i;
                while (i < len && text[i] != '\n') ++i;
                int64_t e = i;
                if (i < len) ++i;                              // past '\n'
                if (e > s && text[e - 1] == '\r') --e;
                int64_t h = s;                                 // a comment ends the line
                while (h < e && text[h] != '#') ++h;
                cont = h == e && e > s && text[e - 1] == '\\';
                if (cont || used_join) {
                    used_join = true;
                    joined.append(text + s, (size_t)((cont ? e - 1 : h) - s));
                    joined.push_back(' ');
                } else {
                    a = s;
                    b = h;
                }
            }
            const char* base = used_join ? joined.data() : text + a;
            const size_t m = used_join ? joined.size() : (size_t)(b - a);
            tok.clear();
            for (size_t k = 0; k < m;) {
                while (k < m && (base[k] == ' ' || base[k] == '\t' || base[k] == '\r')) ++k;
                size_t s = k;
                while (k < m && !(base[k] == ' ' || base[k] == '\t' || base[k] == '\r')) ++k;
                if (k > s) tok.push_back(Tok{base + s, k - s});
            }
            if (tok.empty()) continue;
            const std::string kw(tok[0].p, tok[0].n);
            if (kw == "v") {
                if (tok.size() < 4)   // x y z, then an optional w or vertex colour (ignored)
                    return gi::error(GI_ERR_ARG, "obj line " + std::to_string(lineno) + ": v needs 3 coordinates");
                for (int k = 1; k <= 3; ++k) {
                    double v;
                    if (!parse_double(tok[k], v))
                        return gi::error(GI_ERR_ARG, "obj line " + std::to_string(lineno) + ": bad coordinate");
                    verts.push_back(v);
                }
            } else if (kw == "f") {
                if (tok.size() < 4)
                    return gi::error(GI_ERR_ARG, "obj line " + std::to_string(lineno) + ": a face needs 3 vertices");
                const long long nv = (long long)(verts.size() / 3);
                long long idx[3] = {0, 0, 0};
                for (size_t k = 1; k < tok.size(); ++k) {
                    long long r;
                    if (!parse_index(tok[k], r))
                        return gi::error(GI_ERR_ARG, "obj line " + std::to_string(lineno) + ": bad vertex reference");
                    const long long z = r > 0 ? r - 1 : nv + r;   // 1-based, or relative to the last vertex
                    if (z < 0 || z >= nv)
                        return gi::error(GI_ERR_ARG, "obj line " + std::to_string(lineno) + ": vertex " +
                                                         std::to_string(r) + " out of range");
                    if (k == 1) { idx[0] = z; continue; }
                    idx[1] = idx[2];
                    idx[2] = z;
                    if (k < 3) continue;
                    if (count < cap) {   // ImpTriangle(v0, v_{k-1}, v_k): the fan in face order
                        gi_entity_desc& d = out[count];
                        if (tmpl) d = *tmpl; else std::memset(&d, 0, sizeof d);
                        d.kind = GI_IMP_TRIANGLE;
                        for (int c = 0; c < 11; ++c) d.args[c] = 0.0;
                        for (int t = 0; t < 3; ++t)
                            for (int c = 0; c < 3; ++c) d.args[3 * t + c] = verts[(size_t)(3 * idx[t] + c)];
                    }
                    ++count;
                }
            }
            // vt, vn, vp, o, g, s, usemtl, mtllib, l, p, ...: no reference counterpart, skipped
        }
        *n = count;
        return GI_OK;
    });
}
