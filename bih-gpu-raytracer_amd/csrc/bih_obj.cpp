// bih_obj.cpp -- Wavefront OBJ scene ingestion behind the C ABI (host code).
//
// Replaces the reference's assimp path for the one format it loads
// ("resources/<name>/<name>.obj", src/Main.cpp:55-63):
//   Model::LoadModel / ProcessNode / ProcessMesh   src/Model.cpp:10-95
//   App::LoadModels triangle flattening            src/App.cpp:65-121
// The reference calls Assimp::Importer::ReadFile(path, aiProcess_Triangulate |
// ... | aiProcess_SortByPType) (Model.cpp:13) and then walks
// model -> meshes -> indices in steps of 3.  For an OBJ file assimp (5.0, the
// vendored headers under src/assimp) appends a new mesh every time the group,
// object or material changes, and the node walk visits them in creation
// order, so the flattened soup is every triangle in FILE ORDER.  What this
// file restates from assimp's published algorithm:
//   * vertex coordinates parsed with fast_atoreal_move<float>
//     (src/assimp/fast_atof.h:259-344): integer part through uint64 -> float,
//     at most 15 fraction digits as double * 10^-k, rounded to float and added
//     in float, an optional exponent applied as f *= powf(10, e); ',' is
//     accepted as the decimal point;
//   * `v x y z w` is stored as (x/w, y/w, z/w) (homogeneous vertex);
//   * face indices are 1-based, negative ones count back from the current
//     vertex count, 0 or out of range is an error;
//   * aiProcess_Triangulate: a triangle is kept, a quad is split into two
//     triangles fanned from its (at most one) concave vertex -- the first i
//     whose angles acos(l.d) + acos(r.d) of the normalised edges to its
//     neighbours and its diagonal exceed pi -- else from vertex 0.
// Differences, stated: polygons with more than 4 vertices are fanned from
// vertex 0 (assimp ear-clips them; identical for convex polygons up to the
// triangle order); points and lines (`p`, `l`, one- and two-index faces) are
// dropped (with SortByPType they become separate meshes whose index lists the
// reference would misread as triangles).  No golden OBJ ships with the
// reference (resources/sponza holds only the .mtl and textures), so exact
// parity with assimp's output is unpinned; the tests pin this loader against
// oracle/obj_oracle.py, a Python restatement of the same rules.
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <vector>

#include "../../include/bih.h"

namespace {

// fast_atoreal_move<float> (fast_atof.h:259-344), returns false on a token
// that does not start with a digit or a decimal point followed by a digit.
bool parse_real(const char *&c, float &out) {
    static const double frac_scale[16] = {0.0, 1e-1, 1e-2, 1e-3, 1e-4, 1e-5, 1e-6, 1e-7,
                                          1e-8, 1e-9, 1e-10, 1e-11, 1e-12, 1e-13, 1e-14, 1e-15};
    auto isdig = [](char ch) { return ch >= '0' && ch <= '9'; };
    auto is_point = [](char ch) { return ch == '.' || ch == ','; };
    // uint64 accumulation like strtoul10_64 (fast_atof.h:185-232); on overflow
    // it returns 0 (and leaves the pointer where it was)
    bool overflow = false;
    auto digits = [&](const char *&p, unsigned max_digits, unsigned *taken) -> uint64_t {
        uint64_t v = 0;
        unsigned n = 0;
        while (isdig(*p)) {
            const uint64_t nv = v * 10u + (uint64_t)(*p - '0');
            if (nv < v) {
                overflow = true;
                return 0;
            }
            v = nv;
            ++p;
            ++n;
            if (max_digits && n == max_digits) {
                while (isdig(*p)) ++p;
                break;
            }
        }
        if (taken) *taken = n;
        return v;
    };
    bool neg = (*c == '-');
    if (neg || *c == '+') ++c;
    if (strncasecmp(c, "nan", 3) == 0) {
        out = NAN;
        c += 3;
        return true;
    }
    if (strncasecmp(c, "inf", 3) == 0) {
        c += 3;
        if (strncasecmp(c, "inity", 5) == 0) c += 5;
        out = neg ? -INFINITY : INFINITY;
        return true;
    }
    if (!isdig(c[0]) && !(is_point(c[0]) && isdig(c[1]))) return false;
    float f = 0.0f;
    if (!is_point(*c)) {
        f = (float)digits(c, 0, nullptr);
        if (overflow) {
            // strtoul10_64 overflowed: it returns 0 without advancing, so the
            // rest of the word is never parsed
            while (*c && *c != ' ' && *c != '\t' && *c != '\r') ++c;
            out = neg ? -0.0f : 0.0f;
            return true;
        }
    }
    if (is_point(c[0]) && isdig(c[1])) {
        ++c;
        unsigned k = 0;
        double pl = (double)digits(c, 15, &k);
        pl *= frac_scale[k];
        f += (float)pl;
    } else if (*c == '.') {
        ++c;   // trailing dot
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        bool eneg = (*c == '-');
        if (eneg || *c == '+') ++c;
        if (!isdig(*c)) return false;
        float e = (float)digits(c, 0, nullptr);
        if (eneg) e = -e;
        f *= powf(10.0f, e);
    }
    out = neg ? -f : f;
    return true;
}

bool parse_int(const char *&c, long &out) {
    bool neg = (*c == '-');
    if (neg || *c == '+') ++c;
    if (*c < '0' || *c > '9') return false;
    long v = 0;
    while (*c >= '0' && *c <= '9') {
        v = v * 10 + (*c - '0');
        if (v > (1L << 40)) return false;
        ++c;
    }
    out = neg ? -v : v;
    return true;
}

void skip_ws(const char *&c) {
    while (*c == ' ' || *c == '\t' || *c == '\r') ++c;
}

struct V3 {
    float x, y, z;
};

V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 normalized(V3 a) {   // aiVector3t::Normalize: *this /= Length()
    const float l = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return {a.x / l, a.y / l, a.z / l};
}
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// aiProcess_Triangulate on a quad: fan from the concave vertex, if any
unsigned quad_start(const std::vector<V3> &pos, const long q[4]) {
    const float pi = 3.1415926538f;   // AI_MATH_PI_F
    for (unsigned i = 0; i < 4; ++i) {
        const V3 v = pos[q[i]];
        const V3 left = normalized(sub(pos[q[(i + 3) % 4]], v));
        const V3 diag = normalized(sub(pos[q[(i + 2) % 4]], v));
        const V3 right = normalized(sub(pos[q[(i + 1) % 4]], v));
        const float angle = acosf(dot(left, diag)) + acosf(dot(right, diag));
        if (angle > pi) return i;
    }
    return 0;
}

}  // namespace

extern "C" int bih_scene_load_obj(const char *path, bih_scene *out, uint32_t *err_line) {
    if (err_line) *err_line = 0;
    if (!path || !out) return BIH_ERR_INVALID;
    out->n_tris = 0;
    out->v = nullptr;
    FILE *fp = fopen(path, "rb");
    if (!fp) return BIH_ERR_IO;
    std::vector<V3> pos;
    std::vector<float> soup;
    std::vector<long> face;
    std::vector<char> line(1 << 12);
    uint32_t lineno = 0;
    int rc = BIH_OK;
    auto emit = [&](long a, long b, long c) {
        for (long k : {a, b, c}) {
            soup.push_back(pos[k].x);
            soup.push_back(pos[k].y);
            soup.push_back(pos[k].z);
        }
    };
    for (;;) {
        // read one physical line of any length
        size_t len = 0;
        int ch;
        while ((ch = getc_unlocked(fp)) != EOF && ch != '\n') {
            if (len + 1 >= line.size()) line.resize(line.size() * 2);
            line[len++] = (char)ch;
        }
        if (ch == EOF && len == 0) break;
        line[len] = 0;
        ++lineno;
        const char *c = line.data();
        skip_ws(c);
        if (c[0] == 'v' && (c[1] == ' ' || c[1] == '\t')) {
            c += 2;
            float x[6];
            int n = 0;
            for (;;) {
                skip_ws(c);
                if (!*c || *c == '#') break;
                if (n == 6 || !parse_real(c, x[n])) {
                    n = -1;
                    break;
                }
                ++n;
                if (*c && *c != ' ' && *c != '\t' && *c != '\r') {
                    n = -1;
                    break;
                }
            }
            if (n == 3 || n == 6) {
                pos.push_back({x[0], x[1], x[2]});   // 6: x y z r g b, colour ignored
            } else if (n == 4) {
                if (x[3] == 0.0f) {
                    rc = BIH_ERR_PARSE;
                    break;
                }
                pos.push_back({x[0] / x[3], x[1] / x[3], x[2] / x[3]});
            } else {
                rc = BIH_ERR_PARSE;
                break;
            }
        } else if (c[0] == 'f' && (c[1] == ' ' || c[1] == '\t')) {
            c += 2;
            face.clear();
            for (;;) {
                skip_ws(c);
                if (!*c || *c == '#') break;
                long idx;
                if (!parse_int(c, idx) || idx == 0) {
                    rc = BIH_ERR_PARSE;
                    break;
                }
                const long nv = (long)pos.size();
                const long k = idx > 0 ? idx - 1 : nv + idx;
                if (k < 0 || k >= nv) {
                    rc = BIH_ERR_PARSE;
                    break;
                }
                face.push_back(k);
                // v/vt/vn, v//vn: texture and normal indices are not needed
                while (*c && *c != ' ' && *c != '\t' && *c != '\r') ++c;
            }
            if (rc != BIH_OK) break;
            const size_t m = face.size();
            if (m == 3) {
                emit(face[0], face[1], face[2]);
            } else if (m == 4) {
                const long q[4] = {face[0], face[1], face[2], face[3]};
                const unsigned s = quad_start(pos, q);
                emit(q[s], q[(s + 1) % 4], q[(s + 2) % 4]);
                emit(q[s], q[(s + 2) % 4], q[(s + 3) % 4]);
            } else if (m > 4) {
                for (size_t i = 1; i + 1 < m; ++i) emit(face[0], face[i], face[i + 1]);
            }
            // m < 3: point / line primitive, dropped
        }
        // vt, vn, g, o, s, usemtl, mtllib, l, p, comments: no triangles
        if (ch == EOF) break;
    }
    fclose(fp);
    if (rc != BIH_OK) {
        if (err_line) *err_line = lineno;
        return rc;
    }
    const size_t n = soup.size() / 9;
    if (n > BIH_MAX_TRIS) return BIH_ERR_TOO_LARGE;
    if (n == 0) return BIH_OK;
    float *v = (float *)malloc(soup.size() * sizeof(float));
    if (!v) return BIH_ERR_OOM;
    memcpy(v, soup.data(), soup.size() * sizeof(float));
    out->n_tris = (uint32_t)n;
    out->v = v;
    return BIH_OK;
}

extern "C" void bih_scene_free(bih_scene *scene) {
    if (!scene) return;
    free((void *)scene->v);
    scene->v = nullptr;
    scene->n_tris = 0;
}
