// rt_oracle.cpp — CPU restatement of the reference ray tracer (see rt_oracle.h).
// TEST INFRASTRUCTURE ONLY. Compile with -ffp-contract=off (oracle/Makefile):
// every float expression below must round exactly like the reference's.
#include "rt_oracle.h"

#include <atomic>
#include <chrono>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <immintrin.h>

// The oracle's own JSON reader (independent of the product's json_min.h).
#include "ora_json.h"

namespace ora {

static const double kPI = 3.14159265;          // Raytracer.h:11
static const double kEPS = 1e-6;               // Raytracer.h:12
static const float kOFFSET = (float)0.2;       // SHADOW_CLIPPING_OFFSET, Raytracer.h:13 (used as float arg)

// 0: hoisted (ray-invariant triangle data computed once per load; the default);
// 1: ref-faithful cost model (oracle_set_mode; for the CPU baseline).
static int g_faithful = 0;
// per thread: a shared sink written per triangle test would bounce one cache line
// between the CPU baseline's threads (ref-faithful mode)
static thread_local volatile float g_sink;
// 16-wide hoisted triangle scan where the CPU has AVX-512 (Tracer::scan_avx512;
// $ORACLE_SCALAR=1: the scalar loop). Same bits either way.
static const bool g_avx512 = __builtin_cpu_supports("avx512f") && !(std::getenv("ORACLE_SCALAR") && std::atoi(std::getenv("ORACLE_SCALAR")));
// kEPS compared with a float (Raytracer.cpp:16-18 NearlyEquals, :376 t <= EPSILON)
static const float kEPSf = (float)1e-6 < 1e-6 ? (float)1e-6 : std::nextafter((float)1e-6, 0.0f);

// ---------------------------------------------------------------- Vector3 (Raytracer.h:39-149)
struct V3 {
    float x = 0, y = 0, z = 0;
    V3() {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    V3 operator*(float s) const { return {x * s, y * s, z * s}; }
    V3 operator*(const V3& o) const { return {x * o.x, y * o.y, z * o.z}; }
    V3 operator-(const V3& o) const { return {x - o.x, y - o.y, z - o.z}; }
    V3 operator+(const V3& o) const { return {x + o.x, y + o.y, z + o.z}; }
    V3 operator-() const { return {-x, -y, -z}; }
    void normalize() {  // Raytracer.h:109-116
        float len = std::sqrt(x * x + y * y + z * z);
        if (len > 0) { x /= len; y /= len; z /= len; }
    }
    float length() const { return std::sqrt(x * x + y * y + z * z); }
    static V3 cross(const V3& a, const V3& b) {
        return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    }
    float dot(const V3& o) const { return x * o.x + y * o.y + z * o.z; }
    static V3 reflect(const V3& I, const V3& N) {  // Raytracer.h:143-148
        float d = I.dot(N);
        d *= 2;
        return I - N * d;
    }
};

// ---------------------------------------------------------------- Matrix (Raytracer.h:168-371)
struct M4 {
    float m[4][4];
    M4 operator*(const M4& o) const {
        M4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                r.m[i][j] = 0;
                for (int k = 0; k < 4; ++k) r.m[i][j] += m[i][k] * o.m[k][j];
            }
        return r;
    }
    V3 translation() const { return {m[0][3], m[1][3], m[2][3]}; }
    V3 xform_dir(const V3& d) const {
        return {m[0][0] * d.x + m[0][1] * d.y + m[0][2] * d.z,
                m[1][0] * d.x + m[1][1] * d.y + m[1][2] * d.z,
                m[2][0] * d.x + m[2][1] * d.y + m[2][2] * d.z};
    }
    V3 xform_point(const V3& p) const {  // Raytracer.h:234-248
        float x = m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3];
        float y = m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3];
        float z = m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3];
        float w = m[3][0] * p.x + m[3][1] * p.y + m[3][2] * p.z + m[3][3];
        if (w != 1.0f) { x /= w; y /= w; z /= w; }
        return {x, y, z};
    }
    static void identity(M4& a) {  // LoadIdentityMatrix, Raytracer.cpp:872-878
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) a.m[i][j] = (i == j) ? 1.0f : 0.0f;
    }
    static float det3(const M4& a) {  // Raytracer.h:251-255
        return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
               a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
               a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
    }
    static float det4(const M4& a) {  // Raytracer.h:257-274
        float det = 0;
        for (int i = 0; i < 4; i++) {
            M4 sub;  // uninitialised, as the reference's Matrix (no constructor); det3 reads the written 3x3
            for (int j = 1; j < 4; j++)
                for (int k = 0; k < 4; k++) {
                    if (k < i) sub.m[j - 1][k] = a.m[j][k];
                    else if (k > i) sub.m[j - 1][k - 1] = a.m[j][k];
                }
            det += (i % 2 == 0 ? 1 : -1) * a.m[0][i] * det3(sub);
        }
        return det;
    }
    static void adjoint(const M4& a, M4& adj) {  // Raytracer.h:276-296 (transposed cofactors)
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                M4 sub;
                int si = 0;
                for (int k = 0; k < 4; k++) {
                    if (k == i) continue;
                    int sj = 0;
                    for (int l = 0; l < 4; l++) {
                        if (l == j) continue;
                        sub.m[si][sj] = a.m[k][l];
                        sj++;
                    }
                    si++;
                }
                float c = det3(sub);
                if ((i + j) % 2 != 0) c = -c;
                adj.m[j][i] = c;
            }
    }
    static bool inverse(const M4& a, M4& r) {  // Raytracer.h:354-370
        float det = det4(a);
        if (std::fabs(det) < 1e-10) return false;
        M4 adj;
        adjoint(a, adj);
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) r.m[i][j] = adj.m[i][j] / det;
        return true;
    }
};

// ---------------------------------------------------------------- Pixel (Raytracer.h:373-418)
// static_cast<short>(float) as g++ emits it on x86-64: cvttss2si to int32
// (NaN / out of range -> INT32_MIN), then the low 16 bits.
static inline short f2s(float f) {
    int32_t i;
    if (!(f > -2147483904.0f && f < 2147483648.0f)) i = INT32_MIN;
    else i = (int32_t)f;
    return (short)(uint16_t)(uint32_t)i;
}
struct Pix {
    short r = 0, g = 0, b = 0;
    Pix() {}
    Pix(short a, short c, short d) : r(a), g(c), b(d) {}
    explicit Pix(const V3& v) : r(f2s(v.x * 255)), g(f2s(v.y * 255)), b(f2s(v.z * 255)) {}  // clamp() result discarded (:380)
    Pix clamp() const {
        Pix o;
        o.r = r > 255 ? 255 : (r < 0 ? 0 : r);
        o.g = g > 255 ? 255 : (g < 0 ? 0 : g);
        o.b = b > 255 ? 255 : (b < 0 ? 0 : b);
        return o;
    }
    Pix operator*(float s) const { return Pix(f2s(r * s), f2s(g * s), f2s(b * s)).clamp(); }
    Pix operator+(const Pix& o) const { return Pix((short)(r + o.r), (short)(g + o.g), (short)(b + o.b)); }
};

// ---------------------------------------------------------------- scene
struct Material {  // Raytracer.h:442-463
    V3 cs{1, 1, 1};
    float ka = 0.5f, kd = 0.75f, ks = 0.95f, kt = 0.95f, ior = 2.5f, n = 32.0f;
};
struct Tri { V3 p[3], nrm[3]; };
struct Mesh { int type = 0; std::vector<Tri> tris; float radius = 0; };  // value-initialised (:605)
// The ray-invariant part of IntersectTriangle (Raytracer.cpp:353-365, :377, :389,
// :403) for one triangle of one shape: world vertices, normal, plane offset,
// signed area, hit normal. Computed once with the same float operations, so
// the hoisted test rounds exactly like the per-call one.
struct WTri { V3 v0, v1, v2, N, hn; float D, area; };
// The same values in structure-of-arrays form, padded to a multiple of 16
// with N = 0 (nd = 0: rejected), for the 16-wide scan (scan_avx512).
struct WTriSoA {
    size_t n = 0;  // padded count
    std::vector<float> v0x, v0y, v0z, v1x, v1y, v1z, v2x, v2y, v2z, nx, ny, nz, d, area;
};
struct Shape {
    Material mat;
    V3 S{1, 1, 1}, R, T;
    int mesh = -1;
    std::string geo;  // geometryId (meshMap key, Raytracer.cpp:477)
    M4 model;
    std::vector<WTri> wtris;
    WTriSoA soa;
};
struct Light { int type = -1; V3 color, position, direction; float intensity = 0; };
enum { LDIR = 0, LPOINT = 1, LAMB = 2 };
struct Camera { V3 from, to; };
struct Scene {
    std::vector<Shape> shapes;
    std::vector<Mesh> meshes;
    std::unordered_map<std::string, int> mesh_by_name;  // meshMap (Raytracer.h:552)
    std::vector<Light> lights;
    Camera cam;
};

static std::string read_file(const std::string& p, bool& ok) {
    std::ifstream f(p, std::ios::binary);
    ok = f.is_open();
    std::stringstream ss;
    if (ok) ss << f.rdbuf();
    return ss.str();
}

static float ToRadian(float deg) { return (float)(deg * (kPI / 180)); }  // Raytracer.h:581-583

// ComputeModelMatrix, Raytracer.cpp:528-586. g++ merges cos/sin of one
// argument into glibc sincos (checked in the reference binary), so do we.
static M4 model_matrix(const Shape& s) {
    M4 S, RX, RY, RZ, T;
    M4::identity(S);
    S.m[0][0] = s.S.x; S.m[1][1] = s.S.y; S.m[2][2] = s.S.z; S.m[3][3] = 1.0f;
    double sx, cx, sy, cy, sz, cz;
    ::sincos((double)ToRadian(s.R.x), &sx, &cx);
    ::sincos((double)ToRadian(s.R.y), &sy, &cy);
    ::sincos((double)ToRadian(s.R.z), &sz, &cz);
    M4::identity(RX);
    RX.m[1][1] = (float)cx; RX.m[1][2] = (float)-sx; RX.m[2][1] = (float)sx; RX.m[2][2] = (float)cx;
    M4::identity(RY);
    RY.m[0][0] = (float)cy; RY.m[0][2] = (float)sy; RY.m[2][0] = (float)-sy; RY.m[2][2] = (float)cy;
    M4::identity(RZ);
    RZ.m[0][0] = (float)cz; RZ.m[0][1] = (float)-sz; RZ.m[1][0] = (float)sz; RZ.m[1][1] = (float)cz;
    M4 R = RZ * RY * RX;
    M4::identity(T);
    T.m[0][3] = s.T.x; T.m[1][3] = s.T.y; T.m[2][3] = s.T.z;
    return S * R * T;
}

// IntersectTriangle's ray-invariant values (Raytracer.cpp:353-365, :377, :389,
// :403, :937-942), in the reference's operation order.
static void hoist_triangles(Shape& s, const Mesh& m) {
    s.wtris.resize(m.tris.size());
    for (size_t i = 0; i < m.tris.size(); i++) {
        WTri& w = s.wtris[i];
        w.v0 = s.model.xform_point(m.tris[i].p[0]);
        w.v1 = s.model.xform_point(m.tris[i].p[1]);
        w.v2 = s.model.xform_point(m.tris[i].p[2]);
        V3 e1 = w.v1 - w.v0, e2 = w.v2 - w.v0;
        w.N = V3::cross(e1, e2);
        w.N.normalize();
        w.D = -w.N.dot(w.v0);
        V3 ab = w.v1 - w.v0, ac = w.v2 - w.v0;
        w.area = (float)(0.5 * V3::cross(ab, ac).dot(w.N));
        w.hn = w.N;
        w.hn.normalize();
    }
    WTriSoA& a = s.soa;
    a.n = (s.wtris.size() + 15) / 16 * 16;
    for (auto* v : {&a.v0x, &a.v0y, &a.v0z, &a.v1x, &a.v1y, &a.v1z, &a.v2x, &a.v2y, &a.v2z, &a.nx, &a.ny, &a.nz, &a.d,
                    &a.area})
        v->assign(a.n, 0.0f);
    for (size_t i = 0; i < s.wtris.size(); i++) {
        const WTri& w = s.wtris[i];
        a.v0x[i] = w.v0.x; a.v0y[i] = w.v0.y; a.v0z[i] = w.v0.z;
        a.v1x[i] = w.v1.x; a.v1y[i] = w.v1.y; a.v1z[i] = w.v1.z;
        a.v2x[i] = w.v2.x; a.v2y[i] = w.v2.y; a.v2z[i] = w.v2.z;
        a.nx[i] = w.N.x; a.ny[i] = w.N.y; a.nz[i] = w.N.z;
        a.d[i] = w.D; a.area[i] = w.area;
    }
}

static V3 vec3(const ora_json::Node& a) { return {a[0].f(), a[1].f(), a[2].f()}; }

// LoadMesh, Raytracer.cpp:589-643
static int load_mesh(Scene& sc, std::map<std::string, int>& cache, const std::string& root,
                     const std::string& name, int& idx) {
    auto it = cache.find(name);
    if (it != cache.end()) { idx = it->second; return 0; }
    bool ok;
    std::string text = read_file(root + "/Assets/" + name + ".json", ok);
    if (!ok) { std::fprintf(stderr, "oracle: mesh %s not found\n", name.c_str()); idx = -1; return 1; }
    auto doc = ora_json::read(text);
    const ora_json::Node& j = *doc;
    Mesh mesh;
    std::string type = j["data"][0]["type"].s();  // the type of data[0] only (:606)
    for (const ora_json::Node* item : j["data"].each()) {
        if (type == "polygon") {
            mesh.type = 0;
            Tri t;
            for (int i = 0; i < 3; i++) {
                const ora_json::Node& v = (*item)["v" + std::to_string(i)];
                t.p[i] = vec3(v["v"]);
                t.nrm[i] = vec3(v["n"]);
                (void)v["t"][0].f(); (void)v["t"][1].f();
            }
            mesh.tris.push_back(t);
        } else if (type == "sphere") {
            mesh.type = 1;
            mesh.radius = (*item)["radius"].f();
        }
    }
    sc.meshes.push_back(mesh);
    idx = (int)sc.meshes.size() - 1;
    cache[name] = idx;
    sc.mesh_by_name[name] = idx;
    return 0;
}

// LoadSceneJSON, Raytracer.cpp:645-779
static int load_scene(Scene& sc, const std::string& root, const std::string& path) {
    bool ok;
    std::string text = read_file(root + "/Assets/" + path, ok);
    if (!ok) { std::fprintf(stderr, "oracle: cannot open %s\n", path.c_str()); return 1; }
    int status = 0;
    try {
        auto doc = ora_json::read(text);
        const ora_json::Node& j = *doc;
        // jsonData["scene"] on the non-const document (:667): absent -> null, so
        // no shapes, camera or lights; a null document becomes an object there,
        // any other non-object document is a type error
        if (j.t != ora_json::Node::OBJ && j.t != ora_json::Node::NUL)
            throw std::runtime_error("document is not an object");
        static const ora_json::Node kNull;
        const ora_json::Node& s = j.has("scene") ? j["scene"] : kNull;
        std::map<std::string, int> cache;
        if (s.has("shapes"))
            for (const ora_json::Node* sv : s["shapes"].each()) {
                Shape shp;
                (void)(*sv)["id"].s();
                std::string geo = (*sv)["geometry"].s();
                shp.geo = geo;
                if (sv->has("notes")) (void)(*sv)["notes"].s();  // get<std::string>() (:673-675)
                const ora_json::Node& m = (*sv)["material"];
                shp.mat.cs = vec3(m["Cs"]);
                shp.mat.ka = m["Ka"].f();
                shp.mat.kd = m["Kd"].f();
                shp.mat.ks = m["Ks"].f();
                shp.mat.kt = m["Kt"].f();
                shp.mat.n = m["n"].f();
                for (const ora_json::Node* t : (*sv)["transforms"].each()) {
                    if (t->has("Rx")) shp.R.x = (*t)["Rx"].f();
                    if (t->has("Ry")) shp.R.y = (*t)["Ry"].f();
                    if (t->has("Rz")) shp.R.z = (*t)["Rz"].f();
                    if (t->has("S") && (*t)["S"].t == ora_json::Node::ARR) shp.S = vec3((*t)["S"]);
                    if (t->has("T") && (*t)["T"].t == ora_json::Node::ARR) shp.T = vec3((*t)["T"]);
                }
                status |= load_mesh(sc, cache, root, geo, shp.mesh);
                shp.model = model_matrix(shp);
                if (shp.mesh >= 0 && sc.meshes[shp.mesh].type == 0) hoist_triangles(shp, sc.meshes[shp.mesh]);
                sc.shapes.push_back(shp);
            }
        if (s.has("camera")) {
            const ora_json::Node& c = s["camera"];
            sc.cam.from = vec3(c["from"]);
            sc.cam.to = vec3(c["to"]);
            for (int i = 0; i < 6; i++) (void)c["bounds"][i].f();
            (void)c["resolution"][0].i(); (void)c["resolution"][1].i();
        }
        if (s.has("lights"))
            for (const ora_json::Node* lv : s["lights"].each()) {
                Light l;
                l.color = vec3((*lv)["color"]);
                l.intensity = (*lv)["intensity"].f();
                std::string t = (*lv)["type"].s();
                if (t == "directional") {
                    V3 from = vec3((*lv)["from"]), to = vec3((*lv)["to"]);
                    l.direction = to - from;
                    l.direction.normalize();
                    l.type = LDIR;
                } else if (t == "ambient") {
                    l.type = LAMB;
                } else if (t == "point") {
                    l.type = LPOINT;
                    l.position = vec3((*lv)["position"]);
                } else {
                    std::fprintf(stderr, "oracle: unsupported light type %s\n", t.c_str());
                    return 1;  // reference: lightType left uninitialised (UB)
                }
                sc.lights.push_back(l);
            }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle: scene error: %s\n", e.what());
        return 1;
    }
    return status;
}

// ---------------------------------------------------------------- RNG (member mGenerator, Raytracer.h:592)
// libstdc++ 11: minstd_rand0 = linear_congruential_engine<uint_fast32_t,16807,0,2^31-1>, seed 1;
// uniform_real_distribution<float>::operator() = generate_canonical<float,24>() * (b-a) + a
// (random.h, random.tcc:3348-3378). MSVC: mt19937, seed 5489.
struct DrawSource {
    int engine = 0;
    std::vector<uint32_t> stream;  // engine 1: pre-generated outputs [lo, lo + size)
    uint64_t lo = 0;
    static uint64_t mulmod(uint64_t a, uint64_t b) { return (a * b) % 2147483647ull; }
    static uint64_t powmod(uint64_t a, uint64_t e) {
        uint64_t r = 1;
        while (e) { if (e & 1) r = mulmod(r, a); a = mulmod(a, a); e >>= 1; }
        return r;
    }
};
struct RngCursor {  // one thread's position in the global draw stream
    const DrawSource* src;
    uint64_t index = 0;  // draws consumed so far
    uint64_t state = 1;  // minstd state after `index` draws
    void seek(uint64_t k) {
        index = k;
        if (src->engine == 0) state = DrawSource::powmod(16807, k % 2147483646ull);
    }
    float canonical() {
        float ret;
        if (src->engine == 0) {
            state = (state * 16807ull) % 2147483647ull;
            ret = (float)(unsigned long)(state - 1) / 2147483648.0f;
        } else {
            uint32_t x = src->stream[index - src->lo];
            ret = (float)(unsigned long)x / 4294967296.0f;
        }
        index++;
        if (ret >= 1.0f) ret = std::nextafter(1.0f, 0.0f);
        return ret;
    }
    float uniform(float a, float b) { return canonical() * (b - a) + a; }
};

// ---------------------------------------------------------------- tracer
struct Ray {
    V3 o, d;
    Ray() {}
    Ray(const V3& origin, const V3& dir) : o(origin), d(dir) { d.normalize(); }  // Raytracer.h:431-433
};
struct Hit {
    int type = 0;
    V3 p, n;
    float t = 0;
    const Tri* tri = nullptr;
    const Material* mat = nullptr;
    float a = 0, b = 0, g = 0;
};
struct Counters { uint64_t primary = 0, secondary = 0, shadow = 0, ao = 0, ao_calls = 0, tree_hits = 0; };

struct Tracer {
    const Scene* sc;
    int depth, ao_n, ao_on, n_amb;
    float ao_bmax;  // (float)(2 * PI)

    static float CalcArea(const V3& A, const V3& B, const V3& C, const V3& N) {  // Raytracer.cpp:937-942
        V3 ab = B - A, ac = C - A;
        V3 c = V3::cross(ab, ac);
        return (float)(0.5 * c.dot(N));
    }
    // IntersectTriangle, Raytracer.cpp:348-409 (world vertices from the cached model matrix)
    static bool tri_hit(const Ray& r, const Tri& tri, const M4& M, Hit& h) {
        V3 v0 = M.xform_point(tri.p[0]), v1 = M.xform_point(tri.p[1]), v2 = M.xform_point(tri.p[2]);
        V3 e1 = v1 - v0, e2 = v2 - v0;
        V3 N = V3::cross(e1, e2);
        N.normalize();
        float nd = N.dot(r.d);
        if (std::abs(nd - 0.0f) < kEPS) return false;  // NearlyEquals, Raytracer.cpp:16-18
        float D = -N.dot(v0);
        float t = -(N.dot(r.o) + D) / nd;
        if (t <= kEPS) return false;
        V3 P = r.o + r.d * t;
        float area = CalcArea(v0, v1, v2, N);
        float a = CalcArea(P, v1, v2, N) / area;
        float b = CalcArea(v0, P, v2, N) / area;
        float g = CalcArea(v0, v1, P, N) / area;
        if (a < 0 || b < 0 || g < 0) return false;
        h.p = P; h.type = 0; h.n = N; h.n.normalize(); h.t = t; h.a = a; h.b = b; h.g = g;
        return true;
    }
    // IntersectSphere, Raytracer.cpp:419-464
    static bool sph_hit(const Ray& r, float radius, const M4& M, Hit& h) {
        V3 oc = r.o - M.translation();
        float b = 2.0f * r.d.dot(oc);
        float c = oc.dot(oc) - (radius * radius);
        float disc = (b * b) - (4 * 1.0f * c);
        if (disc < kEPS) return false;
        float sq = std::sqrt(disc);
        float t0 = (-b + sq) / (float)2, t1 = (-b - sq) / (float)2;
        bool g0 = t0 > kEPS, g1 = t1 > kEPS;
        if (!g0 && !g1) return false;
        if (!g0) h.t = t1;
        else if (!g1) h.t = t0;
        else h.t = std::fmin(t0, t1);
        h.p = r.o + (r.d * h.t);
        h.n = h.p - M.translation();
        h.n.normalize();
        h.type = 1;
        return true;
    }
    // The same test on the hoisted record (WTri): identical operations on
    // identical values from `nd` on.
    static bool wtri_hit(const Ray& r, const WTri& w, Hit& h) {
        float nd = w.N.dot(r.d);
        if (std::abs(nd - 0.0f) < kEPS) return false;
        float t = -(w.N.dot(r.o) + w.D) / nd;
        if (t <= kEPS) return false;
        V3 P = r.o + r.d * t;
        float a = CalcArea(P, w.v1, w.v2, w.N) / w.area;
        float b = CalcArea(w.v0, P, w.v2, w.N) / w.area;
        float g = CalcArea(w.v0, w.v1, P, w.N) / w.area;
        if (a < 0 || b < 0 || g < 0) return false;
        h.p = P; h.type = 0; h.n = w.hn; h.t = t; h.a = a; h.b = b; h.g = g;
        return true;
    }
    // IntersectScene, Raytracer.cpp:473-526. any = true: only the boolean is
    // wanted (AO samples :323, directional shadow rays :73), so the first hit
    // decides; the closest-hit rule (first found, later ones only if strictly
    // closer) is kept otherwise.
    bool intersect(const Ray& r, Hit& out, bool any = false) const {
        if (g_faithful) return intersect_faithful(r, out);
        Hit best;
        bool found = false;
        for (const Shape& s : sc->shapes) {
            const Mesh& m = sc->meshes[s.mesh];
            if (m.type == 0) {
                if (g_avx512) {
                    if (scan_avx512(r, s, m, any, best, found) && any) return true;
                    continue;
                }
                for (size_t i = 0; i < s.wtris.size(); i++) {
                    Hit h;
                    if (wtri_hit(r, s.wtris[i], h) && (!found || h.t < best.t)) {
                        found = true; best = h; best.tri = &m.tris[i]; best.mat = &s.mat;
                        if (any) return true;
                    }
                }
            } else {
                Hit h;
                if (sph_hit(r, m.radius, s.model, h) && (!found || h.t < best.t)) {
                    found = true; best = h; best.mat = &s.mat;
                    if (any) return true;
                }
            }
        }
        if (found) out = best;
        return found;
    }
    // The triangles of one shape, 16 at a time: the float operations of
    // wtri_hit in the same order (no FMA: -ffp-contract=off holds for the
    // intrinsics too), every lane's rejections as masks. Each accepted lane is
    // then re-tested by wtri_hit itself in index order and combined with the
    // scalar rule, so the Hit records are the scalar ones. kEPS is a double
    // (Raytracer.h:12): for a float x, x < 1e-6 and x <= 1e-6 both equal
    // x <= kEPSf, the largest float below 1e-6. Returns whether this shape
    // had a hit (any: the first one ends the scan).
    __attribute__((target("avx512f"))) static bool scan_avx512(const Ray& r, const Shape& s, const Mesh& m, bool any,
                                                               Hit& best, bool& found) {
        const WTriSoA& T = s.soa;
        const __m512 ox = _mm512_set1_ps(r.o.x), oy = _mm512_set1_ps(r.o.y), oz = _mm512_set1_ps(r.o.z);
        const __m512 dx = _mm512_set1_ps(r.d.x), dy = _mm512_set1_ps(r.d.y), dz = _mm512_set1_ps(r.d.z);
        const __m512 eps = _mm512_set1_ps(kEPSf), zero = _mm512_setzero_ps(), half = _mm512_set1_ps(0.5f);
        const __m512i absm = _mm512_set1_epi32(0x7fffffff), sgn = _mm512_set1_epi32((int)0x80000000u);
#define ld(v, i) _mm512_loadu_ps((v).data() + (i))
#define add _mm512_add_ps
#define sub _mm512_sub_ps
#define mul _mm512_mul_ps
// CalcArea (Raytracer.cpp:937-942) of edges ab, ac against N, x 0.5
#define area2(abx, aby, abz, acx, acy, acz, nx, ny, nz)                                                       \
    mul(add(add(mul(sub(mul(aby, acz), mul(abz, acy)), nx), mul(sub(mul(abz, acx), mul(abx, acz)), ny)),       \
            mul(sub(mul(abx, acy), mul(aby, acx)), nz)),                                                       \
        half)
        bool hit_here = false;
        for (size_t i = 0; i < T.n; i += 16) {
            const __m512 nx = ld(T.nx, i), ny = ld(T.ny, i), nz = ld(T.nz, i);
            const __m512 nd = add(add(mul(nx, dx), mul(ny, dy)), mul(nz, dz));
            __mmask16 ok = _mm512_cmp_ps_mask(_mm512_castsi512_ps(_mm512_and_si512(_mm512_castps_si512(nd), absm)), eps,
                                              _CMP_NLE_UQ);  // !(|nd| < kEPS)
            if (!ok) continue;
            const __m512 no = add(add(mul(nx, ox), mul(ny, oy)), mul(nz, oz));
            const __m512 num = _mm512_castsi512_ps(_mm512_xor_si512(_mm512_castps_si512(add(no, ld(T.d, i))), sgn));
            const __m512 t = _mm512_div_ps(num, nd);
            ok &= _mm512_cmp_ps_mask(t, eps, _CMP_NLE_UQ);  // !(t <= kEPS)
            if (!ok) continue;
            const __m512 px = add(ox, mul(dx, t)), py = add(oy, mul(dy, t)), pz = add(oz, mul(dz, t));
            const __m512 v0x = ld(T.v0x, i), v0y = ld(T.v0y, i), v0z = ld(T.v0z, i);
            const __m512 v1x = ld(T.v1x, i), v1y = ld(T.v1y, i), v1z = ld(T.v1z, i);
            const __m512 v2x = ld(T.v2x, i), v2y = ld(T.v2y, i), v2z = ld(T.v2z, i);
            const __m512 ar = ld(T.area, i);
            const __m512 a = _mm512_div_ps(
                area2(sub(v1x, px), sub(v1y, py), sub(v1z, pz), sub(v2x, px), sub(v2y, py), sub(v2z, pz), nx, ny, nz), ar);
            ok &= _mm512_cmp_ps_mask(a, zero, _CMP_NLT_UQ);
            if (!ok) continue;
            const __m512 b = _mm512_div_ps(
                area2(sub(px, v0x), sub(py, v0y), sub(pz, v0z), sub(v2x, v0x), sub(v2y, v0y), sub(v2z, v0z), nx, ny, nz),
                ar);
            ok &= _mm512_cmp_ps_mask(b, zero, _CMP_NLT_UQ);
            if (!ok) continue;
            const __m512 g = _mm512_div_ps(
                area2(sub(v1x, v0x), sub(v1y, v0y), sub(v1z, v0z), sub(px, v0x), sub(py, v0y), sub(pz, v0z), nx, ny, nz),
                ar);
            ok &= _mm512_cmp_ps_mask(g, zero, _CMP_NLT_UQ);
            for (unsigned mk = ok; mk; mk &= mk - 1) {
                const size_t k = i + (size_t)__builtin_ctz(mk);
                Hit h;
                if (!wtri_hit(r, s.wtris[k], h)) {
                    std::fprintf(stderr, "oracle: 16-wide triangle scan disagrees with wtri_hit\n");
                    std::abort();
                }
                hit_here = true;
                if (!found || h.t < best.t) {
                    found = true; best = h; best.tri = &m.tris[k]; best.mat = &s.mat;
                }
                if (any) return true;
            }
        }
        return hit_here;
#undef ld
#undef add
#undef sub
#undef mul
#undef area2
    }
    // Ref-faithful mode (CPU-baseline timing only; same results): the work the
    // reference does per IntersectScene call as written — meshMap lookup by
    // string (:477), ComputeModelMatrix per shape (:480), and per triangle test
    // the unused Matrix::Inverse (:350-351) and three TransformPoint (:353-355).
    bool intersect_faithful(const Ray& r, Hit& out) const {
        Hit best;
        bool found = false;
        for (const Shape& s : sc->shapes) {
            const Mesh& m = sc->meshes[sc->mesh_by_name.at(s.geo)];
            const M4 model = model_matrix(s);
            if (m.type == 0) {
                for (const Tri& t : m.tris) {
                    M4 inv;
                    M4::inverse(model, inv);
                    g_sink = inv.m[0][0];  // computed, as in the reference, unused
                    Hit h;
                    if (tri_hit(r, t, model, h) && (!found || h.t < best.t)) {
                        found = true; best = h; best.tri = &t; best.mat = &s.mat;
                    }
                }
            } else {
                Hit h;
                if (sph_hit(r, m.radius, model, h) && (!found || h.t < best.t)) {
                    found = true; best = h; best.mat = &s.mat;
                }
            }
        }
        if (found) out = best;
        return found;
    }

    // CalculateAmbientOcclusion + RandomInHemisphere + RandomUnitVector, Raytracer.cpp:269-330
    float ambient_occlusion(const V3& hp, const V3& n, RngCursor& rng, Counters& c) const {
        c.ao_calls++;
        if (!ao_on) return 1.0f;
        float occ = 0.0f;
        for (int i = 0; i < ao_n; i++) {
            float z = rng.uniform(-1.0f, 1.0f);
            float a = rng.uniform(0.0f, ao_bmax);
            float r = std::sqrt(1 - z * z);
            double s, co;
            ::sincos((double)a, &s, &co);  // cos(a), sin(a) as g++ compiles them
            V3 v((float)((double)r * co), (float)((double)r * s), z);
            v.normalize();
            if (!(v.dot(n) > 0.0)) v = -v;
            Ray ray(hp + v * kOFFSET, v);
            Hit h;
            c.ao++;
            if (intersect(ray, h, true)) occ += 1.0f;
        }
        return 1.0f - ((float)occ / (float)ao_n);
    }

    static float fmax0(float x) { return (float)std::fmax((double)x, 0.0); }
    static float clipf(float x, int lo, int hi) { if (x < lo) return (float)lo; if (x > hi) return (float)hi; return x; }

    // CalculateLocalColor, Raytracer.cpp:213-267
    Pix local_color(const Hit& h, const Light& l, const Material& m) const {
        V3 L;
        if (l.type == LPOINT) { L = l.position - h.p; L.normalize(); }
        else { L = l.direction * -1; L.normalize(); }
        V3 n;
        if (h.type == 0) {
            n = (h.tri->nrm[0] * h.a + h.tri->nrm[1] * h.b) + h.tri->nrm[2] * h.g;  // InterpolateVector3 :333-338
            n.normalize();
        } else {
            n = h.n;
        }
        n.normalize();
        float ds = fmax0(L.dot(n));
        V3 diff = l.color * ds * l.intensity;
        V3 R = V3::reflect(L, n);
        R.normalize();
        V3 V = sc->cam.from - h.p;
        V.normalize();
        float ss = fmax0(V.dot(R));
        ss = powf(ss, m.n);
        V3 spec = l.color * ss * l.intensity;
        V3 lighting = diff * m.kd + spec * m.ks;
        V3 col = m.cs * lighting;
        col.x = clipf(col.x, 0, 1); col.y = clipf(col.y, 0, 1); col.z = clipf(col.z, 0, 1);
        return Pix(col);
    }
    // CalculateRefraction, Raytracer.cpp:168-203
    static V3 refraction(const V3& I, const V3& N, float ior) {
        float cosi = I.dot(N);
        if (cosi < -1) cosi = -1;
        else if (cosi > 1) cosi = 1;
        float n1 = 1, n2 = ior;
        V3 n = N;
        if (cosi < 0) cosi = -1 * cosi;
        else { float t = n1; n1 = n2; n2 = t; n = -N; }
        float eta = n1 / n2;
        float k = 1 - eta * eta * (1 - cosi * cosi);
        if (k < 0) return V3(0, 0, 0);
        return I * eta + n * (eta * cosi - std::sqrt(k));
    }
    // ComputeFresnel, Raytracer.cpp:131-166
    static void fresnel(float ior, const V3& N, const V3& I, float& kr, float& kt) {
        float cosi = clipf(I.dot(N), -1, 1);
        bool inside = cosi > 0;
        float ei = 1, et = ior;
        if (inside) { std::swap(ei, et); cosi = -cosi; }
        float sint = ei / et * std::sqrt(std::max(0.f, 1 - cosi * cosi));
        if (sint >= 1) { kr = 1; kt = 0; }
        else {
            float cost = std::sqrt(std::max(0.f, 1 - sint * sint));
            cosi = std::fabs(cosi);
            float Rs = ((et * cosi) - (ei * cost)) / ((et * cosi) + (ei * cost));
            float Rp = ((ei * cosi) - (et * cost)) / ((ei * cosi) + (et * cost));
            kr = (Rs * Rs + Rp * Rp) / 2;
            kt = 1 - kr;
        }
    }

    // Raycast, Raytracer.cpp:28-129
    Pix raycast(const Ray& ray, int bounces, RngCursor* rng, Counters& c, bool count_only) const {
        Hit info;
        if (!intersect(ray, info)) return Pix(254, 64, 205);  // BG_COLOR, Raytracer.h:597
        c.tree_hits++;
        const Material& m = *info.mat;
        Pix local(0, 0, 0);
        for (const Light& l : sc->lights) {
            if (l.type == LAMB) {
                if (count_only) { c.ao_calls++; c.ao += ao_on ? ao_n : 0; continue; }
                V3 amb = m.cs * m.ka * l.color * l.intensity;
                amb = amb * ambient_occlusion(info.p, info.n, *rng, c);
                local = local + Pix(amb);
                continue;
            }
            V3 L;
            if (l.type == LDIR) L = -(l.direction);
            else L = (l.position - info.p);
            L.normalize();
            Ray lr(info.p + L * kOFFSET, L);
            float dist = (l.position - info.p).length();
            c.shadow++;
            if (count_only) continue;
            Hit lh;
            if (!intersect(lr, lh, l.type == LDIR) || (lh.t > dist && l.type == LPOINT))
                local = local + local_color(info, l, m);
        }
        if (bounces > 0) {
            float kr, kt;
            Pix refl, refr;
            if (m.ks > 0) {
                V3 d = V3::reflect(ray.d, info.n);
                d.normalize();
                Ray rr(info.p + d * kOFFSET, d);
                c.secondary++;
                refl = raycast(rr, bounces - 1, rng, c, count_only);
            }
            if (m.kt > 0) {
                V3 d = refraction(ray.d, info.n, m.ior);
                Ray tr(info.p + d * kOFFSET, d);
                c.secondary++;
                refr = raycast(tr, bounces - 1, rng, c, count_only);
            }
            fresnel(m.ior, info.n, ray.d, kr, kt);
            Pix fr = refl * kr * m.ks;
            Pix ft = refr * kt * m.kt;
            float alb = 1 - m.ks - m.kt;
            alb = std::max(alb, 0.0f);
            local = (local * alb) + (fr * m.ks) + (ft * m.kt);
        }
        return local.clamp();
    }
};

struct Camera2 {
    bool inv_ok = false;
    M4 inv;
    V3 from;
    double kx = 0, ky = 0;
    int w = 0, h = 0;
};

// InitializeRenderer + CalculateViewMatrix, Raytracer.cpp:861-870, :895-915; GenerateRay constants :832-858
static Camera2 init_camera(const Scene& sc, int w, int h) {
    Camera2 c;
    V3 n = sc.cam.from - sc.cam.to;
    n.normalize();
    V3 up(0, 1, 0);
    V3 u = V3::cross(up, n);
    u.normalize();
    V3 v = V3::cross(n, u);
    v.normalize();
    V3 r = sc.cam.from;
    M4 view;
    view.m[0][0] = u.x; view.m[0][1] = u.y; view.m[0][2] = u.z; view.m[0][3] = -r.dot(u);
    view.m[1][0] = v.x; view.m[1][1] = v.y; view.m[1][2] = v.z; view.m[1][3] = -r.dot(v);
    view.m[2][0] = n.x; view.m[2][1] = n.y; view.m[2][2] = n.z; view.m[2][3] = -r.dot(n);
    view.m[3][0] = 0; view.m[3][1] = 0; view.m[3][2] = 0; view.m[3][3] = 1;
    c.inv_ok = M4::inverse(view, c.inv);
    c.from = sc.cam.from;
    float fov = 60.0f;  // Raytracer.cpp:786
    float aspect = (float)w / (float)h;
    double tn = std::tan((double)ToRadian(fov / 2));
    c.kx = aspect * tn;
    c.ky = tn;
    c.w = w; c.h = h;
    return c;
}

static Ray generate_ray(const Camera2& c, int x, int y) {  // GenerateRay, Raytracer.cpp:832-858
    double ndcx = (2.0 * x) / c.w - 1;
    double ndcy = 1 - (2.0 * y) / c.h;
    ndcx *= c.kx;
    ndcy *= c.ky;
    Ray r;
    r.o = c.from;
    V3 d((float)ndcx, (float)ndcy, -1.0f);
    if (c.inv_ok) {
        r.d = c.inv.xform_dir(d);
        r.d.normalize();
    }
    return r;
}

}  // namespace ora

using namespace ora;

// Worker threads: $OMP_NUM_THREADS when set (the GPU box caps a job's CPU share
// there), else every hardware thread.
static int default_threads() {
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
        int n = std::atoi(e);
        if (n > 0) return n;
    }
    int n = (int)std::thread::hardware_concurrency();
    return n > 0 ? n : 1;
}

extern "C" int oracle_set_mode(int faithful) {
    g_faithful = faithful ? 1 : 0;
    return 0;
}

extern "C" int oracle_render(const char* assets_root, const char* scene, int w, int h, int depth,
                             int ao_samples, int ao_enabled, int engine, int threads, int row_begin,
                             int row_end, int16_t* fb, uint64_t* counters, uint64_t* rays_per_row) {
    if (w <= 0 || h <= 0 || depth < 0 || ao_samples <= 0 || row_begin < 0 || row_end > h || row_begin > row_end)
        return 2;
    Scene sc;
    if (load_scene(sc, assets_root, scene) != 0) return 1;
    for (const Shape& s : sc.shapes)
        if (s.mesh < 0) return 1;
    Camera2 cam = init_camera(sc, w, h);
    Tracer tr;
    tr.sc = &sc;
    tr.depth = depth;
    tr.ao_n = ao_samples;
    tr.ao_on = ao_enabled;
    tr.ao_bmax = (float)(2 * kPI);
    tr.n_amb = 0;
    for (auto& l : sc.lights) tr.n_amb += l.type == LAMB;
    if (threads <= 0) threads = default_threads();

    // Pass 1: AO calls per pixel for every pixel in [0, row_end) (raster prefix).
    const int nrows_all = row_end;
    std::vector<uint32_t> calls((size_t)nrows_all * w);
    {
        // work items are pixels (not rows): tiny frames at high AO counts still use every core
        std::atomic<int64_t> next{0};
        const int64_t npix = (int64_t)nrows_all * w;
        auto work = [&] {
            for (;;) {
                int64_t i = next.fetch_add(1);
                if (i >= npix) break;
                Counters c;
                tr.raycast(generate_ray(cam, (int)(i % w), (int)(i / w)), depth, nullptr, c, true);
                calls[(size_t)i] = (uint32_t)c.ao_calls;
            }
        };
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(work);
        for (auto& t : th) t.join();
    }
    std::vector<uint64_t> base((size_t)nrows_all * w + 1, 0);
    for (size_t i = 0; i < calls.size(); i++) base[i + 1] = base[i] + calls[i];
    DrawSource src;
    src.engine = engine;
    const uint64_t per_call = 2ull * (uint64_t)ao_samples;
    if (engine == 1 && ao_enabled) {
        uint64_t total = base.back() * per_call;
        src.stream.resize(total);
        std::mt19937 g;  // default seed 5489
        for (uint64_t i = 0; i < total; i++) src.stream[i] = (uint32_t)g();
    }
    // Pass 2: render rows [row_begin, row_end).
    const int64_t nsel = (int64_t)(row_end - row_begin) * w;
    std::vector<Counters> pixc((size_t)nsel);
    {
        std::atomic<int64_t> next{0};
        auto work = [&] {
            RngCursor rng;
            rng.src = &src;
            for (;;) {
                int64_t i = next.fetch_add(1);
                if (i >= nsel) break;
                const int y = row_begin + (int)(i / w), x = (int)(i % w);
                Counters& c = pixc[(size_t)i];
                size_t pi = (size_t)y * w + x;
                rng.seek(ao_enabled ? base[pi] * per_call : 0);
                Ray r = generate_ray(cam, x, y);
                c.primary++;
                Pix p = tr.raycast(r, depth, &rng, c, fb == nullptr);
                if (fb) {
                    int16_t* o = fb + (size_t)i * 3;
                    o[0] = p.r; o[1] = p.g; o[2] = p.b;
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(work);
        for (auto& t : th) t.join();
    }
    std::vector<Counters> rowc((size_t)(row_end - row_begin));
    for (int64_t i = 0; i < nsel; i++) {
        Counters& r = rowc[(size_t)(i / w)];
        const Counters& c = pixc[(size_t)i];
        r.primary += c.primary; r.secondary += c.secondary; r.shadow += c.shadow;
        r.ao += c.ao; r.ao_calls += c.ao_calls;
    }
    Counters tot;
    for (size_t i = 0; i < rowc.size(); i++) {
        const Counters& c = rowc[i];
        uint64_t row_total = c.primary + c.secondary + c.shadow + c.ao;
        if (rays_per_row) rays_per_row[i] = row_total;
        tot.primary += c.primary; tot.secondary += c.secondary; tot.shadow += c.shadow;
        tot.ao += c.ao; tot.ao_calls += c.ao_calls;
    }
    if (counters) {
        counters[0] = tot.primary + tot.secondary + tot.shadow + tot.ao;
        counters[1] = tot.primary; counters[2] = tot.secondary; counters[3] = tot.shadow;
        counters[4] = tot.ao; counters[5] = tot.ao_calls;
    }
    return 0;
}

// CPU baseline (bench.py cpu_baseline): the reference's Render loop
// (Raytracer.cpp:921-932) over an exact raster range of the FULL-resolution
// w x h frame, pixels [p0, p0 + n), with the serial RNG stream positioned at
// the absolute AO-call index call_base (draw 2 * ao_n * call_base; 0 for a
// range that no AO call precedes, e.g. one starting below the sky rows).
//  threads == 1: one serial stream, pixel after pixel, as the reference does;
//    stops after max_pixels pixels or once budget_s seconds have passed (checked
//    after each pixel) -> *n_done.
//  threads > 1: exactly max_pixels pixels on `threads` threads: a count pass
//    (AO calls per pixel, the work the serial stream needs to be split), the
//    exclusive scan, then the pixels as work items.
// fb receives the range's int16 pixels (n_done x 3); counters as oracle_render
// (the count pass's rays are not counted: they are overhead of the split);
// *seconds the render time (scene load excluded, as Render() excludes it).
extern "C" int oracle_time_prefix(const char* assets_root, const char* scene, int w, int h, int depth,
                                  int ao_samples, int threads, int64_t p0, int64_t max_pixels, double budget_s,
                                  uint64_t call_base, int16_t* fb, uint64_t* counters, int64_t* n_done,
                                  double* seconds) {
    const int64_t npix = (int64_t)w * h;
    if (w <= 0 || h <= 0 || depth < 0 || ao_samples <= 0 || p0 < 0 || max_pixels < 0 || p0 + max_pixels > npix ||
        threads < 1 || !fb || !n_done)
        return 2;
    Scene sc;
    if (load_scene(sc, assets_root, scene) != 0) return 1;
    for (const Shape& s : sc.shapes)
        if (s.mesh < 0) return 1;
    Camera2 cam = init_camera(sc, w, h);
    Tracer tr;
    tr.sc = &sc;
    tr.depth = depth;
    tr.ao_n = ao_samples;
    tr.ao_on = 1;
    tr.ao_bmax = (float)(2 * kPI);
    tr.n_amb = 0;
    for (auto& l : sc.lights) tr.n_amb += l.type == LAMB;
    DrawSource src;
    src.engine = 0;
    const uint64_t per_call = 2ull * (uint64_t)ao_samples;
    Counters tot;
    auto add = [&tot](const Counters& c) {
        tot.primary += c.primary; tot.secondary += c.secondary; tot.shadow += c.shadow;
        tot.ao += c.ao; tot.ao_calls += c.ao_calls;
    };
    auto put = [fb, p0](int64_t i, const Pix& p) {
        int16_t* o = fb + (size_t)(i - p0) * 3;
        o[0] = p.r; o[1] = p.g; o[2] = p.b;
    };
    int64_t done = 0;
    const auto t_start = std::chrono::steady_clock::now();
    if (threads == 1) {
        RngCursor rng;
        rng.src = &src;
        rng.seek(call_base * per_call);
        const auto t0 = std::chrono::steady_clock::now();
        for (int64_t i = p0; i < p0 + max_pixels; i++) {
            Counters c;
            c.primary++;
            put(i, tr.raycast(generate_ray(cam, (int)(i % w), (int)(i / w)), depth, &rng, c, false));
            add(c);
            done++;
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >= budget_s) break;
        }
    } else {
        std::vector<uint64_t> base((size_t)max_pixels + 1, 0);
        std::vector<Counters> pc((size_t)max_pixels);
        std::atomic<int64_t> next{0};
        auto count = [&] {
            for (int64_t k; (k = next.fetch_add(1)) < max_pixels;) {
                Counters c;
                tr.raycast(generate_ray(cam, (int)((p0 + k) % w), (int)((p0 + k) / w)), depth, nullptr, c, true);
                base[(size_t)k + 1] = c.ao_calls;
            }
        };
        auto shade = [&] {
            RngCursor rng;
            rng.src = &src;
            for (int64_t k; (k = next.fetch_add(1)) < max_pixels;) {
                rng.seek((call_base + base[(size_t)k]) * per_call);
                Counters& c = pc[(size_t)k];
                c.primary++;
                put(p0 + k, tr.raycast(generate_ray(cam, (int)((p0 + k) % w), (int)((p0 + k) / w)), depth, &rng, c,
                                       false));
            }
        };
        auto run = [&](const std::function<void()>& fn) {
            next = 0;
            std::vector<std::thread> th;
            for (int t = 0; t < threads; t++) th.emplace_back(fn);
            for (auto& t : th) t.join();
        };
        run(count);
        for (size_t k = 0; k < (size_t)max_pixels; k++) base[k + 1] += base[k];
        run(shade);
        for (const Counters& c : pc) add(c);
        done = max_pixels;
    }
    *n_done = done;
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    if (counters) {
        counters[0] = tot.primary + tot.secondary + tot.shadow + tot.ao;
        counters[1] = tot.primary; counters[2] = tot.secondary; counters[3] = tot.shadow;
        counters[4] = tot.ao; counters[5] = tot.ao_calls;
    }
    return 0;
}

// Frame check of a full-resolution GPU frame (bench.py): pixel segments
// [x0, x0 + n) of rows y of the w x h frame, each row's first AO call at
// row_base[k] (the GPU's exclusive scan of its per-row counts). A count pass
// over each segment's whole row gives the in-row prefix of the segment's first
// pixel and the row's AO-call total (-> row_calls[k], compared with the GPU's
// count by the caller); then the segments' pixels are shaded. Work items are
// pixels on `threads` threads. fb: sum(n) x 3 int16, segment after segment.
// RNG engine of oracle_render_segments: 0 minstd_rand0 (default), 1 mt19937.
static int g_seg_engine = 0;
extern "C" void oracle_set_segments_engine(int engine) { g_seg_engine = engine == 1 ? 1 : 0; }

extern "C" int oracle_render_segments(const char* assets_root, const char* scene, int w, int h, int depth,
                                      int ao_samples, int threads, int n_seg, const int32_t* seg_y,
                                      const int32_t* seg_x0, const int32_t* seg_n, const uint64_t* row_base,
                                      int16_t* fb, uint64_t* row_calls, uint64_t* counters, double* seconds) {
    if (w <= 0 || h <= 0 || depth < 0 || ao_samples <= 0 || threads < 1 || n_seg < 0 || !fb || !row_calls) return 2;
    std::vector<int64_t> off((size_t)n_seg + 1, 0);
    for (int k = 0; k < n_seg; k++) {
        if (seg_y[k] < 0 || seg_y[k] >= h || seg_x0[k] < 0 || seg_n[k] < 0 || seg_x0[k] + seg_n[k] > w) return 2;
        off[(size_t)k + 1] = off[(size_t)k] + seg_n[k];
    }
    Scene sc;
    if (load_scene(sc, assets_root, scene) != 0) return 1;
    for (const Shape& s : sc.shapes)
        if (s.mesh < 0) return 1;
    Camera2 cam = init_camera(sc, w, h);
    Tracer tr;
    tr.sc = &sc;
    tr.depth = depth;
    tr.ao_n = ao_samples;
    tr.ao_on = 1;
    tr.ao_bmax = (float)(2 * kPI);
    tr.n_amb = 0;
    for (auto& l : sc.lights) tr.n_amb += l.type == LAMB;
    const auto t0 = std::chrono::steady_clock::now();
    auto run = [threads](const std::function<void()>& fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; t++) th.emplace_back(fn);
        for (auto& t : th) t.join();
    };
    // count pass over every pixel of the segments' rows
    std::vector<uint32_t> calls((size_t)n_seg * w);
    {
        std::atomic<int64_t> next{0};
        const int64_t total = (int64_t)n_seg * w;
        run([&] {
            for (int64_t i; (i = next.fetch_add(1)) < total;) {
                const int k = (int)(i / w), x = (int)(i % w);
                Counters c;
                tr.raycast(generate_ray(cam, x, seg_y[k]), depth, nullptr, c, true);
                calls[(size_t)i] = (uint32_t)c.ao_calls;
            }
        });
    }
    std::vector<uint64_t> first((size_t)off[(size_t)n_seg]);  // each segment pixel's first AO call
    for (int k = 0; k < n_seg; k++) {
        uint64_t acc = row_base[k], tot = 0;
        for (int x = 0; x < w; x++) {
            if (x >= seg_x0[k] && x < seg_x0[k] + seg_n[k]) first[(size_t)(off[(size_t)k] + x - seg_x0[k])] = acc;
            acc += calls[(size_t)k * w + x];
            tot += calls[(size_t)k * w + x];
        }
        row_calls[k] = tot;
    }
    DrawSource src;
    src.engine = g_seg_engine;
    const uint64_t per_call = 2ull * (uint64_t)ao_samples;
    const int64_t npx = off[(size_t)n_seg];
    if (src.engine == 1 && n_seg > 0) {
        // mt19937 (seed 5489): the draws of the segments' rows, [lo, hi) of the
        // serial stream, by the engine itself (discard = the reference's own
        // stepping, however far out the rows start)
        uint64_t lo = ~0ull, hi = 0;
        for (int k = 0; k < n_seg; k++) {
            lo = std::min(lo, row_base[k] * per_call);
            hi = std::max(hi, (row_base[k] + row_calls[k]) * per_call);
        }
        std::mt19937 g;
        g.discard(lo);
        src.lo = lo;
        src.stream.resize((size_t)(hi - lo));
        for (auto& x : src.stream) x = (uint32_t)g();
    }
    std::vector<Counters> pc((size_t)npx);
    {
        std::atomic<int64_t> next{0};
        run([&] {
            RngCursor rng;
            rng.src = &src;
            for (int64_t i; (i = next.fetch_add(1)) < npx;) {
                int k = 0;
                while (off[(size_t)k + 1] <= i) k++;
                const int x = seg_x0[k] + (int)(i - off[(size_t)k]);
                rng.seek(first[(size_t)i] * per_call);
                Counters& c = pc[(size_t)i];
                c.primary++;
                Pix p = tr.raycast(generate_ray(cam, x, seg_y[k]), depth, &rng, c, false);
                int16_t* o = fb + (size_t)i * 3;
                o[0] = p.r; o[1] = p.g; o[2] = p.b;
            }
        });
    }
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (counters) {
        Counters tot;
        for (const Counters& c : pc) {
            tot.primary += c.primary; tot.secondary += c.secondary; tot.shadow += c.shadow;
            tot.ao += c.ao; tot.ao_calls += c.ao_calls;
        }
        counters[0] = tot.primary + tot.secondary + tot.shadow + tot.ao;
        counters[1] = tot.primary; counters[2] = tot.secondary; counters[3] = tot.shadow;
        counters[4] = tot.ao; counters[5] = tot.ao_calls;
    }
    return 0;
}

// ---- row-level entry points (the multi-rank split of SURVEY §8e, for tests) ----
namespace {
struct Loaded {
    Scene sc;
    Camera2 cam;
    Tracer tr;
};
int load_all(Loaded& L, const char* root, const char* scene, int w, int h, int depth, int ao_n, int ao_on) {
    if (w <= 0 || h <= 0 || depth < 0 || ao_n <= 0) return 2;
    if (load_scene(L.sc, root, scene) != 0) return 1;
    for (const Shape& s : L.sc.shapes)
        if (s.mesh < 0) return 1;
    L.cam = init_camera(L.sc, w, h);
    L.tr.sc = &L.sc;
    L.tr.depth = depth;
    L.tr.ao_n = ao_n;
    L.tr.ao_on = ao_on;
    L.tr.ao_bmax = (float)(2 * kPI);
    L.tr.n_amb = 0;
    return 0;
}
}  // namespace

// AO calls of rows row_begin + k*row_step (k < n_rows) -> out[k].
extern "C" int oracle_count_rows(const char* root, const char* scene, int w, int h, int depth, int ao_n,
                                 int ao_on, int row_begin, int row_step, int n_rows, uint32_t* out) {
    Loaded L;
    int st = load_all(L, root, scene, w, h, depth, ao_n, ao_on);
    if (st) return st;
    for (int k = 0; k < n_rows; k++) {
        int y = row_begin + k * row_step;
        uint64_t calls = 0;
        for (int x = 0; x < w; x++) {
            Counters c;
            L.tr.raycast(generate_ray(L.cam, x, y), depth, nullptr, c, true);
            calls += c.ao_calls;
        }
        out[k] = (uint32_t)calls;
    }
    return 0;
}

// AO calls of the pixels (x0 + k, y), k < n -> out[k] (parity hunts: which
// pixel of a row holds a differing count).
extern "C" int oracle_count_pixels(const char* root, const char* scene, int w, int h, int depth, int ao_n, int ao_on,
                                   int y, int x0, int n, uint32_t* out) {
    Loaded L;
    int st = load_all(L, root, scene, w, h, depth, ao_n, ao_on);
    if (st) return st;
    for (int k = 0; k < n; k++) {
        Counters c;
        L.tr.raycast(generate_ray(L.cam, x0 + k, y), depth, nullptr, c, true);
        out[k] = (uint32_t)c.ao_calls;
    }
    return 0;
}

// Shade the same rows given each row's absolute first AO-call index (minstd_rand0).
extern "C" int oracle_shade_rows(const char* root, const char* scene, int w, int h, int depth, int ao_n,
                                 int ao_on, int row_begin, int row_step, int n_rows, const uint64_t* row_base,
                                 int16_t* fb) {
    Loaded L;
    int st = load_all(L, root, scene, w, h, depth, ao_n, ao_on);
    if (st) return st;
    DrawSource src;
    src.engine = 0;
    RngCursor rng;
    rng.src = &src;
    const uint64_t per_call = 2ull * (uint64_t)ao_n;
    for (int k = 0; k < n_rows; k++) {
        int y = row_begin + k * row_step;
        uint64_t call = row_base[k];
        for (int x = 0; x < w; x++) {
            Counters cc;
            L.tr.raycast(generate_ray(L.cam, x, y), depth, nullptr, cc, true);  // this pixel's AO calls
            rng.seek(ao_on ? call * per_call : 0);
            Counters c;
            Pix p = L.tr.raycast(generate_ray(L.cam, x, y), depth, &rng, c, false);
            int16_t* o = fb + ((size_t)k * w + x) * 3;
            o[0] = p.r; o[1] = p.g; o[2] = p.b;
            call += cc.ao_calls;
        }
    }
    return 0;
}

// FlushFrameBufferToPPM, Raytracer.cpp:796-830
extern "C" int oracle_write_ppm(const char* path, int w, int h, const int16_t* fb) {
    std::ofstream out(path, std::ios::binary);
    if (!out.is_open()) return 1;
    out << "P6\n" << w << " " << h << "\n255\n";
    for (size_t i = 0; i < (size_t)w * h * 3; i++) {
        unsigned char c = static_cast<unsigned char>(std::pow(fb[i] / 255.0f, 1.0f / 2.2f) * 255.0f);
        out.put((char)c);
    }
    return 0;
}
