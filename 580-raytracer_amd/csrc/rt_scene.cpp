// rt_scene.cpp — see rt_scene.h. Compiled with -ffp-contract=off.
#include "rt_scene.h"

#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>

#include "json_min.h"

namespace rt580 {

static const double kPI = 3.14159265;  // Raytracer.h:11

static bool read_text(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

static rv3 json_vec3(const json_min::Value& a) {
    return v3(a.at(0).as_float(), a.at(1).as_float(), a.at(2).as_float());
}

// LoadMesh, Raytracer.cpp:589-643: the type is taken from data[0] only; every
// item of a polygon mesh is a triangle {v0,v1,v2:{v,n,t}}; a sphere mesh keeps
// the radius of its last item; any other type (e.g. Assets/1plane.json "plane")
// leaves the value-initialised mesh: an empty polygon mesh.
static int load_mesh(const std::string& root, const std::string& name, Scene& sc, int& index,
                     std::string& err) {
    auto it = sc.mesh_index.find(name);
    if (it != sc.mesh_index.end()) { index = it->second; return RT_SUCCESS; }
    std::string text;
    if (!read_text(root + "/Assets/" + name + ".json", text)) {
        err = "File with name Assets/" + name + ".json could not be found";
        index = -1;
        return RT_FAILURE;
    }
    json_min::Value j = json_min::parse(text);
    Mesh mesh;
    const std::string type = j.at("data").at(0).at("type").as_string();
    for (const json_min::Value* item : j.at("data").items()) {
        if (type == "polygon") {
            mesh.type = RT_PRIM_TRIANGLE;
            Triangle t;
            for (int i = 0; i < 3; i++) {
                const json_min::Value& v = item->at("v" + std::to_string(i));
                t.pos[i] = json_vec3(v.at("v"));
                t.nrm[i] = json_vec3(v.at("n"));
                (void)v.at("t").at(0).as_float();  // texture coordinates are parsed, unused
                (void)v.at("t").at(1).as_float();
            }
            mesh.tris.push_back(t);
        } else if (type == "sphere") {
            mesh.type = RT_PRIM_SPHERE;
            mesh.radius = item->at("radius").as_float();
        }
    }
    sc.meshes.push_back(mesh);
    index = (int)sc.meshes.size() - 1;
    sc.mesh_index[name] = index;
    return RT_SUCCESS;
}

int load_scene_json(const std::string& root, const std::string& scene_path, Scene& sc,
                    std::string& err) {
    sc = Scene();
    std::string text;
    if (!read_text(root + "/Assets/" + scene_path, text)) {
        err = "Failed to open JSON file Path: Assets/" + scene_path;
        return RT_FAILURE;
    }
    int status = RT_SUCCESS;
    try {
        json_min::Value j = json_min::parse(text);
        // jsonData["scene"] (Raytracer.cpp:667) on the non-const document: a
        // document without "scene" (or with a non-object there) has no shapes,
        // camera or lights and still loads -- so does the document `null`,
        // which operator[] turns into an object; any other non-object
        // document is a type error (tests/golden/loader: null_document,
        // array_document, number_document).
        if (!j.is_object() && !j.is_null())
            throw json_min::error("type_error: cannot use operator[] with a string argument");
        static const json_min::Value kNull;
        const json_min::Value& s = j.contains("scene") ? j.at("scene") : kNull;
        if (s.contains("shapes")) {
            for (const json_min::Value* sv : s.at("shapes").items()) {
                Shape shp;
                shp.id = sv->at("id").as_string();
                shp.geometry = sv->at("geometry").as_string();
                if (sv->contains("notes")) (void)sv->at("notes").as_string();  // get<std::string>() (:673-675)
                const json_min::Value& m = sv->at("material");
                shp.material.cs = json_vec3(m.at("Cs"));
                shp.material.ka = m.at("Ka").as_float();
                shp.material.kd = m.at("Kd").as_float();
                shp.material.ks = m.at("Ks").as_float();
                shp.material.kt = m.at("Kt").as_float();
                shp.material.spec_exp = m.at("n").as_float();
                // Raytracer.cpp:688-716: later elements override earlier ones
                for (const json_min::Value* t : sv->at("transforms").items()) {
                    if (t->contains("Rx")) shp.rotation.x = t->at("Rx").as_float();
                    if (t->contains("Ry")) shp.rotation.y = t->at("Ry").as_float();
                    if (t->contains("Rz")) shp.rotation.z = t->at("Rz").as_float();
                    if (t->contains("S") && t->at("S").is_array()) shp.scale = json_vec3(t->at("S"));
                    if (t->contains("T") && t->at("T").is_array()) shp.translation = json_vec3(t->at("T"));
                }
                std::string merr;
                int st = load_mesh(root, shp.geometry, sc, shp.mesh, merr);
                if (st != RT_SUCCESS) err = merr;
                status |= st;
                sc.shapes.push_back(shp);
            }
        }
        if (s.contains("camera")) {
            const json_min::Value& c = s.at("camera");
            sc.camera.from = json_vec3(c.at("from"));
            sc.camera.to = json_vec3(c.at("to"));
            for (int i = 0; i < 6; i++) (void)c.at("bounds").at(i).as_float();  // parsed, unused by Render
            (void)c.at("resolution").at(0).as_int();
            (void)c.at("resolution").at(1).as_int();
        }
        if (s.contains("lights")) {
            for (const json_min::Value* lv : s.at("lights").items()) {
                Light l;
                l.color = json_vec3(lv->at("color"));
                l.intensity = lv->at("intensity").as_float();
                const std::string& t = lv->at("type").as_string();
                if (t == "directional") {
                    rv3 from = json_vec3(lv->at("from")), to = json_vec3(lv->at("to"));
                    l.direction = v3_normalize(v3_sub(to, from));  // Raytracer.cpp:757-758
                    l.kind = RT_LIGHT_DIRECTIONAL;
                } else if (t == "ambient") {
                    l.kind = RT_LIGHT_AMBIENT;
                } else if (t == "point") {
                    l.kind = RT_LIGHT_POINT;
                    l.position = json_vec3(lv->at("position"));
                } else {
                    // The reference leaves lightType uninitialised here (undefined behaviour).
                    err = "unsupported light type '" + t + "'";
                    return RT_FAILURE;
                }
                sc.lights.push_back(l);
            }
        }
    } catch (const std::exception& e) {
        err = std::string("Error parsing JSON ") + e.what();
        return RT_FAILURE;
    }
    return status;
}

static void identity(Matrix4& a) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) a.m[i][j] = (i == j) ? 1.0f : 0.0f;
}

static Matrix4 mul(const Matrix4& a, const Matrix4& b) {  // Raytracer.h:179-190
    Matrix4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            r.m[i][j] = 0;
            for (int k = 0; k < 4; ++k) r.m[i][j] += a.m[i][k] * b.m[k][j];
        }
    return r;
}

static float to_radian(float deg) { return (float)(deg * (kPI / 180)); }  // Raytracer.h:581-583

Matrix4 compute_model_matrix(const Shape& s) {
    Matrix4 S, RX, RY, RZ, T;
    identity(S);
    S.m[0][0] = s.scale.x; S.m[1][1] = s.scale.y; S.m[2][2] = s.scale.z; S.m[3][3] = 1.0f;
    // The reference's cos(r)/sin(r) pairs are compiled into one glibc sincos call.
    double sx, cx, sy, cy, sz, cz;
    ::sincos((double)to_radian(s.rotation.x), &sx, &cx);
    ::sincos((double)to_radian(s.rotation.y), &sy, &cy);
    ::sincos((double)to_radian(s.rotation.z), &sz, &cz);
    identity(RX);
    RX.m[1][1] = (float)cx; RX.m[1][2] = (float)-sx; RX.m[2][1] = (float)sx; RX.m[2][2] = (float)cx;
    identity(RY);
    RY.m[0][0] = (float)cy; RY.m[0][2] = (float)sy; RY.m[2][0] = (float)-sy; RY.m[2][2] = (float)cy;
    identity(RZ);
    RZ.m[0][0] = (float)cz; RZ.m[0][1] = (float)-sz; RZ.m[1][0] = (float)sz; RZ.m[1][1] = (float)cz;
    Matrix4 R = mul(mul(RZ, RY), RX);
    identity(T);
    T.m[0][3] = s.translation.x; T.m[1][3] = s.translation.y; T.m[2][3] = s.translation.z;
    return mul(mul(S, R), T);
}

static rv3 transform_point(const Matrix4& M, rv3 p) {  // Raytracer.h:234-248
    float x = M.m[0][0] * p.x + M.m[0][1] * p.y + M.m[0][2] * p.z + M.m[0][3];
    float y = M.m[1][0] * p.x + M.m[1][1] * p.y + M.m[1][2] * p.z + M.m[1][3];
    float z = M.m[2][0] * p.x + M.m[2][1] * p.y + M.m[2][2] * p.z + M.m[2][3];
    float w = M.m[3][0] * p.x + M.m[3][1] * p.y + M.m[3][2] * p.z + M.m[3][3];
    if (w != 1.0f) { x /= w; y /= w; z /= w; }
    return v3(x, y, z);
}

static float tri_area_signed(rv3 A, rv3 B, rv3 C, rv3 N) {  // Raytracer.cpp:937-942
    rv3 c = v3_cross(v3_sub(B, A), v3_sub(C, A));
    return (float)(0.5 * v3_dot(c, N));
}

static void set3(float* d, rv3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

void pack_scene(const Scene& sc, PackedScene& out) {
    out = PackedScene();
    for (size_t si = 0; si < sc.shapes.size(); si++) {
        const Shape& shp = sc.shapes[si];
        rt_material m;
        std::memset(&m, 0, sizeof m);
        set3(m.cs, shp.material.cs);
        m.ka = shp.material.ka; m.kd = shp.material.kd; m.ks = shp.material.ks; m.kt = shp.material.kt;
        m.spec_exp = shp.material.spec_exp; m.ior = shp.material.ior;
        out.materials.push_back(m);
        const Mesh& mesh = sc.meshes[shp.mesh];
        Matrix4 M = compute_model_matrix(shp);
        if (mesh.type == RT_PRIM_TRIANGLE) {
            for (const Triangle& t : mesh.tris) {
                rt_prim p;
                rt_prim_shade s;
                std::memset(&p, 0, sizeof p);
                std::memset(&s, 0, sizeof s);
                // IntersectTriangle's ray-invariant part (Raytracer.cpp:353-389)
                rv3 v0 = transform_point(M, t.pos[0]);
                rv3 v1 = transform_point(M, t.pos[1]);
                rv3 v2 = transform_point(M, t.pos[2]);
                rv3 n = v3_normalize(v3_cross(v3_sub(v1, v0), v3_sub(v2, v0)));
                set3(p.p0, v0); set3(p.p1, v1); set3(p.p2, v2); set3(p.nrm, n);
                p.d = -v3_dot(n, v0);
                p.area = tri_area_signed(v0, v1, v2, n);
                p.kind = RT_PRIM_TRIANGLE;
                p.shape = (int32_t)si;
                set3(s.hit_nrm, v3_normalize(n));  // hitInfo.normal.normalize() (:402-403)
                set3(s.vn0, t.nrm[0]); set3(s.vn1, t.nrm[1]); set3(s.vn2, t.nrm[2]);
                out.prims.push_back(p);
                out.shade.push_back(s);
                out.n_triangles++;
            }
        } else {
            rt_prim p;
            rt_prim_shade s;
            std::memset(&p, 0, sizeof p);
            std::memset(&s, 0, sizeof s);
            set3(p.p0, v3(M.m[0][3], M.m[1][3], M.m[2][3]));  // GetTranslation (Raytracer.h:212-214)
            p.d = mesh.radius * mesh.radius;                    // (Raytracer.cpp:423)
            p.kind = RT_PRIM_SPHERE;
            p.shape = (int32_t)si;
            out.prims.push_back(p);
            out.shade.push_back(s);
            out.n_spheres++;
        }
    }
    for (const Light& l : sc.lights) {
        rt_light o;
        std::memset(&o, 0, sizeof o);
        o.kind = l.kind;
        set3(o.color, l.color);
        o.intensity = l.intensity;
        set3(o.position, l.position);
        set3(o.dir, l.direction);
        if (l.kind == RT_LIGHT_DIRECTIONAL) {
            rv3 L = v3_normalize(v3_neg(l.direction));  // Raytracer.cpp:59,65 (== :220-221)
            set3(o.L, L);
            set3(o.L2, v3_normalize(L));                // Ray ctor (Raytracer.h:431-433)
        }
        out.lights.push_back(o);
    }
}

// ---- camera (Raytracer.h:251-370 for the inverse) ----
static float det3(const Matrix4& a) {
    return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
           a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
           a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
}

static float det4(const Matrix4& a) {
    float det = 0;
    for (int i = 0; i < 4; i++) {
        Matrix4 sub;
        std::memset(&sub, 0, sizeof sub);
        for (int j = 1; j < 4; j++)
            for (int k = 0; k < 4; k++) {
                if (k < i) sub.m[j - 1][k] = a.m[j][k];
                else if (k > i) sub.m[j - 1][k - 1] = a.m[j][k];
            }
        det += (i % 2 == 0 ? 1 : -1) * a.m[0][i] * det3(sub);
    }
    return det;
}

static bool inverse(const Matrix4& a, Matrix4& r) {
    float det = det4(a);
    if (std::fabs(det) < 1e-10) return false;
    Matrix4 adj;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            Matrix4 sub;
            std::memset(&sub, 0, sizeof sub);
            int si = 0;
            for (int k = 0; k < 4; k++) {
                if (k == i) continue;
                int sj = 0;
                for (int l = 0; l < 4; l++) {
                    if (l == j) continue;
                    sub.m[si][sj++] = a.m[k][l];
                }
                si++;
            }
            float c = det3(sub);
            if ((i + j) % 2 != 0) c = -c;
            adj.m[j][i] = c;
        }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) r.m[i][j] = adj.m[i][j] / det;
    return true;
}

void make_render_params(const Scene& sc, int width, int height, float fov, rt_render_params& p) {
    std::memset(&p, 0, sizeof p);
    p.abi_version = RT580_ABI_VERSION;
    p.width = width;
    p.height = height;
    p.depth = 4;
    p.ao_samples = 128;
    p.ao_enabled = 1;
    p.rng_engine = RT_RNG_MINSTD_RAND0;
    p.rng_seed = 1;
    p.row_begin = 0;
    p.row_end = height;
    p.row_step = 1;
    // InitializeRenderer (Raytracer.cpp:895-915) + CalculateViewMatrix (:861-870)
    rv3 n = v3_normalize(v3_sub(sc.camera.from, sc.camera.to));
    rv3 up = v3(0, 1, 0);
    rv3 u = v3_normalize(v3_cross(up, n));
    rv3 v = v3_normalize(v3_cross(n, u));
    rv3 r = sc.camera.from;
    Matrix4 view;
    view.m[0][0] = u.x; view.m[0][1] = u.y; view.m[0][2] = u.z; view.m[0][3] = -v3_dot(r, u);
    view.m[1][0] = v.x; view.m[1][1] = v.y; view.m[1][2] = v.z; view.m[1][3] = -v3_dot(r, v);
    view.m[2][0] = n.x; view.m[2][1] = n.y; view.m[2][2] = n.z; view.m[2][3] = -v3_dot(r, n);
    view.m[3][0] = 0; view.m[3][1] = 0; view.m[3][2] = 0; view.m[3][3] = 1;
    // GenerateRay inverts the view matrix per pixel (Raytracer.cpp:849-851): same value each time.
    Matrix4 inv;
    p.view_inverse_ok = inverse(view, inv) ? 1 : 0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) p.view_inv[i * 3 + j] = p.view_inverse_ok ? inv.m[i][j] : 0.0f;
    set3(p.cam_from, sc.camera.from);
    float aspect = (float)width / (float)height;          // Raytracer.cpp:836
    double tn = std::tan((double)to_radian(fov / 2));      // Raytracer.cpp:839-840
    p.ndc_kx = aspect * tn;
    p.ndc_ky = tn;
    p.ao_angle_max = (float)(2 * kPI);                     // uniform_real_distribution(0, 2*PI), :270
}

}  // namespace rt580
