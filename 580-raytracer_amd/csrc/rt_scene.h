// rt_scene.h — host-side scene ingest and flattening for the HIP path.
//
// load_scene_json() restates LoadSceneJSON / LoadMesh (Raytracer.cpp:589-779)
// and produces the reference's in-memory scene; pack_scene() then flattens it
// into the rt_prim / rt_prim_shade / rt_material / rt_light arrays of rt580.h,
// doing once on the host every ray-invariant computation the reference repeats
// per ray (ComputeModelMatrix per shape per IntersectScene call, the world-space
// triangle vertices, plane normals, D and total areas per triangle test), with
// the reference's float arithmetic. make_render_params() restates
// InitializeRenderer (Raytracer.cpp:895-915) and the GenerateRay constants
// (Raytracer.cpp:832-858).
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../../include/rt580.h"
#include "rt_math.h"

namespace rt580 {

struct Matrix4 {
    float m[4][4];
};

struct Material {  // Raytracer.h:442-463 defaults
    rv3 cs = v3(1.0f, 1.0f, 1.0f);
    float ka = 0.5f, kd = 0.75f, ks = 0.95f, kt = 0.95f, ior = 2.5f, spec_exp = 32.0f;
};

struct Triangle {
    rv3 pos[3];
    rv3 nrm[3];
};

struct Mesh {
    int type = RT_PRIM_TRIANGLE;  // value-initialised Mesh (Raytracer.cpp:605): RT_POLYGON
    std::vector<Triangle> tris;
    float radius = 0.0f;
};

struct Shape {
    std::string id, geometry;
    Material material;
    rv3 scale = v3(1, 1, 1), rotation = v3(0, 0, 0), translation = v3(0, 0, 0);
    int mesh = -1;
};

struct Light {
    int kind = RT_LIGHT_AMBIENT;
    rv3 color = v3(0, 0, 0), position = v3(0, 0, 0), direction = v3(0, 0, 0);
    float intensity = 0.0f;
};

struct Camera {
    rv3 from = v3(0, 0, 0), to = v3(0, 0, 0);
};

struct Scene {
    std::vector<Shape> shapes;
    std::vector<Mesh> meshes;
    std::map<std::string, int> mesh_index;
    std::vector<Light> lights;
    Camera camera;
};

struct PackedScene {
    std::vector<rt_prim> prims;
    std::vector<rt_prim_shade> shade;
    std::vector<rt_material> materials;
    std::vector<rt_light> lights;
    int n_triangles = 0, n_spheres = 0;
};

// Returns RT_SUCCESS / RT_FAILURE; `error` receives a message.
int load_scene_json(const std::string& assets_root, const std::string& scene_path, Scene& out,
                    std::string& error);
Matrix4 compute_model_matrix(const Shape& s);  // Raytracer.cpp:528-586
void pack_scene(const Scene& s, PackedScene& out);
// InitializeRenderer + GenerateRay constants; fov 60 (Raytracer.cpp:786).
void make_render_params(const Scene& s, int width, int height, float fov, rt_render_params& p);

}  // namespace rt580
