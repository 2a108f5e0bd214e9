// oracle_scene.h -- primitives, scene, BVH and tracer of the CPU oracle.
// TEST INFRASTRUCTURE (see oracle.h).
#pragma once
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "oracle_math.h"

namespace orc {

enum PrimKind { kTri = 0, kSphere = 1, kPlane = 2 };

// Primitive + Triangle / Sphere / Plane state (Primitives/*.cs).
struct Prim {
    int kind = kTri;
    int id = -1;
    bool two_sided = true, invert = false;
    Col emission = col(0), diffuse = col(0), specular_raw = col(0), refraction_raw = col(0);
    double shininess = 100; // Primitive.cs:31
    double refractive_index = 0;
    // Triangle (Triangle.cs:22-29)
    V4 vp[3], vn[3];
    bool mirror = false, has_normals = false;
    V4 e01, e02, normal;
    // Sphere (Sphere.cs:12-21)
    V4 center;
    double radius = 0, radius_sqr = 0;
    bool transformed = false;
    M4 to_obj = identity4(), to_world = identity4(), to_normal = identity4();
    // Plane (Plane.cs:13-14)
    V4 pnormal;
    double origin_dist = 0;

    bool reflective() const { return shininess > 0; }                 // Primitive.cs:107
    Col specular() const { return reflective() ? specular_raw : col(0); }   // :111-119
    Col refraction() const { return reflective() ? refraction_raw : col(0); } // :121-129
    V4 get_center() const;
    double max_center_distance(V4 dir) const;
    void recalc_triangle(); // Triangle.Recalculate (Triangle.cs:54-66)
};

struct Camera {
    int kind = 0; // 0 frustum, 1 ortho
    V4 init_pos, init_look_at, init_up;
    V4 position, look_at, up;
    double fov_y = 0, size_mult = 0;
    double image_plane = 0, dof_amount = 0, focal_length = 0;
    // InitRender state
    double w2 = 0, h2 = 0, tan_x = 0, tan_y = 0, h_mult = 0, v_mult = 0;
    V4 look, side, up_r;
    void init_render(int w, int h);
    Ray get_ray(double x, double y) const;
};

struct AABB {
    V4 mn, mx, size, ctr;
};
AABB aabb_make(V4 mn, V4 mx);
bool aabb_equals(const AABB& a, const AABB& b);
double aabb_sa(const AABB& a);

// BVH<T> node (Acceleration/BVH.cs:239-279).
struct BNode {
    bool leaf = false;
    int prim = -1;
    BNode *left = nullptr, *right = nullptr;
    AABB vol;
    bool skip = false;
    double cost_cache = -1;
    double cost(); // BVH.cs:368-400
    int child_leaves() const { return (left->leaf ? 1 : 0) + (right->leaf ? 1 : 0); }
    V4 center(const std::vector<Prim>& prims) const;
};

struct Hit {
    int prim = -1; // -1 = no hit (null)
    V4 pos{0, 0, 0, 0};
    double dist = 0;
    V4 normal{0, 0, 0, 0};
    bool inside = false;
};

struct Scene {
    int width = 0, height = 0;
    Col background = col(0);
    double background_alpha = 0;
    Col ambient = col(0);
    bool debug_geom = false;
    int current_camera = 0;
    std::vector<Camera> cameras;
    std::vector<Prim> prims;
    int recursion = 3;
    double air_ior = 1.000293;

    std::deque<BNode> pool;
    BNode* root = nullptr;
    void prepare();                  // Scene.Prepare (Scene.cs:39-49)
    Hit raytrace(const Ray& r, const Hit* skip, std::vector<struct Leaf>& scratch) const;
};

struct Leaf {
    const BNode* node;
    double near_, far_;
};

// Loader
bool load_scene_text(const std::string& text, Scene& out, std::string& err);
// Intersection (exposed for tests)
bool aabb_intersect(const AABB& b, const Ray& r, double& near_, double& far_);
int prim_dotrace(const Prim& p, const Ray& r, Hit out[2]);
Hit prim_raytrace(const Prim& p, const Ray& r, const Hit* skip);

} // namespace orc
