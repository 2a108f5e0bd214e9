// oracle_loader.cpp -- SceneLoader.FromFile restatement (SceneLoader.cs:112-440),
// MatrixStack (MatrixStack.cs) and Cube (Raytracing/Objects/Cube.cs).
// TEST INFRASTRUCTURE (see oracle.h).
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <sstream>
#include <stdexcept>

#include "oracle_scene.h"

namespace orc {

namespace {

struct LoadError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

bool is_word(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_'; }
bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; }

// Emulates lineRegex (SceneLoader.cs:38): cmd word, params separated by whitespace with an
// optional comma that must be followed by whitespace, optional trailing '#' comment.
bool split_line(const std::string& line, std::string& cmd, std::vector<std::string>& params)
{
    size_t i = 0, n = line.size();
    cmd.clear();
    params.clear();
    while (i < n && is_ws(line[i])) i++;
    if (i == n || line[i] == '#') return true;
    if (!is_word(line[i])) return false;
    while (i < n && is_word(line[i])) cmd.push_back(line[i++]);
    while (true) {
        size_t j = i;
        while (j < n && is_ws(line[j])) j++;
        if (j == n || line[j] == '#') return true;
        if (params.empty()) {
            if (j == i) return false; // needs \s+ before the first parameter
        } else {
            bool comma = false;
            if (line[j] == ',') {
                comma = true;
                j++;
                size_t k = j;
                while (j < n && is_ws(line[j])) j++;
                if (j == k) return false; // comma must be followed by whitespace
            } else if (j == i) {
                return false;
            }
            (void)comma;
            if (j == n || line[j] == '#') return false; // dangling comma
        }
        if (line[j] == ',') return false;
        std::string tok;
        while (j < n && !is_ws(line[j]) && line[j] != ',' && line[j] != '#') tok.push_back(line[j++]);
        params.push_back(tok);
        i = j;
    }
}

double parse_dbl(const std::string& s)
{
    if (s.empty() || s.find_first_of("xX") != std::string::npos) throw LoadError("bad number " + s);
    const char* b = s.c_str();
    char* e = nullptr;
    errno = 0;
    double v = std::strtod(b, &e);
    if (e == b || *e != 0) throw LoadError("bad number " + s);
    return v;
}
int parse_int(const std::string& s)
{
    const char* b = s.c_str();
    char* e = nullptr;
    errno = 0;
    long v = std::strtol(b, &e, 10);
    if (e == b || *e != 0 || errno || v > 2147483647L || v < -2147483647L - 1) throw LoadError("bad integer " + s);
    return (int)v;
}

struct Cube {
    V4 pos, size;
    // Cube.CreateRect / Triangle.CreateRectangle (Cube.cs:54-59, Triangle.cs:13-20)
    static Prim rect(V4 pos, V4 up, V4 norm, double dist, double width, double height)
    {
        Ray upr = ray_directional(pos + (norm * (dist / 2)), up);
        V4 side = normalize(cross(upr.d, norm));
        V4 v0 = upr.o + (upr.d * (-height / 2)) + (side * (-width / 2));
        V4 v1 = v0 + (side * width);
        V4 v2 = v0 + (upr.d * height);
        Prim p;
        p.kind = kTri;
        p.vp[0] = v0;
        p.vp[1] = v1;
        p.vp[2] = v2;
        for (int i = 0; i < 3; i++) p.vn[i] = normalize(v4(0, 0, 1, 0));
        p.recalc_triangle();
        p.mirror = true;
        return p;
    }
    std::vector<Prim> children(int sides) const // Cube.GetChildren (Cube.cs:90-116)
    {
        std::vector<Prim> out;
        if (sides & 1) out.push_back(rect(pos, v4(0, 0, 1, 0), v4(1, 0, 0, 0), size.x, size.y, size.z));
        if (sides & 2) out.push_back(rect(pos, v4(0, 0, -1, 0), v4(-1, 0, 0, 0), size.x, size.y, size.z));
        if (sides & 4) out.push_back(rect(pos, v4(0, 0, 1, 0), v4(0, 1, 0, 0), size.y, size.x, size.z));
        if (sides & 8) out.push_back(rect(pos, v4(0, 0, -1, 0), v4(0, -1, 0, 0), size.y, size.x, size.z));
        if (sides & 16) out.push_back(rect(pos, v4(0, 1, 0, 0), v4(0, 0, 1, 0), size.z, size.x, size.y));
        if (sides & 32) out.push_back(rect(pos, v4(0, -1, 0, 0), v4(0, 0, -1, 0), size.z, size.x, size.y));
        return out;
    }
};

// Cube.GetSide (Cube.cs:22-63)
int get_side(const std::string& name)
{
    if (name == "implicit") return 0;
    if (name == "all") return 63;
    if (name.size() == 2 && name[0] == '-') {
        switch (name[1]) {
        case 'x': return 2;
        case 'y': return 8;
        case 'z': return 32;
        }
    }
    char axis = ' ';
    if (name.size() == 2 && name[0] == '+') axis = name[1];
    else if (name.size() == 1) axis = name[0];
    switch (axis) {
    case 'x': return 1;
    case 'y': return 4;
    case 'z': return 16;
    }
    throw LoadError("Unknown Cube side name " + name);
}

void transform_prim(Prim& p, const M4& fwd, const M4& inv)
{
    if (p.kind == kTri) { // Triangle.Transform (Triangle.cs:68-74), Vertex.Transformed (Vertex.cs:27-30)
        for (int i = 0; i < 3; i++) {
            p.vp[i] = mvmul(fwd, p.vp[i]);
            p.vn[i] = normalize(normalize(mvmul(fwd, p.vn[i])));
        }
        p.recalc_triangle();
    } else if (p.kind == kSphere) { // Sphere.Transform (Sphere.cs:29-37)
        if (!meq(fwd, identity4())) p.transformed = true;
        p.to_obj = mmul(p.to_obj, fwd);
        p.to_world = mmul(inv, p.to_world);
        p.to_normal = transpose3x3(p.to_world);
    } else { // Plane.Transform (Plane.cs:29-34)
        V4 c = mvmul(fwd, p.get_center());
        p.pnormal = normalize(mvmul(transpose3x3(inv), p.pnormal));
        p.origin_dist = dot(c, p.pnormal);
    }
}

} // namespace

bool load_scene_text(const std::string& text, Scene& sc, std::string& err)
{
    const Col placeholder = col(-1);
    // Camera state
    double image_plane = 0, dof_amount = 0, focal_length = 0;
    V4 focal_point = v4(0, 0, 0, 0);
    // Primitive state (SceneLoader.cs:128-139)
    bool have_obj = false;
    Cube obj{};
    std::vector<Prim> prims;
    bool two_sided = true, invert = false;
    Col emission = placeholder, diffuse = placeholder, specular = placeholder, refraction = placeholder;
    double shininess = -1, refraction_index = -1;
    std::vector<M4> stack{identity4()}, inv_stack{identity4()};
    std::vector<V4> vertices;
    std::vector<std::pair<V4, V4>> vnormals;

    std::istringstream in(text);
    std::string line, cmd;
    std::vector<std::string> params;
    int line_num = 1;
    while (std::getline(in, line)) {
        if (!split_line(line, cmd, params)) {
            err = "Line did not match expected format. (line " + std::to_string(line_num) + ")";
            return false;
        }
        if (!cmd.empty()) {
            for (auto& c : cmd) c = (char)std::tolower((unsigned char)c);
            size_t pi = 0;
            auto has = [&]() { return pi < params.size(); };
            auto next = [&]() -> const std::string& {
                if (!has()) throw LoadError("A parameter was missing from a command.");
                return params[pi++];
            };
            auto next_dbl = [&]() { return parse_dbl(next()); };
            auto next_int = [&]() { return parse_int(next()); };
            auto next_vec = [&](double w) {
                double x = next_dbl(), y = next_dbl(), z = next_dbl();
                return v4(x, y, z, w);
            };
            auto transf = [&](V4 v) { return mvmul(stack.back(), v); };
            auto next_rgb = [&]() {
                double r = next_dbl(), g = next_dbl(), b = next_dbl();
                return Col{r, g, b};
            };
            auto next_bool = [&]() {
                const std::string& s = next();
                return s == "1" || s == "true" || s == "yes" || s == "y";
            };
            try {
                bool add_cam = false;
                Camera cam;
                if (cmd == "size") {
                    sc.width = next_int();
                    sc.height = next_int();
                } else if (cmd == "background") {
                    sc.background = next_rgb();
                    sc.background_alpha = next_dbl();
                } else if (cmd == "ambient") {
                    const std::string& k = next();
                    if (k == "miss") sc.ambient = placeholder;
                    else if (k == "color") sc.ambient = next_rgb();
                    else throw LoadError("Unknown ambient type " + k);
                } else if (cmd == "recursion" || cmd == "bounce") {
                    sc.recursion = next_int();
                } else if (cmd == "debug") {
                    const std::string& k = next();
                    if (k == "geom") sc.debug_geom = true;
                    else if (k == "off") sc.debug_geom = false;
                    else throw LoadError("Unknown debug type " + k);
                } else if (cmd == "dof") {
                    image_plane = next_dbl();
                    dof_amount = next_dbl();
                    const std::string& k = next();
                    if (k == "at") {
                        focal_point = transf(next_vec(1));
                        focal_length = 0;
                    } else if (k == "to") {
                        focal_length = next_dbl();
                        focal_point = v4(0, 0, 0, 0);
                    } else if (k == "camera") {
                        focal_length = 0;
                        focal_point = v4(0, 0, 0, 0);
                    } else {
                        throw LoadError("Unknown dof focal command " + k);
                    }
                } else if (cmd == "camera" || cmd == "frustum" || cmd == "orthographic") {
                    V4 pos = next_vec(1);
                    V4 look_at = next_vec(1);
                    V4 up = transf(next_vec(0) + pos);
                    pos = transf(pos);
                    up = up - pos;
                    cam.kind = (cmd == "orthographic") ? 1 : 0;
                    cam.init_pos = cam.position = pos;
                    cam.init_look_at = cam.look_at = look_at;
                    cam.init_up = cam.up = up;
                    double v = next_dbl();
                    if (cam.kind == 1) cam.size_mult = v;
                    else cam.fov_y = v * kRad2Deg; // Consts.toRadians
                    add_cam = true;
                } else if (cmd == "twosided") {
                    two_sided = next_bool();
                } else if (cmd == "invert") {
                    invert = next_bool();
                } else if (cmd == "emission") {
                    emission = next_rgb();
                } else if (cmd == "diffuse") {
                    diffuse = next_rgb();
                } else if (cmd == "specular") {
                    specular = next_rgb();
                } else if (cmd == "shininess") {
                    shininess = next_dbl();
                    if (has()) shininess = std::pow(shininess, parse_dbl(next()));
                } else if (cmd == "refraction") {
                    const std::string& k = next();
                    if (k == "off") {
                        refraction = placeholder;
                        refraction_index = -1;
                    } else {
                        double r = parse_dbl(k);
                        double g = next_dbl(), b = next_dbl();
                        refraction = Col{r, g, b};
                        refraction_index = next_dbl();
                    }
                } else if (cmd == "translate") {
                    V4 t = next_vec(0);
                    stack.back() = mmul(stack.back(), m_translate(t.x, t.y, t.z));
                    inv_stack.back() = mmul(m_translate(-t.x, -t.y, -t.z), inv_stack.back());
                } else if (cmd == "scale") {
                    V4 s = next_vec(0);
                    stack.back() = mmul(stack.back(), m_scale(s.x, s.y, s.z));
                    inv_stack.back() = mmul(m_scale(1 / s.x, 1 / s.y, 1 / s.z), inv_stack.back());
                } else if (cmd == "rotate") {
                    V4 axis = next_vec(0);
                    double angle = next_dbl();
                    stack.back() = mmul(stack.back(), m_rotate(angle * kRad2Deg, normalize(axis)));
                    inv_stack.back() = mmul(m_rotate(-(angle * kRad2Deg), normalize(axis)), inv_stack.back());
                } else if (cmd == "pushtransform") {
                    stack.push_back(stack.back());
                    inv_stack.push_back(inv_stack.back());
                } else if (cmd == "poptransform") {
                    if (stack.size() <= 1) throw LoadError("Stack empty.");
                    stack.pop_back();
                    inv_stack.pop_back();
                } else if (cmd == "sphere") {
                    Prim p;
                    p.kind = kSphere;
                    p.center = next_vec(1);
                    p.radius = next_dbl();
                    p.radius_sqr = p.radius * p.radius;
                    prims.push_back(p);
                } else if (cmd == "plane") {
                    Prim p;
                    p.kind = kPlane;
                    p.origin_dist = next_dbl();
                    p.pnormal = normalize(next_vec(0));
                    prims.push_back(p);
                } else if (cmd == "vertex") {
                    vertices.push_back(next_vec(1));
                } else if (cmd == "tri") {
                    int i0 = next_int(), i1 = next_int(), i2 = next_int();
                    if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= (int)vertices.size() || i1 >= (int)vertices.size() ||
                        i2 >= (int)vertices.size())
                        throw LoadError("Index was out of range.");
                    bool mirror = has() && next() == "mirrored";
                    Prim p;
                    p.kind = kTri;
                    p.vp[0] = vertices[i0];
                    p.vp[1] = vertices[i1];
                    p.vp[2] = vertices[i2];
                    for (int k = 0; k < 3; k++) p.vn[k] = normalize(v4(0, 0, 1, 0));
                    p.recalc_triangle();
                    p.mirror = mirror;
                    prims.push_back(p);
                } else if (cmd == "vertexnormal") {
                    V4 pos = next_vec(1);
                    V4 nrm = normalize(next_vec(0));
                    vnormals.push_back({pos, nrm});
                } else if (cmd == "trinormal") {
                    int i0 = next_int(), i1 = next_int(), i2 = next_int();
                    if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= (int)vnormals.size() || i1 >= (int)vnormals.size() ||
                        i2 >= (int)vnormals.size())
                        throw LoadError("Index was out of range.");
                    Prim p;
                    p.kind = kTri;
                    p.has_normals = true;
                    int idx[3] = {i0, i1, i2};
                    for (int k = 0; k < 3; k++) {
                        p.vp[k] = vnormals[idx[k]].first;
                        p.vn[k] = vnormals[idx[k]].second;
                    }
                    p.normal = v4(0, 0, 0, 0);
                    p.recalc_triangle();
                    prims.push_back(p);
                } else if (cmd == "cube") {
                    V4 pos = next_vec(1);
                    V4 size = next_vec(0);
                    obj = Cube{pos, size};
                    have_obj = true;
                    if (has()) {
                        const std::string& k = next();
                        int sides;
                        if (k == "all") {
                            sides = 63;
                        } else if (k == "only") {
                            sides = 0;
                            while (has()) sides |= get_side(next());
                        } else if (k == "not") {
                            sides = 63;
                            while (has()) sides &= ~get_side(next());
                        } else {
                            throw LoadError("Unknown option provided for cube construction: " + k);
                        }
                        for (auto& p : obj.children(sides)) prims.push_back(p);
                    }
                } else if (cmd == "instance") {
                    if (!have_obj) throw LoadError("Object reference not set to an instance of an object.");
                    while (has())
                        for (auto& p : obj.children(get_side(next()))) prims.push_back(p);
                } else {
                    // maxverts, maxvertnorms and unknown commands: ignored (SceneLoader.cs:362-369)
                }

                if (add_cam) { // SceneLoader.cs:372-386
                    cam.image_plane = image_plane;
                    cam.dof_amount = dof_amount;
                    if (!eq3(focal_point, v4(0, 0, 0, 0))) cam.focal_length = length(focal_point - cam.position);
                    else if (focal_length != 0) cam.focal_length = focal_length;
                    else cam.focal_length = length(cam.init_look_at - cam.position);
                    sc.cameras.push_back(cam);
                }
                for (Prim& p : prims) { // SceneLoader.cs:388-413
                    p.two_sided = two_sided;
                    p.invert = invert;
                    if (!ceq(emission, placeholder)) p.emission = emission;
                    if (!ceq(diffuse, placeholder)) p.diffuse = diffuse;
                    if (!ceq(specular, placeholder)) p.specular_raw = specular;
                    if (shininess != -1) p.shininess = shininess;
                    if (!ceq(refraction, placeholder)) {
                        p.refraction_raw = refraction;
                        p.refractive_index = refraction_index;
                    }
                    transform_prim(p, stack.back(), inv_stack.back());
                    p.id = (int)sc.prims.size();
                    sc.prims.push_back(p);
                }
                prims.clear();
            } catch (const std::exception& e) {
                err = "Error while parsing command " + cmd + " on line " + std::to_string(line_num) + ": " + e.what();
                return false;
            }
        }
        line_num++;
    }
    return true;
}

} // namespace orc
