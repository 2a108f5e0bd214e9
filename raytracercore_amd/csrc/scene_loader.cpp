// scene_loader.cpp -- scene text -> rt_prim / rt_camera / rt_scene_params.
//
// Restates SceneLoader.FromFile (SceneLoader.cs:112-440) with MatrixStack
// (MatrixStack.cs:10-30), Cube (Raytracing/Objects/Cube.cs:22-116), Triangle /
// Sphere / Plane construction and Transform (Triangle.cs:13-74, Sphere.cs:23-37,
// Plane.cs:18-34) and Vertex (Vertex.cs).  The C# host keeps its own loader; this one lets
// non-.NET hosts, the tests and the benchmark drive the library from the same scene files.
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace rtc {
namespace {

struct Mat {
    double d[16];
};
Mat ident()
{
    Mat m{};
    m.d[0] = m.d[5] = m.d[10] = m.d[15] = 1;
    return m;
}
// Mat4x4D * Mat4x4D: Vector<double>.Dot(row, column) in (p0+p1)+(p2+p3) order (Mat4x4D.cs:99-124)
Mat mat_mul(const Mat& a, const Mat& b)
{
    Mat r;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            const double* row = a.d + 4 * y;
            double p0 = row[0] * b.d[x], p1 = row[1] * b.d[4 + x], p2 = row[2] * b.d[8 + x], p3 = row[3] * b.d[12 + x];
            r.d[4 * y + x] = (p0 + p1) + (p2 + p3);
        }
    return r;
}
bool mat_eq(const Mat& a, const Mat& b)
{
    for (int i = 0; i < 16; i++)
        if (!(a.d[i] == b.d[i])) return false;
    return true;
}
Mat transpose3(const Mat& m)
{
    Mat r{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.d[4 * i + j] = m.d[4 * j + i];
    r.d[15] = 1;
    return r;
}
Mat translate(double x, double y, double z)
{
    Mat m = ident();
    m.d[3] = x;
    m.d[7] = y;
    m.d[11] = z;
    return m;
}
Mat scale_m(double x, double y, double z)
{
    Mat m{};
    m.d[0] = x;
    m.d[5] = y;
    m.d[10] = z;
    m.d[15] = 1;
    return m;
}
Mat rotate(double angle, Vec4d a) // MatrixTransforms.Rotate (MatrixTransforms.cs:25-37)
{
    double c = cos(angle), s = sin(angle), k = 1 - c;
    Mat m{};
    m.d[0] = c + a.x * a.x * k;       m.d[1] = a.x * a.y * k - a.z * s; m.d[2] = a.x * a.z * k + a.y * s;
    m.d[4] = a.y * a.x * k + a.z * s; m.d[5] = c + a.y * a.y * k;       m.d[6] = a.y * a.z * k - a.x * s;
    m.d[8] = a.z * a.x * k - a.y * s; m.d[9] = a.z * a.y * k + a.x * s; m.d[10] = c + a.z * a.z * k;
    m.d[15] = 1;
    return m;
}

const double kPi = 3.14159265358979323846;
const double kRad2Deg = kPi / 180.0; // Consts.RAD2DEG (Consts.cs:9)

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

rt_vec4d to_abi(Vec4d v) { return rt_vec4d{v.x, v.y, v.z, v.w}; }
Vec4d from_abi(rt_vec4d v) { return Vec4d{v.x, v.y, v.z, v.w}; }

// Triangle.Recalculate's vertex normals for plain triangles: WithNormal(Normal) normalises.
void finish_triangle(rt_prim& p)
{
    if (p.flags & RT_FLAG_HASNORMALS) return;
    Vec4d v0 = from_abi(p.p[0]), e1 = sub(from_abi(p.p[1]), v0), e2 = sub(from_abi(p.p[2]), v0);
    Vec4d n = normalize_v(normalize_v(cross_s(e1, e2)));
    for (int k = 0; k < 3; k++) p.n[k] = to_abi(n);
}

rt_prim new_prim(int kind)
{
    rt_prim p;
    std::memset(&p, 0, sizeof p);
    p.kind = kind;
    p.shininess = 100; // Primitive() (Primitive.cs:24-32)
    Mat I = ident();
    std::memcpy(p.to_obj, I.d, sizeof I.d);
    std::memcpy(p.to_world, I.d, sizeof I.d);
    std::memcpy(p.to_normal, I.d, sizeof I.d);
    return p;
}

rt_prim make_triangle(Vec4d a, Vec4d b, Vec4d c, bool mirror)
{
    rt_prim p = new_prim(RT_PRIM_TRIANGLE);
    p.p[0] = to_abi(a);
    p.p[1] = to_abi(b);
    p.p[2] = to_abi(c);
    if (mirror) p.flags |= RT_FLAG_MIRROR;
    finish_triangle(p);
    return p;
}

// Cube.CreateRect -> Triangle.CreateRectangle (Cube.cs:54-59, Triangle.cs:13-20)
rt_prim cube_face(Vec4d pos, Vec4d up, Vec4d norm, double dist, double width, double height)
{
    Vec4d o = add(pos, scale(norm, dist / 2));
    Vec4d u = normalize_v(up);
    Vec4d side = normalize_v(cross_s(u, norm));
    Vec4d v0 = add(add(o, scale(u, -height / 2)), scale(side, -width / 2));
    Vec4d v1 = add(v0, scale(side, width));
    Vec4d v2 = add(v0, scale(u, height));
    return make_triangle(v0, v1, v2, true);
}

void cube_children(Vec4d pos, Vec4d size, int sides, std::vector<rt_prim>& out) // Cube.GetChildren (:90-116)
{
    if (sides & 1) out.push_back(cube_face(pos, v4d(0, 0, 1, 0), v4d(1, 0, 0, 0), size.x, size.y, size.z));
    if (sides & 2) out.push_back(cube_face(pos, v4d(0, 0, -1, 0), v4d(-1, 0, 0, 0), size.x, size.y, size.z));
    if (sides & 4) out.push_back(cube_face(pos, v4d(0, 0, 1, 0), v4d(0, 1, 0, 0), size.y, size.x, size.z));
    if (sides & 8) out.push_back(cube_face(pos, v4d(0, 0, -1, 0), v4d(0, -1, 0, 0), size.y, size.x, size.z));
    if (sides & 16) out.push_back(cube_face(pos, v4d(0, 1, 0, 0), v4d(0, 0, 1, 0), size.z, size.x, size.y));
    if (sides & 32) out.push_back(cube_face(pos, v4d(0, -1, 0, 0), v4d(0, 0, -1, 0), size.z, size.x, size.y));
}

int side_bits(const std::string& s) // Cube.GetSide (Cube.cs:22-63)
{
    if (s == "implicit") return 0;
    if (s == "all") return 63;
    if (s.size() == 2 && s[0] == '-') {
        if (s[1] == 'x') return 2;
        if (s[1] == 'y') return 8;
        if (s[1] == 'z') return 32;
    }
    char a = (s.size() == 2 && s[0] == '+') ? s[1] : (s.size() == 1 ? s[0] : ' ');
    if (a == 'x') return 1;
    if (a == 'y') return 4;
    if (a == 'z') return 16;
    throw ParseError("Unknown Cube side name " + s + ".");
}

void apply_transform(rt_prim& p, const Mat& fwd, const Mat& inv) // Primitive.Transform overrides
{
    if (p.kind == RT_PRIM_TRIANGLE) {
        for (int k = 0; k < 3; k++) {
            p.p[k] = to_abi(mat_vec(fwd.d, from_abi(p.p[k])));
            p.n[k] = to_abi(normalize_v(normalize_v(mat_vec(fwd.d, from_abi(p.n[k])))));
        }
        finish_triangle(p);
    } else if (p.kind == RT_PRIM_SPHERE) {
        if (!mat_eq(fwd, ident())) p.flags |= RT_FLAG_TRANSFORMED;
        Mat to_obj, to_world;
        std::memcpy(to_obj.d, p.to_obj, sizeof to_obj.d);
        std::memcpy(to_world.d, p.to_world, sizeof to_world.d);
        to_obj = mat_mul(to_obj, fwd);
        to_world = mat_mul(inv, to_world);
        Mat to_normal = transpose3(to_world);
        std::memcpy(p.to_obj, to_obj.d, sizeof to_obj.d);
        std::memcpy(p.to_world, to_world.d, sizeof to_world.d);
        std::memcpy(p.to_normal, to_normal.d, sizeof to_normal.d);
    } else {
        Vec4d n = from_abi(p.p[0]);
        Vec4d c = mat_vec(fwd.d, add(v4d(0, 0, 0, 1), scale(n, p.radius)));
        n = normalize_v(mat_vec(transpose3(inv).d, n));
        p.p[0] = to_abi(n);
        p.radius = dot_s(c, n);
    }
}

// lineRegex (SceneLoader.cs:38) as a scanner.
bool tokenize(const std::string& line, std::string& cmd, std::vector<std::string>& args)
{
    auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; };
    auto word = [](char c) { return std::isalnum((unsigned char)c) || c == '_'; };
    size_t i = 0, n = line.size();
    cmd.clear();
    args.clear();
    while (i < n && ws(line[i])) i++;
    if (i == n || line[i] == '#') return true;
    if (!word(line[i])) return false;
    while (i < n && word(line[i])) cmd += line[i++];
    for (;;) {
        size_t j = i;
        while (j < n && ws(line[j])) j++;
        if (j == n || line[j] == '#') return true;
        if (!args.empty() && line[j] == ',') {
            size_t k = ++j;
            while (j < n && ws(line[j])) j++;
            if (j == k || j == n || line[j] == '#') return false;
        } else if (j == i) {
            return false;
        }
        if (line[j] == ',') return false;
        size_t s = j;
        while (j < n && !ws(line[j]) && line[j] != ',' && line[j] != '#') j++;
        args.emplace_back(line, s, j - s);
        i = j;
    }
}

double to_double(const std::string& s)
{
    if (s.find_first_of("xX") != std::string::npos) throw ParseError("Input string was not in a correct format.");
    char* e = nullptr;
    double v = std::strtod(s.c_str(), &e);
    if (s.empty() || *e) throw ParseError("Input string was not in a correct format.");
    return v;
}
int to_int(const std::string& s)
{
    char* e = nullptr;
    errno = 0;
    long v = std::strtol(s.c_str(), &e, 10);
    if (s.empty() || *e || errno || v > 2147483647L || v < -2147483648L)
        throw ParseError("Input string was not in a correct format.");
    return (int)v;
}

} // namespace

bool parse_scene_text(const char* text, ParsedScene& out, std::string& err)
{
    const rt_color placeholder{-1, -1, -1};
    auto same = [](rt_color a, rt_color b) { return a.r == b.r && a.g == b.g && a.b == b.b; };
    out = ParsedScene{};
    std::memset(&out.params, 0, sizeof out.params);
    out.params.recursion = 3;           // Scene.Recursion (Scene.cs:33)
    out.params.air_ior = 1.000293;      // Scene.AirRefractiveIndex (Scene.cs:35)
    out.background = rt_color{0, 0, 0};

    double image_plane = 0, dof_amount = 0, focal_length = 0;
    Vec4d focal_point{0, 0, 0, 0};
    bool have_cube = false;
    Vec4d cube_pos{0, 0, 0, 0}, cube_size{0, 0, 0, 0};
    std::vector<rt_prim> pending;
    bool two_sided = true, invert = false;
    rt_color emission = placeholder, diffuse = placeholder, specular = placeholder, refraction = placeholder;
    double shininess = -1, refraction_index = -1;
    std::vector<Mat> stack{ident()}, inv_stack{ident()};
    std::vector<Vec4d> vertices;
    std::vector<std::pair<Vec4d, Vec4d>> vnormals;

    std::istringstream in(text ? text : "");
    std::string line, cmd;
    std::vector<std::string> args;
    for (int line_no = 1; std::getline(in, line); line_no++) {
        if (!tokenize(line, cmd, args)) {
            err = "Line did not match expected format. (line " + std::to_string(line_no) + ")";
            return false;
        }
        if (cmd.empty()) continue;
        for (char& c : cmd) c = (char)std::tolower((unsigned char)c);
        size_t ai = 0;
        auto more = [&] { return ai < args.size(); };
        auto next = [&]() -> const std::string& {
            if (!more()) throw ParseError("A parameter was missing from a command.");
            return args[ai++];
        };
        auto num = [&] { return to_double(next()); };
        auto vec = [&](double w) {
            double x = num(), y = num(), z = num();
            return v4d(x, y, z, w);
        };
        auto rgb = [&] {
            double r = num(), g = num(), b = num();
            return rt_color{r, g, b};
        };
        auto flag = [&] {
            const std::string& s = next();
            return s == "1" || s == "true" || s == "yes" || s == "y";
        };
        try {
            bool new_camera = false;
            rt_camera cam;
            std::memset(&cam, 0, sizeof cam);
            if (cmd == "size") {
                out.params.width = to_int(next());
                out.params.height = to_int(next());
            } else if (cmd == "background") {
                out.background = rgb();
                out.background_alpha = num();
            } else if (cmd == "ambient") {
                const std::string& k = next();
                if (k == "miss") out.params.ambient = placeholder;
                else if (k == "color") out.params.ambient = rgb();
                else throw ParseError("Unknown ambient type " + k + ".");
            } else if (cmd == "recursion" || cmd == "bounce") {
                out.params.recursion = to_int(next());
            } else if (cmd == "debug") {
                const std::string& k = next();
                if (k == "geom") out.params.debug_geom = 1;
                else if (k == "off") out.params.debug_geom = 0;
                else throw ParseError("Unknown debug type " + k + ".");
            } else if (cmd == "dof") {
                image_plane = num();
                dof_amount = num();
                const std::string& k = next();
                if (k == "at") {
                    focal_point = mat_vec(stack.back().d, vec(1));
                    focal_length = 0;
                } else if (k == "to") {
                    focal_length = num();
                    focal_point = v4d(0, 0, 0, 0);
                } else if (k == "camera") {
                    focal_length = 0;
                    focal_point = v4d(0, 0, 0, 0);
                } else {
                    throw ParseError("Unknown dof focal command " + k + ".");
                }
            } else if (cmd == "camera" || cmd == "frustum" || cmd == "orthographic") {
                Vec4d pos = vec(1), look_at = vec(1);
                Vec4d up = mat_vec(stack.back().d, add(vec(0), pos));
                pos = mat_vec(stack.back().d, pos);
                up = sub(up, pos);
                cam.kind = cmd == "orthographic" ? RT_CAMERA_ORTHO : RT_CAMERA_FRUSTUM;
                cam.position = to_abi(pos);
                cam.look_at = to_abi(look_at);
                cam.up = to_abi(up);
                double v = num();
                if (cam.kind == RT_CAMERA_ORTHO) cam.size_mult = v;
                else cam.fov_y = v * kRad2Deg;
                new_camera = true;
            } else if (cmd == "twosided") {
                two_sided = flag();
            } else if (cmd == "invert") {
                invert = flag();
            } else if (cmd == "emission") {
                emission = rgb();
            } else if (cmd == "diffuse") {
                diffuse = rgb();
            } else if (cmd == "specular") {
                specular = rgb();
            } else if (cmd == "shininess") {
                shininess = num();
                if (more()) shininess = pow(shininess, to_double(next()));
            } else if (cmd == "refraction") {
                const std::string& k = next();
                if (k == "off") {
                    refraction = placeholder;
                    refraction_index = -1;
                } else {
                    double r = to_double(k), g = num(), b = num();
                    refraction = rt_color{r, g, b};
                    refraction_index = num();
                }
            } else if (cmd == "translate") {
                Vec4d t = vec(0);
                stack.back() = mat_mul(stack.back(), translate(t.x, t.y, t.z));
                inv_stack.back() = mat_mul(translate(-t.x, -t.y, -t.z), inv_stack.back());
            } else if (cmd == "scale") {
                Vec4d s = vec(0);
                stack.back() = mat_mul(stack.back(), scale_m(s.x, s.y, s.z));
                inv_stack.back() = mat_mul(scale_m(1 / s.x, 1 / s.y, 1 / s.z), inv_stack.back());
            } else if (cmd == "rotate") {
                Vec4d axis = vec(0);
                double angle = num();
                stack.back() = mat_mul(stack.back(), rotate(angle * kRad2Deg, normalize_v(axis)));
                inv_stack.back() = mat_mul(rotate(-(angle * kRad2Deg), normalize_v(axis)), inv_stack.back());
            } else if (cmd == "pushtransform") {
                stack.push_back(stack.back());
                inv_stack.push_back(inv_stack.back());
            } else if (cmd == "poptransform") {
                if (stack.size() <= 1) throw ParseError("Stack empty.");
                stack.pop_back();
                inv_stack.pop_back();
            } else if (cmd == "sphere") {
                rt_prim p = new_prim(RT_PRIM_SPHERE);
                p.p[0] = to_abi(vec(1));
                p.radius = num();
                pending.push_back(p);
            } else if (cmd == "plane") {
                rt_prim p = new_prim(RT_PRIM_PLANE);
                p.radius = num();
                p.p[0] = to_abi(normalize_v(vec(0)));
                pending.push_back(p);
            } else if (cmd == "vertex") {
                vertices.push_back(vec(1));
            } else if (cmd == "tri") {
                int idx[3];
                for (int& k : idx) {
                    k = to_int(next());
                    if (k < 0 || k >= (int)vertices.size()) throw ParseError("Index was out of range.");
                }
                bool mirror = more() && next() == "mirrored";
                pending.push_back(make_triangle(vertices[idx[0]], vertices[idx[1]], vertices[idx[2]], mirror));
            } else if (cmd == "vertexnormal") {
                Vec4d pos = vec(1);
                Vec4d nrm = normalize_v(vec(0));
                vnormals.push_back({pos, nrm});
            } else if (cmd == "trinormal") {
                int idx[3];
                for (int& k : idx) {
                    k = to_int(next());
                    if (k < 0 || k >= (int)vnormals.size()) throw ParseError("Index was out of range.");
                }
                rt_prim p = new_prim(RT_PRIM_TRIANGLE);
                p.flags |= RT_FLAG_HASNORMALS;
                for (int k = 0; k < 3; k++) {
                    p.p[k] = to_abi(vnormals[idx[k]].first);
                    p.n[k] = to_abi(vnormals[idx[k]].second);
                }
                pending.push_back(p);
            } else if (cmd == "cube") {
                cube_pos = vec(1);
                cube_size = vec(0);
                have_cube = true;
                if (more()) {
                    const std::string& k = next();
                    int sides;
                    if (k == "all") {
                        sides = 63;
                    } else if (k == "only") {
                        sides = 0;
                        while (more()) sides |= side_bits(next());
                    } else if (k == "not") {
                        sides = 63;
                        while (more()) sides &= ~side_bits(next());
                    } else {
                        throw ParseError("Unknown option provided for cube construction: " + k);
                    }
                    cube_children(cube_pos, cube_size, sides, pending);
                }
            } else if (cmd == "instance") {
                if (!have_cube) throw ParseError("Object reference not set to an instance of an object.");
                while (more()) cube_children(cube_pos, cube_size, side_bits(next()), pending);
            }
            // other commands (maxverts, output, point, directional, ...) are ignored (:362-369)

            if (new_camera) { // SceneLoader.cs:372-386
                cam.image_plane = image_plane;
                cam.dof_amount = dof_amount;
                Vec4d pos = from_abi(cam.position);
                if (!eq3(focal_point, v4d(0, 0, 0, 0))) cam.focal_length = length_s(sub(focal_point, pos));
                else if (focal_length != 0) cam.focal_length = focal_length;
                else cam.focal_length = length_s(sub(from_abi(cam.look_at), pos));
                out.cameras.push_back(cam);
            }
            for (rt_prim& p : pending) { // SceneLoader.cs:388-413
                p.flags &= ~(RT_FLAG_TWOSIDED | RT_FLAG_INVERT);
                if (two_sided) p.flags |= RT_FLAG_TWOSIDED;
                if (invert) p.flags |= RT_FLAG_INVERT;
                if (!same(emission, placeholder)) p.emission = emission;
                if (!same(diffuse, placeholder)) p.diffuse = diffuse;
                if (!same(specular, placeholder)) p.specular = specular;
                if (shininess != -1) p.shininess = shininess;
                if (!same(refraction, placeholder)) {
                    p.refraction = refraction;
                    p.refractive_index = refraction_index;
                }
                apply_transform(p, stack.back(), inv_stack.back());
                out.prims.push_back(p);
            }
            pending.clear();
        } catch (const std::exception& e) {
            err = "Error while parsing command " + cmd + " on line " + std::to_string(line_no) + ": " + e.what();
            return false;
        }
    }
    return true;
}

} // namespace rtc
