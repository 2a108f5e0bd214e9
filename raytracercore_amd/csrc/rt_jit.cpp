// rt_jit.cpp -- scene-specialised brute-force path kernels (see rt_jit.h), built with hiprtc.
#include "rt_jit.h"

#include <hip/hiprtc.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include "rt_jit_sources.h" // generated: kernels_path.hip and the headers it includes

namespace rtc {

namespace {

std::atomic<int> g_jit{-1}; // -1: not yet read from RTCORE_JIT

template <class T>
void put_words(std::ostringstream& o, const char* name, const std::vector<T>& v)
{
    static_assert(sizeof(T) % 4 == 0, "records are whole words");
    const size_t n = v.size() * sizeof(T) / 4;
    std::vector<uint32_t> w(n ? n : 1, 0u);
    if (n) std::memcpy(w.data(), v.data(), n * 4);
    o << "__device__ static const uint32_t " << name << "[" << w.size() << "] __attribute__((aligned(16))) = {";
    char buf[16];
    for (size_t i = 0; i < w.size(); i++) {
        std::snprintf(buf, sizeof buf, "%s0x%x", i ? "," : "", w[i]);
        o << buf;
    }
    o << "};\n";
}

uint64_t fnv1a(uint64_t h, const void* p, size_t n)
{
    const unsigned char* c = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; i++) {
        h ^= c[i];
        h *= 1099511628211ull;
    }
    return h;
}

std::string cache_dir()
{
    if (const char* e = std::getenv("RTCORE_JIT_CACHE")) return e;
    if (const char* x = std::getenv("XDG_CACHE_HOME")) return std::string(x) + "/rtcore_jit";
    if (const char* h = std::getenv("HOME")) return std::string(h) + "/.cache/rtcore_jit";
    return "/tmp/rtcore_jit_" + std::to_string((unsigned)getuid());
}

// The disk cache holds code objects this process will load and run, so it is used only when the
// directory is the caller's own and nobody else can write into it: created with mode 0700, and an
// existing directory must be owned by the caller and not group- or world-writable.
bool cache_dir_trusted(const std::string& dir, bool create)
{
    struct stat st;
    if (stat(dir.c_str(), &st) != 0) {
        if (!create) return false;
        std::error_code ec;
        const std::filesystem::path parent = std::filesystem::path(dir).parent_path();
        if (!parent.empty()) std::filesystem::create_directories(parent, ec);
        if (mkdir(dir.c_str(), 0700) != 0 && errno != EEXIST) return false;
        if (stat(dir.c_str(), &st) != 0) return false;
    }
    return S_ISDIR(st.st_mode) && st.st_uid == getuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

// Keeps at most kDiskKeep code objects in the cache directory: the least recently used (by mtime,
// which a cache hit refreshes) go first, so a host that moves the camera often does not grow it
// without bound.
constexpr size_t kDiskKeep = 64;
void prune_cache(const std::string& dir)
{
    std::error_code ec;
    std::vector<std::pair<std::filesystem::file_time_type, std::filesystem::path>> cos;
    for (const auto& e : std::filesystem::directory_iterator(dir, ec))
        if (e.path().extension() == ".co") cos.push_back({e.last_write_time(ec), e.path()});
    if (cos.size() <= kDiskKeep) return;
    std::sort(cos.begin(), cos.end());
    for (size_t i = 0; i + kDiskKeep < cos.size(); i++) std::filesystem::remove(cos[i].second, ec);
}

bool read_file(const std::string& path, std::vector<char>& out)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    return !out.empty();
}

void write_file_atomic(const std::string& dir, const std::string& path, const std::vector<char>& data)
{
    std::error_code ec;
    if (!cache_dir_trusted(dir, true)) return; // the cache is an optimisation only
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    {
        std::ofstream f(tmp, std::ios::binary);
        if (!f) return;
        f.write(data.data(), (std::streamsize)data.size());
        if (!f) return;
    }
    std::filesystem::rename(tmp, path, ec);
    if (ec) std::filesystem::remove(tmp, ec);
    prune_cache(dir);
}

// RTCORE_JIT_FLAGS: extra compiler flags for experiments (e.g. "-DRT_PATH_WAVES=8"), space-separated
std::vector<std::string> jit_extra_flags()
{
    std::vector<std::string> out;
    if (const char* e = std::getenv("RTCORE_JIT_FLAGS")) {
        std::istringstream in(e);
        for (std::string f; in >> f;) out.push_back(f);
    }
    return out;
}

std::string main_source(bool grouped)
{
    return std::string("#include \"rt_jit_prelude.h\"\n#define RT_SCENE_CONST\n#define RT_SCENE_CONST_GROUPED ") +
           (grouped ? "1" : "0") + "\n#include \"kernels_path.hip\"\n";
}

// The compiler options of a scene-specialised build: the library's own kernel flags (Makefile
// HIPFLAGS: no fused multiply-adds the source does not write, no SLP packing -- v_pk_* issue no
// faster than two plain ops on gfx950), then RTCORE_JIT_FLAGS.  They are part of the cache key.
std::vector<std::string> compile_options(const std::string& arch)
{
    std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-std=c++17", "-ffp-contract=off",
                                     "-fno-slp-vectorize", "-munsafe-fp-atomics"};
    for (const std::string& f : jit_extra_flags()) opts.push_back(f);
    return opts;
}

bool compile(const std::string& arch, const std::string& main_src, const std::string& header, std::vector<char>& code,
             std::string& err)
{
    std::vector<const char*> names, texts;
    for (int k = 0; k < kJitSrcCount; k++) {
        names.push_back(kJitSrcNames[k]);
        texts.push_back(kJitSrcTexts[k]);
    }
    names.push_back("rt_scene_const.h");
    texts.push_back(header.c_str());
    hiprtcProgram prog = nullptr;
    if (hiprtcCreateProgram(&prog, main_src.c_str(), "rt_jit_main.hip", (int)names.size(), texts.data(), names.data()) !=
        HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return false;
    }
    const std::vector<std::string> opt_s = compile_options(arch);
    std::vector<const char*> opts;
    for (const std::string& o : opt_s) opts.push_back(o.c_str());
    const hiprtcResult r = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        err = "hiprtc: " + std::string(hiprtcGetErrorString(r)) + ": " + log.substr(0, 2000);
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code.resize(n);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return n > 0;
}

struct Entry {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    int refs = 0;        // scenes holding fn (jit_kernel / jit_release)
    uint64_t stamp = 0;  // last use, for the eviction of unreferenced modules
};
std::mutex g_mu;
std::map<std::pair<int, uint64_t>, Entry> g_cache; // (device, key) -> loaded module
uint64_t g_stamp = 0;

// Unloads the least recently used unreferenced modules beyond kJitKeep (g_mu held).  A released
// module may still run in launches queued before its release, so the device is synchronised first.
void evict_unreferenced()
{
    std::vector<std::pair<uint64_t, std::pair<int, uint64_t>>> idle;
    for (const auto& kv : g_cache)
        if (kv.second.refs == 0 && kv.second.mod) idle.push_back({kv.second.stamp, kv.first});
    if ((int)idle.size() <= kJitKeep) return;
    std::sort(idle.begin(), idle.end());
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (size_t i = 0; i + kJitKeep < idle.size(); i++) {
        const auto key = idle[i].second;
        Entry& e = g_cache[key];
        if (hipSetDevice(key.first) == hipSuccess && hipDeviceSynchronize() == hipSuccess) {
            (void)hipModuleUnload(e.mod);
            g_cache.erase(key);
        }
    }
    (void)hipSetDevice(cur);
}

} // namespace

bool jit_enabled()
{
    int v = g_jit.load();
    if (v < 0) {
        const char* e = std::getenv("RTCORE_JIT");
        v = (e && e[0] == '0') ? 0 : 1;
        int expect = -1;
        g_jit.compare_exchange_strong(expect, v);
        v = g_jit.load();
    }
    return v == 1;
}

void jit_set_enabled(bool on) { g_jit.store(on ? 1 : 0); }

std::string jit_scene_header(const PathScene& ps, const CameraF& cam, bool with_camera, const std::vector<GroupRec>& groups,
                             const std::vector<RectRec>& rects, const std::vector<FrameRec>& frames,
                             const std::vector<TestRec>& tests, const std::vector<XformF>& xf)
{
    std::ostringstream o;
    o << "// generated by rt_jit.cpp: one launch's scene as constants\n#pragma once\n";
    o << "#define RT_SCENE_CONST_VN " << (ps.n_vn > 0 ? 1 : 0) << "\n"; // vertex-normal triangles (their re-hit test)
    PathScene p = ps;
    p.hot4 = nullptr; // brute-force kernels only
    p.n_hot4 = 0;
    p.width = 0;      // read from the launch record (one build serves every frame size)
    put_words(o, "kSceneW", std::vector<PathScene>{p});
    if (with_camera) {
        o << "#define RT_SCENE_CONST_CAMERA 1\n";
        put_words(o, "kCameraW", std::vector<CameraF>{cam});
    } else { // camera-independent: its kind and depth-of-field switch only
        o << "#define RT_SCENE_CONST_CAMERA 0\n#define RT_SCENE_CAMERA_KIND " << cam.kind
          << "\n#define RT_SCENE_CAMERA_DOF " << (cam.dof != 0.0f ? 1 : 0) << "\n";
    }
    put_words(o, "kGroupsW", groups);
    put_words(o, "kRectsW", rects);
    put_words(o, "kFramesW", frames);
    put_words(o, "kTestsW", tests);
    put_words(o, "kXfW", xf);
    return o.str();
}

bool jit_kernel(int device, const std::string& header, bool grouped, JitKernel& out, std::string& err)
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        err = "hipGetDeviceProperties failed";
        return false;
    }
    const std::string arch = prop.gcnArchName;
    // the key covers everything the code object depends on: the embedded sources, the generated
    // header, the entry source, every compiler option, the device architecture and the compiler
    // and runtime versions (a ROCm upgrade must not load objects built by the old compiler)
    uint64_t key = 1469598103934665603ull;
    key = fnv1a(key, "rtcore-jit-2", 12);
    key = fnv1a(key, arch.data(), arch.size());
    for (int k = 0; k < kJitSrcCount; k++) key = fnv1a(key, kJitSrcTexts[k], std::strlen(kJitSrcTexts[k]));
    key = fnv1a(key, header.data(), header.size());
    const std::string main_src = main_source(grouped);
    key = fnv1a(key, main_src.data(), main_src.size());
    for (const std::string& f : compile_options(arch)) key = fnv1a(key, f.data(), f.size() + 1);
    int versions[3] = {0, 0, 0};
    (void)hiprtcVersion(&versions[0], &versions[1]);
    (void)hipRuntimeGetVersion(&versions[2]);
    key = fnv1a(key, versions, sizeof versions);

    std::lock_guard<std::mutex> lock(g_mu);
    out = JitKernel{};
    Entry& e = g_cache[{device, key}];
    if (!e.mod) {
        // the module belongs to the device's context: load it there whatever device is current
        int cur = 0;
        (void)hipGetDevice(&cur);
        struct Restore {
            int dev;
            ~Restore() { (void)hipSetDevice(dev); }
        } restore{cur};
        if (hipSetDevice(device) != hipSuccess) {
            err = "hipSetDevice failed";
            g_cache.erase({device, key});
            return false;
        }
        char hex[32];
        std::snprintf(hex, sizeof hex, "%016llx", (unsigned long long)key);
        const std::string dir = cache_dir(), path = dir + "/" + hex + ".co";
        auto load = [&](const std::vector<char>& code) {
            if (hipModuleLoadData(&e.mod, code.data()) == hipSuccess &&
                hipModuleGetFunction(&e.fn, e.mod, "rt_path_const") == hipSuccess)
                return true;
            if (e.mod) (void)hipModuleUnload(e.mod);
            e = Entry{};
            return false;
        };
        std::vector<char> code;
        bool loaded = false;
        if (cache_dir_trusted(dir, false) && read_file(path, code)) {
            loaded = load(code);
            if (loaded) {
                out.from_cache = true;
                utimes(path.c_str(), nullptr); // most recently used (prune_cache)
            } else {
                // an unusable cache file (another ROCm, a damaged disk): drop it and rebuild
                std::error_code ec;
                std::filesystem::remove(path, ec);
                (void)hipGetLastError();
            }
        }
        if (!loaded) {
            const auto t0 = std::chrono::steady_clock::now();
            if (!compile(arch, main_src, header, code, err)) {
                g_cache.erase({device, key});
                return false;
            }
            out.compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (!load(code)) {
                err = "loading the scene-specialised module failed";
                (void)hipGetLastError();
                g_cache.erase({device, key});
                return false;
            }
            write_file_atomic(dir, path, code);
        }
    } else {
        out.from_cache = true;
    }
    out.fn = e.fn;
    e.refs++;
    e.stamp = ++g_stamp;
    evict_unreferenced(); // e is referenced, so it stays
    return true;
}

void jit_release(int device, hipFunction_t fn)
{
    std::lock_guard<std::mutex> lock(g_mu);
    for (auto& kv : g_cache)
        if (kv.first.first == device && kv.second.fn == fn && kv.second.refs > 0) {
            kv.second.refs--;
            return;
        }
}

size_t jit_compile_check(const std::string& arch, bool grouped, std::string& err)
{
    const std::string header = jit_scene_header(PathScene{}, CameraF{}, grouped, {}, {}, {}, {}, {});
    std::vector<char> code;
    if (!compile(arch, main_source(grouped), header, code, err)) return 0;
    return code.size();
}

} // namespace rtc
