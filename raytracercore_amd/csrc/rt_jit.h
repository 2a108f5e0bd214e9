// rt_jit.h -- scene-specialised brute-force path kernels, compiled at run time with hiprtc.
//
// The brute-force kernels test every primitive record of a small scene (<= 48 primitives) in
// every loop iteration, each record field an SGPR operand.  On gfx950 a VALU instruction with an
// SGPR operand issues in ~4.2 cycles, with a VGPR or literal operand in ~2.5 (tools/micro), and
// the per-record loop counters, scalar loads and flag branches cost SALU issue besides.  A build
// of kernels_path.hip with the scene's records as compile-time constants (RT_SCENE_CONST) folds
// the fields into literal operands, unrolls the primitive loops and resolves the flag branches:
// bounce.txt C2 24.4 -> 21.0 ms.  Same arithmetic, same results as the generic kernel (tested).
#pragma once
#include <string>
#include <vector>

#include "rt_kernels.h"

namespace rtc {

// The generated header (kSceneW, kGroupsW, kRectsW, kFramesW, kTestsW, kXfW) of one scene and
// slot order.  with_camera: the camera's values as well (kCameraW; the grouped order, whose group
// order is per camera anyway); otherwise only its kind and whether it has depth of field are
// compiled in (RT_SCENE_CAMERA_KIND, RT_SCENE_CAMERA_DOF) and the kernel reads the camera from
// device memory, so one build serves every camera of those two facts.
std::string jit_scene_header(const PathScene& ps, const CameraF& cam, bool with_camera, const std::vector<GroupRec>& groups,
                             const std::vector<RectRec>& rects, const std::vector<FrameRec>& frames,
                             const std::vector<TestRec>& tests, const std::vector<XformF>& xf);

struct JitKernel {
    hipFunction_t fn = nullptr;
    double compile_ms = 0;  // 0 when served from the in-process or on-disk cache
    bool from_cache = false;
};

// The grouped (culling) or flat entry point built for `header` on `device` (the current device),
// cached per process and on disk (RTCORE_JIT_CACHE, else $HOME/.cache/rtcore_jit, else /tmp).
// Returns false with `err` set when hiprtc or the module load fails.  A successful call holds a
// reference on the module until jit_release; the process keeps at most kJitKeep modules nobody
// references and unloads the least recently used beyond that (after synchronising its device), so
// a caller that moves the camera often does not accumulate one loaded module per camera.
bool jit_kernel(int device, const std::string& header, bool grouped, JitKernel& out, std::string& err);
void jit_release(int device, hipFunction_t fn);
constexpr int kJitKeep = 16;

// Host only: compiles the embedded sources for `arch` with an empty scene; the code object size,
// or 0 with `err` set (the CPU tests' check that the run-time build compiles).
size_t jit_compile_check(const std::string& arch, bool grouped, std::string& err);

// Process-wide switch (rt_set_jit; RTCORE_JIT=0 turns the default off).
bool jit_enabled();
void jit_set_enabled(bool on);

} // namespace rtc
