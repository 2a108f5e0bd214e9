"""Compile the scene-specialised kernel for a dumped header (tools/jit_dump.py) on the CPU with hiprtc,
the same way rt_jit.cpp does, and write the code object and its disassembly.
usage: tools/jit_isa.py HEADER {0|1 grouped} OUT_PREFIX [extra hiprtc flags...]"""
import ctypes as C
import os
import subprocess
import sys

CSRC = os.environ.get("RTCORE_CSRC") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracercore_amd", "csrc")
NAMES = ["rt_jit_prelude.h", "kernels_path.hip", "../../include/rtcore_rng.h", "rt_kernels.h", "rt_internal.h",
         "../../include/rtcore.h"]


def main():
    header, grouped, out = sys.argv[1], sys.argv[2], sys.argv[3]
    extra = sys.argv[4:]
    rtc = C.CDLL("/opt/rocm/lib/libhiprtc.so")
    names = NAMES + ["rt_scene_const.h"]
    texts = [open(os.path.join(CSRC, n), "rb").read() for n in NAMES] + [open(header, "rb").read()]
    main_src = (b'#include "rt_jit_prelude.h"\n#define RT_SCENE_CONST\n#define RT_SCENE_CONST_GROUPED ' +
                grouped.encode() + b'\n#include "kernels_path.hip"\n')
    prog = C.c_void_p()
    arr = C.c_char_p * len(names)
    r = rtc.hiprtcCreateProgram(C.byref(prog), main_src, b"rt_jit_main.hip", len(names), arr(*texts),
                                arr(*[n.encode() for n in names]))
    assert r == 0, r
    opts = [b"--offload-arch=gfx950", b"-O3", b"-std=c++17", b"-ffp-contract=off", b"-fno-slp-vectorize",
            b"-munsafe-fp-atomics"] + [e.encode() for e in extra]
    r = rtc.hiprtcCompileProgram(prog, len(opts), (C.c_char_p * len(opts))(*opts))
    n = C.c_size_t()
    rtc.hiprtcGetProgramLogSize(prog, C.byref(n))
    log = C.create_string_buffer(n.value + 1)
    rtc.hiprtcGetProgramLog(prog, log)
    if r != 0:
        sys.exit("hiprtc failed: " + log.value.decode(errors="replace")[:4000])
    rtc.hiprtcGetCodeSize(prog, C.byref(n))
    code = C.create_string_buffer(n.value)
    rtc.hiprtcGetCode(prog, code)
    with open(out + ".co", "wb") as f:
        f.write(code.raw)
    dis = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", out + ".co"],
                         capture_output=True, text=True, check=True).stdout
    with open(out + ".s", "w") as f:
        f.write(dis)
    print("wrote", out + ".co", out + ".s", len(dis.splitlines()), "lines")


if __name__ == "__main__":
    main()
