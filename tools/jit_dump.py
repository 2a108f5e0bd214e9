"""Write the scene-specialised build's generated header for bounce.txt and die.txt (1080p) to gpurun_out/
(inspection: compile it with hipcc --save-temps to read the specialised kernel's ISA)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracercore_amd as rc  # noqa: E402

os.makedirs("gpurun_out", exist_ok=True)
for name in ("bounce.txt", "die.txt"):
    os.environ["RTCORE_JIT_DUMP"] = "gpurun_out/hdr_" + name.replace(".txt", ".h")
    g = rc.GpuRaytracer(rc.SceneLoader.from_file(rc.scene_path(name)), 0, size=(1920, 1080))
    s = g.render_tile(0, 0, 64, 64, 2, seed=1)
    print(name, g.build_stats())
    g.close()
