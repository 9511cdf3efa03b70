"""In-tree build of libirm_hip.so (hipcc, gfx950 only).

    python -m irm_motion_planning_amd.build [--force]

The .so lands next to this file so that it travels with the repository
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libirm_hip.so")
SOURCES = ["irm_kernels.hip", "irm_host.cpp"]
HEADERS = ["irm_kernels.hpp", os.path.join("..", "..", "include", "irm.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-Wall", "-Wno-unused-function"]


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [__file__]
    return any(os.path.getmtime(d) > t for d in deps)


VARIANTS = {
    "": ("libirm_hip.so", []),
    "prof": ("libirm_hip_prof.so", ["-DIRM_PHASE_PROFILE"]),
}


def build(force=False, verbose=False, variant=""):
    name, extra = VARIANTS[variant]
    out = os.path.join(HERE, name)
    if variant:
        cmd = [HIPCC] + FLAGS + extra + ["-o", out] + [os.path.join(CSRC, s) for s in SOURCES]
        subprocess.check_call(cmd, cwd=CSRC)
        return out
    if not force and not _stale():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    return OUT


def asm(out_dir):
    """Emit the gfx950 assembly of the kernels (for ISA inspection)."""
    os.makedirs(out_dir, exist_ok=True)
    cmd = [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "--cuda-device-only", "-S",
           "-o", os.path.join(out_dir, "irm_kernels.s"), os.path.join(CSRC, "irm_kernels.hip")]
    subprocess.check_call(cmd, cwd=CSRC)


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    if "--prof" in sys.argv:
        build(variant="prof", verbose=True)
