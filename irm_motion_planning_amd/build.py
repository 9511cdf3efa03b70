"""In-tree build of libirm_hip.so (hipcc, gfx950 only).

    python -m irm_motion_planning_amd.build [--force] [--prof] [-j N]

The optimiser templates (csrc/irm_kernels_impl.hpp) are instantiated in one
object per problem shape (csrc/irm_opt_inst.hip compiled with IRM_INST_*), so
the objects build in parallel; the host-API kernels and dispatch
(irm_kernels.hip) and the C ABI (irm_host.cpp) are two more objects.  The .so
lands next to this file so that it travels with the repository snapshot to the
GPU box (it is git-ignored, not gpurun-ignored); objects stay in _obj/.
"""
import glob
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
OUT = os.path.join(HERE, "libirm_hip.so")
HEADERS = [os.path.join(CSRC, h) for h in ("irm_kernels.hpp", "irm_kernels_impl.hpp")] + \
    [os.path.join(HERE, "..", "include", "irm.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -amdgpu-atomic-optimizer-strategy=None: every LDS atomic in the kernels is issued by one lane (flag
# words); the optimizer's scan over the active lanes is a ~25-instruction waterfall per round there.
# -ffp-contract=off: no fused multiply-add the source does not write (fmaf / pkfma) — the results do
# not depend on the compiler's contraction choices, which moved with unrelated code before (round 3).
# -fno-slp-vectorize: no packing of scalar f32 arithmetic into v_pk_* (the explicit f32x2 code of the
# obstacle potential stays packed): the packed forms needed v_mov pairs around them and measured
# slower (C3 0.763 -> 0.726 ms, same box, profiles/r04_*).
CFLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
          "-ffp-contract=off", "-fno-slp-vectorize",
          "-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]
FIX_SHAPES = [(3, 50), (3, 64), (3, 128), (3, 256), (7, 128), (7, 256)]  # IRM_FIX_SHAPES in irm_kernels_impl.hpp
DENSE_SHAPES = [(7, 256)]  # the dense operator's k_lean (irm_kernels.hip launch_optimize)
MAX_D = 8

VARIANTS = {
    "": ("libirm_hip.so", []),
    "prof": ("libirm_hip_prof.so", ["-DIRM_PHASE_PROFILE"]),
    # every unit with the default scheduler (tools/sched_check.py compares it bit for bit)
    "defsched": ("libirm_hip_defsched.so", ["-DIRM_DEFAULT_SCHED"]),
    # the DynShape units with the iterative-ILP scheduler too (the D = 5 divergence check)
    "dynilp": ("libirm_hip_dynilp.so", ["-DIRM_DYN_ILP"]),
    # the BLS trial stages count ĝ's mismatches against the IEEE division (tools/div_check.py)
    "divchk": ("libirm_hip_divchk.so", ["-DIRM_DIV_CHECK"]),
}


# Machine scheduler per unit: the general optimiser (and C4's two-waypoints-per-lane lean kernel) ran
# 5-10 % faster with LLVM's iterative-ILP strategy (faithful C3 5.78 -> 5.21 ms, C4 1.97 -> 1.88 ms);
# the one-waypoint-per-lane lean kernels are 1-2 % faster with the default.
ILP_SCHED = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
LEAN_ILP_SHAPES = {(3, 256)}


def source_files():
    """Everything the library is compiled from (the build provenance hash covers exactly these)."""
    return sorted(glob.glob(os.path.join(CSRC, "*"))) + [os.path.normpath(os.path.join(HERE, "..", "include", "irm.h"))]


def source_hash(variant=""):
    """First 16 hex digits of the SHA-256 over the sources (names relative to the repo root, then
    contents), the compile flags of every unit and the variant's name and extra flags.  irm_build_id()
    of a library built here returns it (-DIRM_SOURCE_HASH on irm_host.cpp); __graft_entry__.smoke()
    compares the two, so a stale prebuilt library — or one built with other flags (a profiling or
    experimental variant) — fails."""
    root = os.path.normpath(os.path.join(HERE, ".."))
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    name, extra = variant_spec(variant)
    h.update(("\0".join([name] + CFLAGS + extra) + "\0").encode())
    for oname, src, flags in _units():
        h.update(("\0".join([oname, src] + flags) + "\0").encode())
    return h.hexdigest()[:16]


def variant_spec(variant):
    """(library file name, extra flags) of a build variant: the named ones of VARIANTS, or an ad-hoc
    experiment registered by add_variant (same-box A/B builds, tools/gpu/*.sh)."""
    return VARIANTS[variant]


def add_variant(name, flags):
    VARIANTS[name] = (f"libirm_hip_{name}.so", list(flags))


def _units():
    """(object name, source, extra flags) of every compilation unit, before the build id."""
    u = [("irm_kernels", "irm_kernels.hip", []), ("irm_host", "irm_host.cpp", [])]
    # (DynShape units keep the default scheduler: with iterative-ILP the D = 5 register-resident
    # variant, which spills heavily, left the exact-iteration band — tests/test_gpu_parity.py::
    # test_generic_shapes_match_reference_iteration[64-5] — so it is not used there)
    u += [(f"opt_dyn{d}", "irm_opt_inst.hip", [f"-DIRM_INST_DYN={d}"]) for d in range(1, MAX_D + 1)]
    u += [(f"opt_fix{d}_{n}", "irm_opt_inst.hip", [f"-DIRM_INST_FIX_D={d}", f"-DIRM_INST_FIX_N={n}"]
           + (ILP_SCHED if (d, n) in LEAN_ILP_SHAPES else [])) for d, n in FIX_SHAPES]
    u += [(f"opt_gen{d}_{n}", "irm_opt_inst.hip", [f"-DIRM_INST_GEN_D={d}", f"-DIRM_INST_GEN_N={n}"] + ILP_SCHED)
          for d, n in FIX_SHAPES]
    u += [(f"opt_dense{d}_{n}", "irm_opt_inst.hip", [f"-DIRM_INST_DENSE_D={d}", f"-DIRM_INST_DENSE_N={n}"])
          for d, n in DENSE_SHAPES]
    return u


def units(variant=""):
    """(object name, source, extra flags) of every compilation unit (irm_host carries the build id)."""
    bid = f'-DIRM_SOURCE_HASH="{source_hash(variant)}"'
    return [(o, src, fl + [bid] if o == "irm_host" else fl) for o, src, fl in _units()]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, variant="", jobs=None):
    name, extra = variant_spec(variant)
    out = os.path.join(HERE, name)
    odir = os.path.join(OBJ, variant or "release")
    os.makedirs(odir, exist_ok=True)
    jobs = jobs or min(16, os.cpu_count() or 1)
    todo, objs = [], []
    # a change of flags rebuilds every object; the stamp is written only after every object compiled and
    # the link succeeded (and removed when a compile fails), so a build interrupted after a flag change
    # cannot leave objects of the old flags looking current
    stamp = os.path.join(odir, "flags.txt")
    flagtxt = "\n".join(CFLAGS + extra)
    if not os.path.exists(stamp) or open(stamp).read() != flagtxt:
        force = True
        if os.path.exists(stamp):
            os.remove(stamp)
    for oname, src, flags in units(variant):
        obj = os.path.join(odir, oname + ".o")
        objs.append(obj)
        deps = [os.path.join(CSRC, src), __file__] + HEADERS
        if oname == "irm_host":  # carries the hash of every source
            deps = deps + source_files()
        if "-DIRM_DYN_ILP" in extra and oname.startswith("opt_dyn"):
            flags = flags + ILP_SCHED
        if force or _newer(obj, deps):
            todo.append([HIPCC] + CFLAGS + extra + flags + ["-c", "-o", obj, os.path.join(CSRC, src)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd, cwd=CSRC)

    if "-DIRM_DEFAULT_SCHED" in extra:
        def drop_sched(cmd):
            out, i = [], 0
            while i < len(cmd):
                if cmd[i:i + 2] == ILP_SCHED:
                    i += 2
                    continue
                out.append(cmd[i])
                i += 1
            return out
        todo = [drop_sched(cmd) for cmd in todo]
    try:
        if todo:
            with ThreadPoolExecutor(jobs) as ex:
                list(ex.map(run, todo))
        if todo or force or _newer(out, objs):
            run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    except BaseException:
        if os.path.exists(stamp):
            os.remove(stamp)
        raise
    with open(stamp, "w") as fh:
        fh.write(flagtxt)
    return out


def asm(out_dir, inst=("-DIRM_INST_FIX_D=3", "-DIRM_INST_FIX_N=128")):
    """Emit the gfx950 assembly of one instantiation unit (for ISA inspection)."""
    os.makedirs(out_dir, exist_ok=True)
    cmd = [HIPCC] + [f for f in CFLAGS if f != "-fPIC"] + ["--cuda-device-only", "-S", *inst,
           "-o", os.path.join(out_dir, "irm_opt.s"), os.path.join(CSRC, "irm_opt_inst.hip")]
    subprocess.check_call(cmd, cwd=CSRC)


if __name__ == "__main__":
    jobs = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else None
    if "--variant" in sys.argv:  # ad-hoc experiment: --variant NAME [--extra "FLAGS"]
        vname = sys.argv[sys.argv.index("--variant") + 1]
        vflags = sys.argv[sys.argv.index("--extra") + 1].split() if "--extra" in sys.argv else []
        add_variant(vname, vflags)
        build(force="--force" in sys.argv, variant=vname, verbose=False, jobs=jobs)
        print("built", VARIANTS[vname][0], source_hash(vname))
        sys.exit(0)
    build(force="--force" in sys.argv, verbose=True, jobs=jobs)
    for v in VARIANTS:  # e.g. --defsched (tools/sched_check.py)
        if v and v != "prof" and f"--{v}" in sys.argv:  # --defsched, --dynilp, --divchk
            build(force="--force" in sys.argv, variant=v, verbose=True, jobs=jobs)
    if "--prof" in sys.argv:
        build(force="--force" in sys.argv, variant="prof", verbose=True, jobs=jobs)
