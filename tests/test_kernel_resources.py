"""Register / scratch budget of the optimiser kernels on the benched paths, as hipcc builds them for gfx950
(CPU: device assembly only, no GPU).  Guards two regressions found in round 4:
  * spills of the C3 / C7 k_lean variants (the bench, dual-loop and BLS flows of the headline config and
    of north_star's 7-DoF shape) — every one of them is spill-free;
  * a kernel argument whose address escapes (a run-time select between &P.J and an LDS pointer) made the
    compiler copy all of KParams into scratch and read every parameter from there, with no spill
    reported — so the C3 variants must also reserve no scratch at all."""
import os
import re
import shutil
import subprocess
import sys
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _kernels(asm):
    """(demangled name, vgpr, spill, scratch) of every kernel in a hipcc -S device assembly file."""
    meta = asm[asm.index("amdhsa.kernels:"):]
    rows = []
    for blk in re.split(r"\n  - ", meta)[1:]:
        kv = dict(re.findall(r"^\s*\.(\w+):\s+(\S.*)$", blk, re.M))
        if "name" in kv:
            rows.append((kv["name"], int(kv.get("vgpr_count", 0)), int(kv.get("vgpr_spill_count", 0)),
                         int(kv.get("private_segment_fixed_size", 0))))
    names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True,
                           text=True).stdout.split("\n")
    return [(nm,) + r[1:] for r, nm in zip(rows, names)]


@pytest.fixture(scope="module")
def unit_kernels():
    from irm_motion_planning_amd import build
    if not os.path.exists(build.HIPCC) or shutil.which("c++filt") is None:
        pytest.skip("hipcc / c++filt not available")
    units = {u[0]: u for u in build.units()}
    tmp = tempfile.mkdtemp()
    procs = {}
    for name in ("opt_fix3_128", "opt_fix7_128"):
        _, src, flags = units[name]
        out = os.path.join(tmp, name + ".s")
        procs[name] = (out, subprocess.Popen([build.HIPCC] + build.CFLAGS + flags + ["--cuda-device-only", "-S", "-o", out, src],
                                             cwd=build.CSRC, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    res = {}
    for name, (out, p) in procs.items():
        assert p.wait(timeout=600) == 0, name
        with open(out) as f:
            res[name] = [k for k in _kernels(f.read()) if "k_lean" in k[0]]
    shutil.rmtree(tmp, ignore_errors=True)
    return res


def test_c3_lean_kernels_spill_free_without_scratch(unit_kernels):
    ks = unit_kernels["opt_fix3_128"]
    assert len(ks) >= 6, ks
    for name, vgpr, spill, scratch in ks:
        assert spill == 0 and scratch == 0, (name, vgpr, spill, scratch)


def test_c7_lean_kernels_spill_free(unit_kernels):
    ks = unit_kernels["opt_fix7_128"]
    assert len(ks) >= 6, ks
    for name, vgpr, spill, scratch in ks:
        assert spill == 0, (name, vgpr, spill, scratch)
