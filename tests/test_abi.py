"""The C-ABI boundary (include/irm.h) without a GPU: the library loads, exports
every declared symbol, its structs match the ctypes mirror byte for byte, the
host-side entry points behave, and context creation fails loudly — never
falls back to the CPU — when no gfx950 device is present.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO, params, ref_args

HEADER = os.path.join(REPO, "include", "irm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(irm_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from irm_motion_planning_amd._abi import load_library
    return load_library()


def test_library_exports_every_declared_symbol(lib):
    from irm_motion_planning_amd._abi import PROTOTYPES
    names = declared_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(PROTOTYPES) == names  # the ctypes mirror binds exactly the header


def test_library_is_gfx950_code_object():
    from irm_motion_planning_amd._abi import LIB_PATH
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", LIB_PATH],
                         capture_output=True, text=True)
    blob = out.stdout + out.stderr
    if out.returncode != 0 or "gfx" not in blob:
        data = open(LIB_PATH, "rb").read()
        assert b"gfx950" in data
        return
    assert "gfx950" in blob


LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "irm.h"
#define F(T, f) printf(#T " " #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("sizeof irm_params %zu\nsizeof irm_stats %zu\nsizeof irm_info %zu\nsizeof irm_batch_dev %zu\n"
         "sizeof irm_launch_plan %zu\n", sizeof(irm_params), sizeof(irm_stats), sizeof(irm_info),
         sizeof(irm_batch_dev), sizeof(irm_launch_plan));
  %FIELDS%
  return 0;
}
"""


def test_struct_layout_matches_ctypes(tmp_path):
    from irm_motion_planning_amd import _abi
    structs = {"irm_params": _abi.IrmParams, "irm_stats": _abi.IrmStats, "irm_info": _abi.IrmInfo,
               "irm_batch_dev": _abi.IrmBatchDev, "irm_launch_plan": _abi.IrmLaunchPlan}
    fields = "\n".join(f"F({cn}, {f})" for cn, cls in structs.items() for f, _ in cls._fields_)
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C.replace("%FIELDS%", fields))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    lines = subprocess.check_output([str(exe)], text=True).split("\n")
    got = {}
    for ln in lines:
        if not ln:
            continue
        a, b, c = ln.split()
        got[(a, b)] = int(c)
    for cn, cls in structs.items():
        assert got[("sizeof", cn)] == ctypes.sizeof(cls), cn
        for f, _ in cls._fields_:
            assert got[(cn, f)] == getattr(cls, f).offset, (cn, f)


def test_build_id_is_the_source_hash(lib):
    """The library names the sources it was built from (build.py embeds the hash); smoke() asserts
    it equals the checked-out sources' hash, so a stale prebuilt library fails loudly."""
    from irm_motion_planning_amd import build
    assert lib.irm_build_id().decode() == build.source_hash()


def test_params_default_equals_reference_argparse_defaults(lib):
    """irm_params_default() carries main.py:13-102's defaults (and J of trajectory.py:42)."""
    from irm_motion_planning_amd._abi import IrmParams
    d = IrmParams()
    lib.irm_params_default(ctypes.byref(d))
    a = params()  # parse_args([]) → params_from_args
    for f, _ in IrmParams._fields_:
        x, y = getattr(d, f), getattr(a, f)
        if hasattr(x, "__len__"):
            np.testing.assert_array_equal(np.array(list(x)), np.array(list(y)), err_msg=f)
        else:
            assert x == y, f
    assert d.n_timesteps == 50 and d.n_joints == 3 and d.optimizer == 1
    assert d.rbf_variance == np.float32(0.1) and d.max_inner_iteration == 200 and d.max_outer_iteration == 10


def test_default_jac_matches_reference(lib, g_setup):
    """irm_default_jac = I + 0.15·normal(PRNGKey(0)) with JAX's legacy threefry (host code)."""
    from irm_motion_planning_amd.context import default_jac
    np.testing.assert_array_equal(default_jac(3), g_setup["J"])
    np.testing.assert_allclose(default_jac(7), np.eye(7, dtype=np.float32) + np.float32(0.15) * g_setup["Z7"],
                               rtol=0, atol=1e-7)


def _create(p):
    from irm_motion_planning_amd._abi import load_library
    h = ctypes.c_void_p()
    rc = load_library().irm_ctx_create(ctypes.byref(h), ctypes.byref(p))
    return rc, load_library().irm_last_error().decode()


@pytest.mark.parametrize("field,value,msg", [
    ("n_timesteps", 1, "n_timesteps"),
    ("n_timesteps", 513, "n_timesteps"),
    ("n_joints", 9, "n_joints"),
    ("optimizer", 7, "optimizer"),
    ("rbf_variance", 0.0, "rbf_variance"),
])
def test_ctx_create_validates_params(field, value, msg):
    p = params()
    setattr(p, field, value)
    rc, err = _create(p)
    assert rc == -22 and msg in err


def test_ctx_create_gd_lr_mismatch():
    """optimizer_GD.py:34-36's exit(-1) case is IRM_EINVAL in the library."""
    p = params("--optimizer-name", "gd")
    p.n_gd_lr = 3
    rc, err = _create(p)
    assert rc == -22 and "dual_lr" in err


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU node is present")
def test_no_cpu_fallback_without_gpu():
    """No GPU → IRM_EDEVICE with a message; the product never computes on the host."""
    from irm_motion_planning_amd._abi import IrmError
    from irm_motion_planning_amd.context import Context
    rc, err = _create(params())
    assert rc == -19 and "no CPU fallback" in err
    with pytest.raises(IrmError):
        Context(params())


def test_missing_library_fails_loudly(tmp_path):
    from irm_motion_planning_amd._abi import IrmError, load_library
    with pytest.raises(IrmError):
        load_library(str(tmp_path / "libirm_hip.so"))


def test_params_from_args_reference_errors():
    """robot.py:21-23 and optimizer_GD.py:34-36 exit(-1) → IrmError; float N (main.py:33)."""
    from irm_motion_planning_amd._abi import IrmError
    from irm_motion_planning_amd.params import params_from_args
    with pytest.raises(IrmError):
        params_from_args(ref_args("--n-joints", 4))
    with pytest.raises(IrmError):
        params_from_args(ref_args("--optimizer-name", "gd", "--gd-lr", "1e-3", "1e-4"))
    assert params_from_args(ref_args("--n-timesteps", "64.0")).n_timesteps == 64
    p = params_from_args(ref_args("--gd-lr", "1e-3", "--max-outer-iteration", "1", "--optimizer-name", "gd"))
    assert p.n_gd_lr == 1 and p.gd_lr[0] == np.float32(1e-3)
