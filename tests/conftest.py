"""Shared fixtures.

Markers: `gpu` — needs an MI355X (run with `pytest -m gpu` on the GPU box);
everything else runs on CPU in the build container.

Parity is judged against two checkers:
  * tests/golden/*.npz — vectors produced by the unmodified reference
    (oracle/tools/gen_golden.py, run in the build container only);
  * oracle/ — the C restatement of the reference (CPU), same seeded inputs.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")

START = np.array([0.0, 0.0, 0.0], np.float32)  # environment.py:14
GOAL = np.array([1.2, 0.8, 0.3], np.float32)  # environment.py:15


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libirm_hip.so")


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def g_setup():
    return golden("ref_setup")


@pytest.fixture(scope="session")
def g_eval():
    return golden("ref_eval_n50")


@pytest.fixture(scope="session")
def g_gd():
    return golden("ref_gd_steps_n50")


@pytest.fixture(scope="session")
def g_e2e():
    return golden("ref_e2e")


@pytest.fixture(scope="session")
def g_vis():
    return golden("ref_visualization")


def ref_args(*argv):
    """argparse namespace with the reference's defaults (main.py:13-102) plus argv."""
    from irm_motion_planning_amd import main as irm_main
    return irm_main.parse_args([str(a) for a in argv])


def params(*argv, **overrides):
    from irm_motion_planning_amd.params import params_from_args
    return params_from_args(ref_args(*argv), **overrides)


def oracle_for(*argv, **overrides):
    from oracle.oracle import Oracle
    return Oracle(params(*argv, **overrides))


def obstacles(n=11):
    from irm_motion_planning_amd.environment import OBSTACLES
    return OBSTACLES[:n].astype(np.float32)


# End-to-end cases recorded by gen_golden.py: tag -> (argv, n_obstacles)
E2E_CASES = {
    "bls_n50_lmax0.0": (["--lambda-max-cost", "0.0"], 11),
    "bls_n50_lmax0.25": (["--lambda-max-cost", "0.25"], 11),
    "bls_n50_lmax0.5": ([], 11),
    "bls_n50_lmax0.75": (["--lambda-max-cost", "0.75"], 11),
    "bls_n50_lmax1.0": (["--lambda-max-cost", "1.0"], 11),
    "gd_n50": (["--optimizer-name", "gd"], 11),
    "bls_n128": (["--n-timesteps", "128"], 11),
    "c1_gd_n64_o3": (["--optimizer-name", "gd", "--n-timesteps", "64"], 3),
    "c2_bls_n128_o10": (["--n-timesteps", "128"], 10),
}

# Quality band (see check_quality).
QUALITY_TOL = 0.01
BETTER_TOL = 0.03


def check_quality(g, tag, avg, mx, ok):
    """End-to-end parity for the chaotic / noise-terminated loops.

    The reference's own outcome moves with ±1 ulp on α0 (gen_golden.py records
    that ensemble), and its fp32 α-space iteration drifts from the exact-arithmetic
    iteration (oracle/ref64.py; tests/test_oracle_golden.py::test_fp32_alpha_drift).
    Required: the constraint flag is one the reference ensemble produced; the
    avg / max obstacle cost is no worse than the ensemble's worst + QUALITY_TOL and
    no better than the ensemble's best − BETTER_TOL.
    """
    ens_avg = np.append(g[f"{tag}__ens_avg_cost"], g[f"{tag}__avg_cost"])
    ens_max = np.append(g[f"{tag}__ens_max_cost"], g[f"{tag}__max_cost"])
    ens_ok = np.append(g[f"{tag}__ens_constraints_ok"], g[f"{tag}__constraints_ok"])
    print(f"{tag}: avg {avg:.4f} (ref [{ens_avg.min():.4f}, {ens_avg.max():.4f}]) "
          f"max {mx:.4f} (ref [{ens_max.min():.4f}, {ens_max.max():.4f}]) ok {ok}")
    assert ens_avg.min() - BETTER_TOL <= avg <= ens_avg.max() + QUALITY_TOL, (tag, avg, ens_avg)
    assert ens_max.min() - BETTER_TOL <= mx <= ens_max.max() + QUALITY_TOL, (tag, mx, ens_max)
    assert bool(ok) in set(bool(x) for x in ens_ok), (tag, ok, ens_ok)
