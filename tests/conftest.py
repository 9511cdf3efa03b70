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


def e2e_reference(tag):
    """The reference's outcomes for an end-to-end case: the run and its ±1-ulp ensemble, with the
    reference's fp32 BLAS matmuls (ref_e2e*.npz) and with correctly rounded matmuls (*_xm.npz, the
    contraction arithmetic of this build; oracle/tools/gen_golden_bench.py --matmul exact)."""
    out = {}
    for variant, names in (("blas", ("ref_e2e", "ref_e2e_r02", "ref_e2e_n500")),
                           ("xm", ("ref_e2e_xm", "ref_e2e_r02_xm", "ref_e2e_n500_xm"))):
        for name in names:
            g = _golden_cached(name)
            if f"{tag}__avg_cost" in g:
                out[variant] = {k: np.append(g[f"{tag}__ens_{k}"], g[f"{tag}__{k}"])
                                for k in ("avg_cost", "max_cost", "constraints_ok", "grad_calls")}
    assert "blas" in out and "xm" in out, tag
    return out


_GCACHE = {}


def _golden_cached(name):
    if name not in _GCACHE:
        _GCACHE[name] = golden(name)
    return _GCACHE[name]


def constraint_margin(report, eps_p=0.01, eps_v=0.01, pmax=2.0, pmin=-1.0, vmax=7.0):
    """Smallest relative distance of a constraintsFulfilled quantity (trajectory.py:129-137,
    robot.py:90-113; irm_constraints' report layout) to its threshold."""
    r = np.asarray(report, np.float64)
    vals = [(r[0], eps_p), (r[1], eps_p), (r[2], eps_v), (r[3], eps_v), (r[4], pmax), (-r[5], -pmin), (r[6], vmax)]
    return min(abs(v - t) / abs(t) for v, t in vals)


KNIFE_EDGE = 0.02


def check_quality(tag, avg, mx, ok, report=None):
    """End-to-end parity for the chaotic / noise-terminated loops.

    The reference's own outcome moves with ±1 ulp on α0 and with the rounding of its matmuls
    (gen_golden*.py record both).  Required: the constraint flag is one the reference produced; the
    avg / max obstacle cost is no worse than the reference's worst + QUALITY_TOL and no better than
    its best − BETTER_TOL.
    """
    r = e2e_reference(tag)
    ens_avg = np.concatenate([r[v]["avg_cost"] for v in r])
    ens_max = np.concatenate([r[v]["max_cost"] for v in r])
    ens_ok = np.concatenate([r[v]["constraints_ok"] for v in r])
    print(f"{tag}: avg {avg:.4f} (ref [{ens_avg.min():.4f}, {ens_avg.max():.4f}]) "
          f"max {mx:.4f} (ref [{ens_max.min():.4f}, {ens_max.max():.4f}]) ok {ok}")
    assert ens_avg.min() - BETTER_TOL <= avg <= ens_avg.max() + QUALITY_TOL, (tag, avg, ens_avg)
    assert ens_max.min() - BETTER_TOL <= mx <= ens_max.max() + QUALITY_TOL, (tag, mx, ens_max)
    if bool(ok) not in set(bool(x) for x in ens_ok):
        # a flag the reference did not produce is accepted only on a knife edge: the deciding
        # quantity within KNIFE_EDGE (2 %) of its threshold (e.g. gd_n128: |T[N-1] − g| = 0.00996
        # against eps 0.01, where every reference run stopped just outside)
        assert report is not None, (tag, ok, ens_ok)
        m = constraint_margin(report)
        print(f"{tag}: flag {ok} on a knife edge (closest constraint {m:.2%} from its threshold)")
        assert m <= KNIFE_EDGE, (tag, ok, ens_ok, m)


# inner-iteration count within ±30 % of the reference's
ITER_BAND = 0.3
# ... where that count is a property of the run: if the reference's own ±1-ulp runs take counts more
# than this factor apart, the loop's termination is a coin flip (a first step whose improvement sits at
# loop_loss_reduction, the chaotic BLS cases) and the count is reported, not asserted.
ITER_COIN_FLIP = 5.0


def check_iterations(tag, grad_evals):
    """Gradient evaluations (= executed inner iterations) inside [0.7·min, 1.3·max] of the reference's
    runs — its ±1-ulp ensembles with its fp32 BLAS matmuls and with correctly rounded ones.  The
    dual-loop counts are set by summation noise: gd_n50 takes 272-334 gradient calls with BLAS
    matmuls and 760 with exact ones, gd_n500 188-191 and 399-402 — the same algorithm — so the band
    spans both arithmetics (this build's G is a rank-32 fp32 MFMA contraction, between the two)."""
    r = e2e_reference(tag)
    calls = np.concatenate([r[v]["grad_calls"] for v in r]).astype(float)
    lo, hi = (1 - ITER_BAND) * calls.min(), (1 + ITER_BAND) * calls.max()
    print(f"{tag}: grad evals {int(grad_evals)} (ref, BLAS / exact matmuls: [{int(calls.min())}, {int(calls.max())}])")
    if calls.max() > ITER_COIN_FLIP * max(calls.min(), 1.0):
        return
    assert lo <= float(grad_evals) <= hi, (tag, grad_evals, calls)
