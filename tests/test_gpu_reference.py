"""The HIP path against reference-produced fixtures at the bench shapes (GPU, through the C ABI).

Same fixtures and tolerances as tests/test_reference_bench.py (which pins the CPU oracle to them):
tests/golden/ref_bench_c3.npz / ref_bench_c4.npz / ref_bls_trials.npz / ref_e2e_r02.npz, written by
oracle/tools/gen_golden_bench.py from the unmodified reference.

  * C3 (BASELINE configs[2]: N=128, the reference's 11 obstacles; 32 problems) and C4 (N=256, 50
    random obstacles; 8 problems), GD single loop in bench mode from the reference's α0, against the
    reference with its own fp32 BLAS matmuls: k = 1..5 (C4 also 10, 20, 50) steps within
    max(2·spread_k, 1e-3) (SURVEY.md §8c's 1e-3, widened to the reference's own ±1-ulp sensitivity
    after k steps), loss rtol 1e-3; 200 steps within max(2·spread, 3e-3) of the reference's
    trajectory and the final loss inside the reference ensemble's range ± 1e-3 relative.  k_lean
    carries α in fp32 with the reference's rounding (irm_kernels_impl.hpp), which is
    what keeps it inside this band: the same iteration in exact arithmetic ends 1-4e-2 away at C3.
  * BLS line search (optimizer_BLS.py:135-179), the first 4 inner iterations of problem 0 from the
    kernel's line-search log (irm_debug_bls_trace): accept / reject sequence identical, lr exact,
    losses / ‖g‖ / alpha_norm rtol 1e-5 from a well-conditioned α and 2e-3 / 5e-3 / 3e-2 from the
    reference's α0 (K@α0 carries fp32 noise there).
  * Reference control flow end to end (GD λ_max table, N=128 / 256, BLS at N=256 with C4's
    obstacles): conftest.check_quality and the ±30 % gradient-evaluation band.
"""
import numpy as np
import pytest

from conftest import GOAL, START, check_iterations, check_quality, golden, params
from test_reference_bench import (BENCH_ARGS, BLS_CASES, BLS_LOG_ARGS, E2E_R02, bench_band, check_bls_log,
                                  check_first_steps, e2e_alpha0, e2e_obstacles, loss_band)

pytestmark = pytest.mark.gpu

_CTX = {}


def ctx(*argv, **overrides):
    from irm_motion_planning_amd.context import Context
    key = (tuple(str(a) for a in argv), tuple(sorted(overrides.items())))
    if key not in _CTX:
        _CTX[key] = Context(params(*argv, **overrides))
    return _CTX[key]


# Problems of the committed fixtures at which the reference's BLAS and exact-matmul runs part at a
# decision knife edge: C3 problems 8 (k = 1, 2) and 15 (k = 4) in the k-step test, C4
# problem 7 after 200 steps (the N = 256 run is chaotic by then).  Named, not counted.
KNIFE_EDGE_PROBLEMS = {"c3": {8, 15}, "c4": set()}
VIA_XM_PROBLEMS = {"c3": set(), "c4": {7}}


@pytest.fixture(scope="module")
def fx():
    names = ("ref_bench_c3", "ref_bench_c4", "ref_bls_trials", "ref_e2e_r02")
    return {name: golden(name) for name in names}


def _exact(c, alpha):
    """K·α·J in exact arithmetic (the reference's own evaluate adds the fp32 noise of K@α, |α| ≈ 1e3)."""
    _, K, _, J = c.kernel_matrices()
    return np.asarray(K, np.float64) @ np.asarray(alpha, np.float64) @ np.asarray(J, np.float64)


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_gd_first_steps_match_reference(fx, cfg):
    """The k-step GD iterates (C3: k = 1..5 on 32 problems; C4: k = 1..5, 10, 20, 50 on 8 problems)
    against the reference run with its own fp32 BLAS matmuls (test_reference_bench.check_first_steps):
    |traj − ref| ≤ max(2·spread_k, 1e-3) with spread_k the reference's own change after k steps under
    ±1 ulp on α0 — except at an argmax knife edge of the max-cost term (two waypoint potentials within
    the reference's K@α0 noise), where the result must match the reference re-run with correctly rounded
    matmuls instead; loss within max(1e-3 relative, 3·its ±1-ulp change).  The widest band used is
    printed."""
    from conftest import oracle_for
    z = fx["ref_bench_" + cfg]
    zx = golden("ref_bench_" + cfg + "_xm")
    N = int(z["traj_final"].shape[1])
    widest, edges = 0.0, []
    for i, k in enumerate(z["ks"]):
        c = ctx(*BENCH_ARGS, "--n-timesteps", N, "--max-inner-iteration", int(k))
        o = oracle_for(*BENCH_ARGS, "--n-timesteps", N, "--max-inner-iteration", int(k))
        alpha, traj, st = c.optimize(z["start"], z["goal"], z["obstacles"], alpha0=z["alpha0"])
        assert np.all(st["grad_evals"] == k)
        errs = []
        for b in range(len(z["start"])):
            zm, err, band, m = check_first_steps(o, z, zx, b, i, traj[b])
            widest = max(widest, band)
            errs.append(err)
            if m is not None:
                edges.append((int(k), b, m))
            assert abs(float(st["final_loss"][b]) - zm["loss_k"][b, i]) <= loss_band(o, zm, b, i), (k, b)
        print(f"{cfg} {k} steps: |traj - ref (BLAS)| max {max(errs):.2e} over {len(errs)} problems")
    print(f"{cfg}: widest band used {widest:.2e}; argmax knife edges {edges}")
    # the problems whose max-cost argmax is a knife edge of the reference's own K@α0 noise (measured
    # margins 8e-5 / 3e-6 at C3, none at C4): only these may take the exact-matmul reference's band
    assert {b for _, b, _ in edges} <= KNIFE_EDGE_PROBLEMS[cfg] and len(edges) <= 3, edges


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_gd_200_steps_inside_reference_spread(fx, cfg):
    """200 bench-mode GD steps (C3: 32 problems, C4: 8) against the reference's own run and its ±1-ulp
    ensemble: |traj − ref| ≤ bench_band(spread), the final loss inside the ensemble's range ± 1e-3
    relative.  At C4 the run is chaotic by 200 steps (spreads up to 0.2, near-tied max-cost argmaxes at
    almost every step of N = 256); there a problem may instead lie in the band of the reference re-run
    with correctly rounded matmuls — the reference's own outcome moves between its two contraction
    arithmetics by as much as its ±1-ulp spread (|BLAS − exact| 1.7e-3 … 0.17 at C4) — and the C4 path is
    pinned step by step up to k = 50 by test_gd_first_steps_match_reference."""
    z = fx["ref_bench_" + cfg]
    zx = golden("ref_bench_" + cfg + "_xm")
    N = int(z["traj_final"].shape[1])
    c = ctx(*BENCH_ARGS, "--n-timesteps", N, "--max-inner-iteration", int(z["steps"]))
    alpha, traj, st = c.optimize(z["start"], z["goal"], z["obstacles"], alpha0=z["alpha0"])
    assert np.all(st["grad_evals"] == int(z["steps"]))
    np.testing.assert_array_equal(c.evaluate(alpha), traj)  # traj_out = K·α_out·J, correctly rounded
    via_xm = []
    for b in range(len(z["start"])):
        res = []
        for name, zz in (("blas", z), ("xm", zx)):
            ref = _exact(c, zz["alpha_final"][b])
            spread = max(float(np.abs(_exact(c, a) - ref).max()) for a in zz["ens_alpha_final"][b])
            err = float(np.abs(traj[b] - ref).max())
            losses = np.append(zz["ens_loss_final"][b], zz["loss_final"][b])
            tol = 1e-3 * abs(float(zz["loss_final"][b]))
            loss = float(st["final_loss"][b])
            ok = err <= bench_band(spread) and losses.min() - tol <= loss <= losses.max() + tol
            res.append((ok, name, err, spread, loss, losses.min(), losses.max()))
        print(f"{cfg}[{b}] 200 steps: " + "; ".join(
            f"{n}: |traj - ref| {e:.2e} (band {bench_band(sp):.2e}), loss {lo:.6f} (ref [{a:.6f}, {m:.6f}])"
            for _, n, e, sp, lo, a, m in res))
        if cfg == "c3":
            assert res[0][0], (cfg, b, res[0])  # C3: the BLAS reference alone
        else:
            assert res[0][0] or res[1][0], (cfg, b, res)
            if not res[0][0]:
                via_xm.append(b)
    print(f"{cfg}: problems inside the exact-matmul reference's band only: {via_xm}")
    assert set(via_xm) <= VIA_XM_PROBLEMS[cfg], via_xm


@pytest.mark.parametrize("N,kind", BLS_CASES)
def test_bls_line_search_log_matches_reference(fx, N, kind):
    z = fx["ref_bls_trials"]
    pre = f"n{N}_{kind}__"
    c = ctx("--n-timesteps", N, *BLS_LOG_ARGS)
    c.bls_trace_enable(256)
    _, _, st = c.optimize(START, GOAL, z[pre + "obstacles"], alpha0=z[pre + "alpha_init"])
    tr = c.bls_trace(int(st["bls_trials"]))
    print(f"N={N} {kind}: {len(tr)} trials, accepted {tr[:, 6].astype(int).tolist()}")
    check_bls_log(tr, z, N, kind)


@pytest.mark.parametrize("tag", sorted(E2E_R02))
def test_end_to_end_r02(tag):
    argv, src = E2E_R02[tag]
    c = ctx(*argv)
    obs = e2e_obstacles(src)
    alpha, _, st = c.optimize(START, GOAL, obs, alpha0=e2e_alpha0(tag))
    avg = float(c.eval_cost(alpha, obs, START, GOAL, 0, 0, 0))
    mx = float(c.eval_cost(alpha, obs, START, GOAL, 0, 0, 1))
    ok, rep = c.constraints(alpha, START, GOAL)
    check_quality(tag, avg, mx, ok, rep)
    check_iterations(tag, st["grad_evals"])


def test_bls_n500_ulp_ensemble_inside_reference_band():
    """bls_n500 is noise-terminated (one ulp of α, |α| ≈ 1.6e3, moves the endpoint velocities by ~2e-3):
    its outcome is judged as a distribution.  The general kernel's BLS, evaluating every trial's fp32
    iterate exactly, from the reference's α0 moved by ±1 ulp (gen_golden.py's ensemble scheme, seeds
    100-104): every run fulfils the constraints, with gradient evaluations inside the reference
    ensemble's band (measured: 76-127 over 11 seeds, the oracle's 76-128, the reference's 89-122; with
    trial trajectories taking their rounding one step late the same seeds gave 47-67, 3 of 11 failing)."""
    from conftest import e2e_reference, oracle_for
    argv, src = E2E_R02["bls_n500"]
    c = ctx(*argv)
    o = oracle_for(*argv)
    obs = e2e_obstacles(src)
    a0 = e2e_alpha0("bls_n500")
    r = e2e_reference("bls_n500")
    calls = np.concatenate([r[v]["grad_calls"] for v in r]).astype(float)
    # band: the reference ensemble's range widened to the oracle's own spread (76-128) plus a small
    # margin — tight enough to exclude the one-step-late scheme's 47-67
    lo, hi = 0.8 * calls.min(), 1.15 * calls.max()
    got = []
    for seed in range(5):
        sgn = np.random.default_rng(100 + seed).choice([-1.0, 1.0], a0.shape).astype(np.float32)
        ap = np.nextafter(a0, a0 + sgn * np.float32(np.inf)).astype(np.float32)
        al, _, st = c.optimize(START, GOAL, obs, alpha0=ap)
        ok = o.constraints(np.asarray(al, np.float32), START, GOAL)[0]
        got.append(int(st["grad_evals"]))
        assert ok and bool(st["constraints_ok"]), (seed, got)
    print(f"bls_n500 ±1-ulp ensemble: grad evals {got} (reference {calls.astype(int).tolist()})")
    assert all(lo <= x <= hi for x in got), (got, lo, hi)
