"""The vectorised fp32 CPU baseline (oracle/batched_np.py, bench.py's cpu_baseline "batched" variant)
against the scalar C oracle: the same GD iteration (optimizer_GD.py:76-91, bench mode) on the same α0.
The two differ only in contraction rounding (fp32 sgemm vs fp64-accumulated, rounded once), which the
iteration carries as the reference's own BLAS-vs-exact spread (1e-3 after 20 C3 steps)."""
import numpy as np


def test_batched_gd_matches_oracle():
    import bench
    from irm_motion_planning_amd.params import params_from_args
    from oracle import batched_np
    from oracle.oracle import Oracle
    args = bench.make_args("c3", False, 20)
    p = params_from_args(args)
    o = Oracle(p)
    _, K, dK, J = o.kernel_matrices()
    s, g, obs = bench.make_problem("c3", 1, 0)
    B = 6
    a0 = np.stack([o.init_alpha(s[b], g[b]) for b in range(B)])
    a, loss = batched_np.BatchedGD(K, dK, J, p).run(a0, s[:B], g[:B], obs, 20)
    Kd, Jd = K.astype(np.float64), J.astype(np.float64)
    for b in range(B):
        ao, so = o.optimize(a0[b], obs, s[b], g[b])
        assert so["grad_evals"] == 20
        err = float(np.abs(Kd @ a[b] @ Jd - Kd @ ao @ Jd).max())
        assert err < 5e-3, (b, err)
        assert abs(float(loss[b]) - so["final_loss"]) <= 1e-3 * abs(so["final_loss"]), (b, loss[b], so)
    # the process-parallel driver computes the same batch (to the rounding of a narrower sgemm)
    a2, l2, _ = batched_np.run_processes(K, dK, J, p, a0, s[:B], g[:B], obs, 20, 2)
    np.testing.assert_allclose(a2, a, rtol=0, atol=1e-2)
    np.testing.assert_allclose(l2, loss, rtol=1e-3)  # sgemm rounding moves with the chunk width


def test_batched_baseline_only_for_the_gd_bench_loop():
    import bench
    assert bench.cpu_baseline_batched(bench.make_args("c3bls", False, 20), None, None, None, 1) is None
    assert bench.cpu_baseline_batched(bench.make_args("c3", True, 20), None, None, None, 1) is None
