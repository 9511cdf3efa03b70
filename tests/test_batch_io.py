"""Batched output files and the replanning API's host side (CPU)."""
import numpy as np
import pytest

from conftest import GOAL, START


def test_batch_problems_problem0_is_reference_env():
    from irm_motion_planning_amd import batch_io
    s, g = batch_io.batch_problems(16, 3, seed=1)
    assert s.shape == g.shape == (16, 3) and s.dtype == np.float32
    np.testing.assert_array_equal(s[0], START)
    np.testing.assert_array_equal(g[0], GOAL)
    assert np.all((s[1:] >= -0.5) & (s[1:] < 0.5)) and np.all((g[1:] >= 0.2) & (g[1:] < 1.6))
    s2, _ = batch_io.batch_problems(16, 3, seed=1)
    np.testing.assert_array_equal(s, s2)  # seeded
    s7, g7 = batch_io.batch_problems(4, 7, seed=4)
    assert s7.shape == (4, 7) and not np.array_equal(s7[0], np.zeros(7))


def test_result_files_use_reference_format(tmp_path):
    """main.py:145-153 write np.savetxt defaults; the reference's loaders read them back
    (visualization.py:91 loadtxt; visualize_series.py:164 reshape((-1, N, D)))."""
    from irm_motion_planning_amd import batch_io
    rng = np.random.default_rng(0)
    traj = rng.standard_normal((5, 50, 3)).astype(np.float32)
    batch_io.write_result(tmp_path / batch_io.RESULT, traj[0])
    txt = (tmp_path / batch_io.RESULT).read_text().splitlines()
    assert len(txt) == 50 and len(txt[0].split(" ")) == 3 and "e" in txt[0]
    assert len(txt[0].split(" ")[0].split("e")[0].split(".")[1]) == 18  # '%.18e'
    np.testing.assert_array_equal(np.loadtxt(tmp_path / batch_io.RESULT).astype(np.float32), traj[0])
    batch_io.write_result_batch(tmp_path / batch_io.RESULT_BATCH, traj)
    back = batch_io.read_result_batch(tmp_path / batch_io.RESULT_BATCH, 50, 3)
    np.testing.assert_array_equal(back.astype(np.float32), traj)
    # the batch file has the series layout: the reference's series reader takes it as is
    np.testing.assert_array_equal(np.loadtxt(tmp_path / batch_io.RESULT_BATCH).reshape((-1, 50, 3)).astype(np.float32),
                                  traj)
    batch_io.write_series(tmp_path / batch_io.SERIES, traj[:3], 50, 3)
    assert np.loadtxt(tmp_path / batch_io.SERIES).shape == (3, 150)


def test_series_batch_and_summary_round_trip(tmp_path):
    from irm_motion_planning_amd import batch_io
    ser = np.arange(2 * 4 * 6 * 3, dtype=np.float32).reshape(2, 4, 6, 3)
    batch_io.write_series_batch(tmp_path / batch_io.SERIES_BATCH, ser, [4, 2])
    frames = batch_io.read_series_batch(tmp_path / batch_io.SERIES_BATCH)
    assert [f.shape for f in frames] == [(4, 6, 3), (2, 6, 3)]
    np.testing.assert_array_equal(frames[1], ser[1, :2])
    st = {"inner_iterations": np.array([3, 4]), "outer_iterations": np.array([1, 2]),
          "grad_evals": np.array([9, 8])}
    batch_io.write_summary(tmp_path / batch_io.SUMMARY_BATCH, [1.5, 2.5], [2.0, 3.0], [True, False], st)
    tab = np.loadtxt(tmp_path / batch_io.SUMMARY_BATCH)
    np.testing.assert_array_equal(tab, [[1.5, 2.0, 1, 3, 1, 9], [2.5, 3.0, 0, 4, 2, 8]])


def test_replanner_refuses_without_device():
    """No CPU fallback: without a gfx950 device the replanner fails loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from conftest import ref_args
    from irm_motion_planning_amd._abi import IrmError
    from irm_motion_planning_amd.replanning import Replanner
    with pytest.raises(IrmError):
        Replanner(ref_args("--optimizer-name", "gd"), batch=4, n_obstacles=11)
