"""Batched problems and the reference's output files for a batch.

The reference writes one trajectory per run (main.py:145-153):

  trajectory_result.txt   N × D          np.savetxt defaults ('%.18e', ' ', '\\n')
  trajectory_series.txt   frames × N·D   (visualize_series.py:164 reads it back with
                                          .reshape((-1, n_timesteps, n_joints)))

A batched run keeps both files for problem 0 — the reference environment's own
start/goal — so every reference visualisation script reads them unchanged, and adds

  trajectory_result_batch.txt   B × N·D        one row per problem, the series layout
                                               (np.loadtxt(...).reshape((-1, N, D)))
  trajectory_series_batch.npz   series (B × S × N × D), series_len (B)  with --extended-vis
  trajectory_batch_summary.txt  per problem: avg cost, max cost, constraint flag,
                                inner / outer iterations, gradient evaluations
"""
import numpy as np

from .environment import GOAL_CONFIG, START_CONFIG

RESULT = "trajectory_result.txt"
SERIES = "trajectory_series.txt"
RESULT_BATCH = "trajectory_result_batch.txt"
SERIES_BATCH = "trajectory_series_batch.npz"
SUMMARY_BATCH = "trajectory_batch_summary.txt"
SUMMARY_COLUMNS = ("avg_cost", "max_cost", "constraints_ok", "inner_iterations", "outer_iterations", "grad_evals")


def batch_problems(batch, n_joints, seed):
    """B start/goal pairs (B × D float32).

    Problem 0 is the reference environment (environment.py:14-15) when D = 3;
    the rest are drawn like SURVEY.md §8d's C3 batch: start U(−0.5, 0.5)^D,
    goal U(0.2, 1.6)^D from numpy default_rng(seed).
    """
    rng = np.random.default_rng(seed)
    start = rng.uniform(-0.5, 0.5, (batch, n_joints)).astype(np.float32)
    goal = rng.uniform(0.2, 1.6, (batch, n_joints)).astype(np.float32)
    if n_joints == 3 and batch > 0:
        start[0] = START_CONFIG
        goal[0] = GOAL_CONFIG
    return start, goal


def write_result(path, traj):
    """One trajectory (N × D) exactly as main.py:145-146 writes it."""
    np.savetxt(path, np.asarray(traj))


def write_series(path, frames, n_timesteps, n_joints):
    """Snapshots (frames × N × D) as main.py:150-153 writes them."""
    np.savetxt(path, np.asarray(frames).reshape((-1, n_joints * n_timesteps)))


def write_result_batch(path, traj):
    """B × N × D → B rows of N·D values (same format and row layout as the series file)."""
    traj = np.asarray(traj)
    np.savetxt(path, traj.reshape(traj.shape[0], -1))


def read_result_batch(path, n_timesteps, n_joints):
    return np.loadtxt(path, ndmin=2).reshape((-1, n_timesteps, n_joints))


def write_series_batch(path, series, series_len):
    np.savez(path, series=np.asarray(series, np.float32), series_len=np.asarray(series_len, np.int32))


def read_series_batch(path):
    """[frames_b (series_len_b × N × D) for each problem b] — allow_pickle stays off."""
    with np.load(path) as z:
        ser, ln = z["series"], z["series_len"]
    return [ser[b, : int(ln[b])] for b in range(ser.shape[0])]


def write_summary(path, avg, mx, ok, stats):
    cols = [np.asarray(avg, np.float64), np.asarray(mx, np.float64), np.asarray(ok, np.int64),
            np.asarray(stats["inner_iterations"]), np.asarray(stats["outer_iterations"]),
            np.asarray(stats["grad_evals"])]
    table = np.stack([np.asarray(c, np.float64) for c in cols], axis=1)
    np.savetxt(path, table, fmt=["%.9g", "%.9g", "%d", "%d", "%d", "%d"], header=" ".join(SUMMARY_COLUMNS))
