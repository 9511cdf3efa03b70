# the three oracle-band tests under each build, then the step ladder of C4 problem 42
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T="tests/test_gpu_parity.py::test_bench_c4_random_obstacles tests/test_gpu_parity.py::test_dense_operator_at_n256 tests/test_gpu_parity.py::test_per_problem_obstacles_and_edge_counts"
for v in base c1; do
  IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_$v.so timeout -k 10 300 python -m pytest -q -rf -s -m gpu $T > gpurun_out/f3_$v.log 2>&1; rc=$?
  echo "== $v rc $rc"; grep -E "^FAILED|passed|failed" gpurun_out/f3_$v.log
  [ $rc -gt 1 ] && exit $rc
done
for v in c1 release; do
  if [ $v = release ]; then L=libirm_hip.so; else L=libirm_hip_$v.so; fi
  echo "== drift $v"; IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/$L timeout -k 10 300 python tools/drift_diag.py c4 42 || exit 2
done
