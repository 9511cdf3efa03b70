# dense C5: phase profile (IRM_PHASE_PROFILE build of the previous sources), dense tests, and the
# operand-prefetch build against the previous library (bit-identity + interleaved timing)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_prof.so timeout -k 10 200 python tools/phase_profile.py c5@-1 c3@-1 > gpurun_out/phase_dense.txt 2>&1 || { echo "phase profile failed"; tail -5 gpurun_out/phase_dense.txt; exit 2; }
cat gpurun_out/phase_dense.txt
timeout -k 10 300 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests/ -k "dense or operator_rank" > gpurun_out/dense_tests.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/dense_tests.log | tail -10
[ $rc -ne 0 ] && exit $rc
VARIANT=base CONFIGS="c5 --operator-rank -1|c3 --operator-rank -1" bash tools/gpu/abcheck.sh
IRM_PROFILE_LEAN=1 IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_prof.so timeout -k 10 200 python tools/phase_profile.py c3bls c3 > gpurun_out/phase_lean.txt 2>&1 || { echo "lean phase profile failed"; tail -5 gpurun_out/phase_lean.txt; exit 2; }
cat gpurun_out/phase_lean.txt
