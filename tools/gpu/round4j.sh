# round-2 sources (the commit that kept the DynShape units on the default scheduler) with the DynShape units
# under the default and the iterative-ILP scheduler: the D = 5 generic-shape case, once each; then the
# round-end profiles of the default bench command (r04)
cd $GRAFT_REPO_ROOT/r2chk
for v in def ilp; do
  if [ $v = def ]; then L=$GRAFT_REPO_ROOT/r2chk/irm_motion_planning_amd/libirm_hip_def.so; else L=$GRAFT_REPO_ROOT/r2chk/irm_motion_planning_amd/libirm_hip.so; fi
  IRM_LIB=$L timeout -k 10 300 python -u -m pytest -q -rf -s --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "generic_shapes_match_reference_iteration" > $GRAFT_REPO_ROOT/gpurun_out/r2_$v.log 2>&1; echo "r2 $v rc $?"; grep -E "^FAILED|passed|failed|N=64 D=5" $GRAFT_REPO_ROOT/gpurun_out/r2_$v.log | tail -10
done
cd $GRAFT_REPO_ROOT && bash tools/final_profile.sh r04
