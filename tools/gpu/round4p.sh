# phase profile of the final lean kernels (IRM_PHASE_PROFILE build of the current sources): BLS bench and C3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IRM_PROFILE_LEAN=1 IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_prof.so timeout -k 10 200 python tools/phase_profile.py c3bls c3 > gpurun_out/phase_lean_r04.txt 2>&1 || { echo "lean phase profile failed"; tail -5 gpurun_out/phase_lean_r04.txt; exit 2; }
cat gpurun_out/phase_lean_r04.txt
