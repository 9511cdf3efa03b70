# per-phase cycle breakdown of the lean kernel (IRM_PHASE_PROFILE build) for the given configs
cd $GRAFT_REPO_ROOT
export IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_prof.so IRM_PROFILE_LEAN=1
timeout -k 10 240 python tools/phase_profile.py ${CONFIGS:-c3 c3bls} > gpurun_out/phase.log 2>&1; rc=$?; cat gpurun_out/phase.log | grep -v amdgpu.ids; exit $rc
