cd $GRAFT_REPO_ROOT
export IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_prof.so IRM_PROFILE_LEAN=1
echo "---- k_lean"; timeout -k 10 120 python tools/phase_profile.py c3 || exit 2
