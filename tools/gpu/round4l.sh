# round-1 sources (r2chk/): first GD step where the default- and ILP-scheduled DynShape<5> builds part;
# then the cross-workgroup priority A/B for the 256-thread lean kernels (C7)
cd $GRAFT_REPO_ROOT/r2chk
IRM_LIB=$GRAFT_REPO_ROOT/r2chk/irm_motion_planning_amd/libirm_hip_def.so timeout -k 10 120 python firstdiv.py $GRAFT_REPO_ROOT/gpurun_out/fd_def.npz > $GRAFT_REPO_ROOT/gpurun_out/fd_def.log 2>&1 || { echo "fd def failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/fd_def.log; exit 2; }
IRM_LIB=$GRAFT_REPO_ROOT/r2chk/irm_motion_planning_amd/libirm_hip.so timeout -k 10 120 python firstdiv.py $GRAFT_REPO_ROOT/gpurun_out/fd_ilp.npz > $GRAFT_REPO_ROOT/gpurun_out/fd_ilp.log 2>&1 || { echo "fd ilp failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/fd_ilp.log; exit 2; }
python firstdiv_cmp.py $GRAFT_REPO_ROOT/gpurun_out/fd_def.npz $GRAFT_REPO_ROOT/gpurun_out/fd_ilp.npz
cd $GRAFT_REPO_ROOT && bash tools/gpu/round4k.sh
