# round-1 sources: the ILP build with the cross-row permlane swaps padded by wait states (r2chk/ nop
# library) — deterministic again? then the BLS faithful line's rounds, kernel stats and SQ counters (r04)
cd $GRAFT_REPO_ROOT/r2chk
IRM_LIB=$GRAFT_REPO_ROOT/r2chk/irm_motion_planning_amd/libirm_hip_nop.so timeout -k 10 120 python firstdiv.py $GRAFT_REPO_ROOT/gpurun_out/fd_nop.npz > $GRAFT_REPO_ROOT/gpurun_out/fd_nop.log 2>&1 || { echo "fd nop failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/fd_nop.log; exit 2; }
echo "== def vs nop-padded ILP"; python firstdiv_cmp.py $GRAFT_REPO_ROOT/gpurun_out/fd_def.npz $GRAFT_REPO_ROOT/gpurun_out/fd_nop.npz
cd $GRAFT_REPO_ROOT
tools/gpu_steps.sh \
  "bls_rounds:240:python tools/faithful_rounds.py c3bls > gpurun_out/r04_c3bls_faithful_rounds.txt" \
  "bls_prof:600:bash tools/profile_round.sh r04_c3bls_faithful --config c3bls --faithful" \
  "bls_sq:600:bash tools/pmc_sq.sh r04_c3bls_faithful --config c3bls --faithful > gpurun_out/r04_c3bls_faithful_sq_counters.txt"
