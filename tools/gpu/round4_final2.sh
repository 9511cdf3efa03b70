# round-end evidence, part 2 (r04): default bench line + C4 + C3 faithful, rocprof kernel stats + PMC
# traffic, PMC-counted flops and SQ counters of the default bench command; then the BLS faithful line's
# round distribution, kernel stats and SQ counters
cd $GRAFT_REPO_ROOT
bash tools/final_profile.sh r04 || exit $?
tools/gpu_steps.sh \
  "bls_rounds:240:python tools/faithful_rounds.py c3bls > gpurun_out/r04_c3bls_faithful_rounds.txt" \
  "bls_prof:600:bash tools/profile_round.sh r04_c3bls_faithful --config c3bls --faithful" \
  "bls_sq:600:bash tools/pmc_sq.sh r04_c3bls_faithful --config c3bls --faithful > gpurun_out/r04_c3bls_faithful_sq_counters.txt"
