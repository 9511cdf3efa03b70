# Round-3 evidence: C3 kernel stats + HBM traffic + counted flops + SQ counters; the BLS faithful line's
# stats, SQ counters and per-problem round breakdown; C3 faithful breakdown
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
R=r03
tools/gpu_steps.sh \
  "prof:600:bash tools/profile_round.sh $R" \
  "flops:300:bash tools/pmc_flops.sh $R" \
  "sq:600:bash tools/pmc_sq.sh $R > gpurun_out/${R}_sq_counters.txt" \
  "prof_bls:600:bash tools/profile_round.sh ${R}_c3bls_faithful --config c3bls --faithful" \
  "sq_bls:600:bash tools/pmc_sq.sh ${R}_bls > gpurun_out/${R}_c3bls_faithful_sq_counters.txt --config c3bls --faithful" \
  "rounds_bls:300:python tools/faithful_rounds.py c3bls > gpurun_out/${R}_c3bls_faithful_rounds.txt" \
  "rounds_c3:300:python tools/faithful_rounds.py c3 > gpurun_out/${R}_c3_faithful_rounds.txt"
