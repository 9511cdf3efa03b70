# scratch-fix A/B + round-3 ILP D=5 check, then the full suite and every config's bench line (r04)
cd $GRAFT_REPO_ROOT
bash tools/gpu/round4h.sh
cd $GRAFT_REPO_ROOT && bash tools/gpu/round4_final1.sh
