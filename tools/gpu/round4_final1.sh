# round-end evidence, part 1: the full -m gpu suite + smoke, then every config's bench line (r04)
cd $GRAFT_REPO_ROOT
bash tools/gpu/suite_nox.sh || exit $?
bash tools/gpu/round_lines.sh r04
