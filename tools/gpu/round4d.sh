cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu/suite_nox.sh || exit $?
timeout -k 10 300 python tools/help_ab.py c3bls 1024 || exit $?
timeout -k 10 120 python tools/help_ab.py c2 1 || exit $?
LIBS="base release" CONFIGS="c3|c3bls|c2 --faithful|c3bls --faithful|c7 --faithful|c5 --faithful|c4|c7|c5" REPS=1 bash tools/gpu/varab.sh
