# full -m gpu suite, then the faithful lines
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/c2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/c2_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc"; exit $rc; fi
CONFIGS="c3 --faithful|c4 --faithful|c5 --faithful|c7 --faithful|c3bls --faithful|c3|c4" bash tools/gpu/ab1.sh
