# printed measurements of the reference-pinning GPU tests (for DESIGN.md)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_reference.py > gpurun_out/refnums.log 2>&1
rc=$?; grep -E "widest|problems inside|ensemble|grad evals|max over|passed|failed" gpurun_out/refnums.log | tail -40; exit $rc
