# full -m gpu suite without -x (every failure listed) + smoke; stops on a crash / timeout
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests/ ${TESTS:-} ${KEXPR:+-k "$KEXPR"} > gpurun_out/suite.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/suite.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc2=$?; tail -2 gpurun_out/smoke.log; [ $rc2 -ne 0 ] && exit $rc2; exit 0
