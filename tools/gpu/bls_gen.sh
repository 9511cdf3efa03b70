# k_optimize BLS (exact trial evaluation) checks: the trial-log test, the e2e ensemble, then the full -m gpu suite
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "general_kernel_bls" > gpurun_out/bg1.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|trials|passed|failed" gpurun_out/bg1.log | tail -20
if [ $rc -ne 0 ]; then echo "rc $rc"; exit $rc; fi
timeout -k 10 300 python -u tools/e2e_ensemble.py bls_n500 > gpurun_out/bg_ens.log 2>&1 || { echo "ensemble rc $?"; tail -5 gpurun_out/bg_ens.log; exit 3; }
tail -13 gpurun_out/bg_ens.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/bg2.log 2>&1
rc=$?; tail -5 gpurun_out/bg2.log; exit $rc
