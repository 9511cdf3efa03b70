cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u ${SCRIPT:-tools/bls_general_diverge.py} ${1:-bls_n500} > gpurun_out/diverge.log 2>&1; rc=$?; cat gpurun_out/diverge.log | tail -60; exit $rc
