# BLS: stage 1 stores only the y'' columns of slots taking a new direction; the velocity half only for
# those: BLS / helper / neighbour GPU tests, bit-identity on sched_check's cases, interleaved timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests/ -k "bls or BLS or helpers or neighbour or flows or c2" > gpurun_out/q_tests.log 2>&1; rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/q_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
VARIANT=base CONFIGS="c3bls|c3bls --faithful|c2 --faithful" bash tools/gpu/abcheck.sh
