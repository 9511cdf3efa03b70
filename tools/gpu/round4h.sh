# eval_exact's J source as a compile-time choice (no KParams copy in scratch): bit-identity against the
# previous library and interleaved timing of the dual-loop / BLS lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VARIANT=base CONFIGS="c3 --faithful|c3bls --faithful|c2 --faithful|c3bls" bash tools/gpu/abcheck.sh
# round-3 sources with the DynShape units under iterative-ILP (r3chk/, built in the container): the D = 5 case
# that left its band in round 3, run once
cd $GRAFT_REPO_ROOT/r3chk && timeout -k 10 300 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "generic_shapes_match_reference_iteration" > $GRAFT_REPO_ROOT/gpurun_out/r3ilp.log 2>&1; echo "r3 ilp rc $?"; grep -E "^FAILED|passed|failed|N=64 D=5" $GRAFT_REPO_ROOT/gpurun_out/r3ilp.log | tail -12
