# dense operand-stream restructure (stage-1 batches prefetched across units, stage-2 split reads batched)
# against the previous library: bit-identity and interleaved timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VARIANT=base CONFIGS="c5 --operator-rank -1|c3 --operator-rank -1" bash tools/gpu/abcheck.sh
