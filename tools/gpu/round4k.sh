# cross-workgroup wave priority for the 256-thread lean kernels (C7): bit-identity + interleaved timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VARIANT=base CONFIGS="c7|c7 --faithful" bash tools/gpu/abcheck.sh
