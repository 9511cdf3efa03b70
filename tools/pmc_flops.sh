#!/bin/bash
# Issued fp32 flops of the optimiser launch from SQ instruction counters (GPU box), one rocprofv3
# --pmc pass (6 SQ counters), then tools/summarize_flops.py writes profiles/<tag>_flops.json, which
# bench.py reads for roofline.counted_flops_per_launch.
#   tools/pmc_flops.sh r02 [--config c3 ...]
R=${1:?round tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/flops_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 \
    SQ_INSTS_VALU_TRANS_F32 SQ_WAVES --output-format csv -d "$OUT/p1" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/p1.log" 2>&1 || { echo "flops pass failed"; exit 3; }
cd "$ROOT" && python3 tools/summarize_flops.py "$R" "$OUT" "$@"
