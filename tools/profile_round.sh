#!/bin/bash
# Kernel-time and HBM-traffic profiles of the default bench command (GPU box).
#   tools/profile_round.sh r01 [extra bench args...]
# 1. rocprofv3 --kernel-trace --stats        → per-kernel durations
# 2. rocprofv3 --pmc FETCH_SIZE (own pass)   → L2→fabric read bytes
# 3. rocprofv3 --pmc WRITE_SIZE (own pass)   → write bytes
# then tools/summarize_profile.py copies the summaries into profiles/.
R=${1:?round tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/stats.log" 2>&1 || { echo "stats pass failed"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 5 --warmup 1 "$@" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --steps 5 --warmup 1 "$@" > "$OUT/write.log" 2>&1 || { echo "write pass failed"; exit 3; }
cd "$ROOT" && python3 tools/summarize_profile.py "$R" "$OUT" "$@"
