#!/bin/bash
# Round-end evidence on the GPU box: default bench line (with CPU baseline), C4 and faithful C3 lines,
# rocprof kernel stats + PMC traffic, PMC-counted flops and SQ counters of the default bench command.
#   tools/final_profile.sh r02
R=${1:?round tag}
mkdir -p gpurun_out
tools/gpu_steps.sh \
  "bench:180:python bench.py > gpurun_out/${R}_bench.json" \
  "bench_c4:180:python bench.py --config c4 > gpurun_out/${R}_bench_c4.json" \
  "bench_faithful:180:python bench.py --faithful > gpurun_out/${R}_bench_c3_faithful.json" \
  "prof:600:bash tools/profile_round.sh $R" \
  "flops:300:bash tools/pmc_flops.sh $R" \
  "sq:600:bash tools/pmc_sq.sh $R > gpurun_out/${R}_sq_counters.txt"
