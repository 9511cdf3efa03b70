# same-box A/B of a build variant against the release library, interleaved runs
#   VARIANT=nogdefer CONFIGS="c3|c3 --faithful" bash tools/gpu/ab2.sh
cd $GRAFT_REPO_ROOT
V=${VARIANT:-nogdefer}
IFS='|' read -ra CFGS <<< "${CONFIGS:-c3}"
for rep in 1 2 3; do
  for c in "${CFGS[@]}"; do
    tag=$(echo $c | tr ' ' '_' | tr -d '-')
    for lib in release $V; do
      if [ $lib = release ]; then L=irm_motion_planning_amd/libirm_hip.so; else L=irm_motion_planning_amd/libirm_hip_$lib.so; fi
      IRM_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab2_${tag}_$lib.json 2> gpurun_out/ab2.err || { echo "bench $c $lib failed"; tail -3 gpurun_out/ab2.err; exit 2; }
      python -c "import json;d=json.loads(open('gpurun_out/ab2_${tag}_$lib.json').read().strip().splitlines()[-1]);print('$rep $tag $lib', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
    done
  done
done
