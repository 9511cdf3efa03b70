# same-box timing of several library variants, interleaved (release = libirm_hip.so)
#   VARIANTS="release base nogb" CONFIGS="c3|c3 --faithful" REPS=3 bash tools/gpu/abn.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IFS='|' read -ra CFGS <<< "${CONFIGS:-c3}"
for rep in $(seq 1 ${REPS:-3}); do
  for c in "${CFGS[@]}"; do
    tag=$(echo $c | tr ' ' '_' | tr -d '-')
    for lib in ${VARIANTS:-release base}; do
      if [ $lib = release ]; then L=irm_motion_planning_amd/libirm_hip.so; else L=irm_motion_planning_amd/libirm_hip_$lib.so; fi
      IRM_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/abn_${tag}_$lib.json 2> gpurun_out/abn.err || { echo "bench $c $lib failed"; tail -3 gpurun_out/abn.err; exit 2; }
      python -c "import json;d=json.loads(open('gpurun_out/abn_${tag}_$lib.json').read().strip().splitlines()[-1]);print('$rep $tag $lib', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
    done
  done
done
