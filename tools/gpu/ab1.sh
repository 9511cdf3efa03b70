# bench lines of the release library for the '|'-separated CONFIGS
cd $GRAFT_REPO_ROOT
IFS='|' read -ra CFGS <<< "${CONFIGS:-c3}"
for c in "${CFGS[@]}"; do
  tag=$(echo $c | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab1_${tag}.json 2> gpurun_out/ab1.err || { echo "bench $c failed"; tail -3 gpurun_out/ab1.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/ab1_${tag}.json').read().strip().splitlines()[-1]);print('$tag', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
done
