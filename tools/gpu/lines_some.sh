# Bench lines (with CPU baselines) of the given configs into gpurun_out/<tag>_bench_<config>.json
#   R=r03 CONFIGS="c5|c7 --faithful" bash tools/gpu/lines_some.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
IFS='|' read -ra CFGS <<< "${CONFIGS:?}"
for a in "${CFGS[@]}"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $a > gpurun_out/${R}_bench_$tag.json 2> gpurun_out/${R}_bench_$tag.err || { echo "bench $a rc $?"; tail -3 gpurun_out/${R}_bench_$tag.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/${R}_bench_$tag.json').read().strip().splitlines()[-1]);print('$a', '%.4g'%d['value'], d['unit'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
