# Bench lines of every config for the round's profiles (GPU box); CPU baselines included.
#   bash tools/gpu/round_lines.sh r03
R=${1:?round tag}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for a in "c3 --faithful" "c3bls" "c3bls --faithful" "c2 --faithful" "c4" "c4 --faithful" "c5" "c5 --faithful" "c5 --operator-rank -1" "c7" "c7 --faithful"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $a > gpurun_out/${R}_bench_$tag.json 2> gpurun_out/${R}_bench_$tag.err || { echo "bench $a rc $?"; tail -3 gpurun_out/${R}_bench_$tag.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/${R}_bench_$tag.json').read().strip().splitlines()[-1]);print('$a', '%.4g'%d['value'], d['unit'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
