# faithful / bench lines of the current build (A/B against an earlier run)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for a in ${CONFIGS:-"c3" "c3 --faithful" "c3bls --faithful" "c4 --faithful" "c5 --faithful" "c7 --faithful"}; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $a > gpurun_out/ab/bench_$tag.json 2> gpurun_out/ab/bench_$tag.err || { echo "bench $a rc $?"; tail -3 gpurun_out/ab/bench_$tag.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/ab/bench_$tag.json').read().strip().splitlines()[-1]);print('$a', '%.4g'%d['value'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
