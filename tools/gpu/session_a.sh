# full -m gpu suite (stops on a crash) and the bench lines of every config
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/sa_tests.log 2>&1
rc=$?; tail -5 gpurun_out/sa_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
mkdir -p gpurun_out/r03
for a in "c3" "c3 --faithful" "c3bls" "c3bls --faithful" "c4" "c4 --faithful" "c5" "c5 --operator-rank -1" "c5 --faithful" "c7" "c7 --faithful" "c2 --faithful"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --config $a > gpurun_out/r03/bench_$tag.json 2> gpurun_out/r03/bench_$tag.err || { echo "bench $a rc $?"; tail -3 gpurun_out/r03/bench_$tag.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/r03/bench_$tag.json').read().strip().splitlines()[-1]);print('$a', '%.4g'%d['value'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], 'cpu %.3g'%(d['cpu_baseline'] or {}).get('value',0))"
done
