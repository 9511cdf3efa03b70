# register-pressure changes: full -m gpu suite, then the faithful lines they affect (and C3 / C3 BLS as
# controls) and the per-problem round breakdown of the faithful C4 / C5 / C7 runs
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/rg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rg_tests.log
if [ $rc -ne 0 ]; then echo "tests rc $rc: stopping"; exit $rc; fi
mkdir -p gpurun_out/rg
for a in "c3" "c3 --faithful" "c3bls --faithful" "c4 --faithful" "c5 --faithful" "c7 --faithful" "c5" "c7"; do
  tag=$(echo $a | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $a > gpurun_out/rg/bench_$tag.json 2> gpurun_out/rg/bench_$tag.err || { echo "bench $a rc $?"; tail -3 gpurun_out/rg/bench_$tag.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/rg/bench_$tag.json').read().strip().splitlines()[-1]);print('$a', '%.4g'%d['value'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
done
for c in c4 c5 c7; do timeout -k 10 120 python tools/faithful_rounds.py $c > gpurun_out/rg/rounds_$c.txt 2>&1 || exit 2; cat gpurun_out/rg/rounds_$c.txt; done
