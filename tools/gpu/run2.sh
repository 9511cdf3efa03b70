set -e
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "launch_plan or rank_cuts or batched" -s > gpurun_out/run2_tests.log 2>&1 || { echo TESTS FAILED; tail -50 gpurun_out/run2_tests.log; exit 1; }
tail -5 gpurun_out/run2_tests.log
for a in "--config c3" "--config c3 --tb 2" "--config c7" "--config c3bls --faithful"; do
  echo "== $a"
  timeout -k 10 120 python bench.py $a --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/exp1.json 2>gpurun_out/exp1.err
  python -c "import json;d=json.loads(open('gpurun_out/exp1.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['config']['traj_per_block'],d['roofline']['kernel'])"
done
