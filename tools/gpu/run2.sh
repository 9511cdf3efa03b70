# GPU session script: selected parity tests, then bench lines (stops on a crash / timeout)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "${IRM_TESTS:-launch_plan or batched}" -s > gpurun_out/run2_tests.log 2>&1
rc=$?
tail -4 gpurun_out/run2_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
for a in ${IRM_BENCH:-"c3" "c3:--tb:2" "c7" "c3bls:--faithful"}; do
  a=${a//:/ }
  echo "== $a"
  timeout -k 10 120 python bench.py --config $a --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/exp1.json 2>gpurun_out/exp1.err || { echo "bench rc $?"; tail -5 gpurun_out/exp1.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/exp1.json').read().strip().splitlines()[-1]);print(d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['config']['traj_per_block'],d['roofline']['kernel'])"
done
