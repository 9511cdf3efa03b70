cd $GRAFT_REPO_ROOT
for c in c3 c3o0 c3o44 c3n64; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/oc.json 2>gpurun_out/oc.err || { echo "bench rc $?"; tail -3 gpurun_out/oc.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/oc.json').read().strip().splitlines()[-1]);print('$c', d['value'], d['roofline']['kernel_ms'], d['roofline']['kernel'][:60])"
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_reference.py -k "dense_operator or first_steps or 200_steps" -s > gpurun_out/run4_tests.log 2>&1; echo "tests rc $?"; grep -E "passed|failed|widest|knife|dense -" gpurun_out/run4_tests.log
