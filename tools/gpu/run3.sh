cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1

timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "ensemble or tracks_general or rank_cuts or launch_plan or batched" -s > gpurun_out/run3_tests.log 2>&1
rc=$?; tail -4 gpurun_out/run3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err; echo "bench rc $?"; tail -c 3000 gpurun_out/bench_c3.json
