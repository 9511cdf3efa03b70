# k_lean2 (IRM_LEAN2=1) vs k_lean: correctness against the oracle / general kernel and C3 timing
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
b() { timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/l2.json 2>gpurun_out/l2.err || { echo "bench rc $?"; tail -5 gpurun_out/l2.err; exit 2; }
      python -c "import json;d=json.loads(open('gpurun_out/l2.json').read().strip().splitlines()[-1]);print('   ', d['value'], d['roofline']['kernel_ms'], d['roofline']['kernel'][:50])"; }
echo "k_lean"; b
echo "k_lean2"; IRM_LEAN2=1 b
IRM_LEAN2=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "bench_c3_full or smooth_objective_tracks_oracle and c3 or tracks_general and c3 or neighbours and c3 or lean_gd_kernel_matches_oracle" -s > gpurun_out/l2_tests.log 2>&1; echo "tests rc $?"; grep -E "passed|failed|lean -|traj - oracle" gpurun_out/l2_tests.log | head -30
