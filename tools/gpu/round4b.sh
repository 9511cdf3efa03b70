cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
KEXPR="bls or BLS or helpers or neighbour or tiny" bash tools/gpu/suite_nox.sh || exit $?
echo "== D=5 iterative-ILP build: the generic-shape iteration test"
IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_dynilp.so timeout -k 10 300 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_generic_shapes_match_reference_iteration" > gpurun_out/ilp5.log 2>&1; tail -3 gpurun_out/ilp5.log
echo "== helpers on / off"
for h in 0 1; do
  for c in "c3bls --faithful" "c2 --faithful" "c3bls"; do
    IRM_LEAN_NOHELP=$h timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/h.json 2> gpurun_out/h.err || { echo "bench failed"; tail -3 gpurun_out/h.err; exit 2; }
    python -c "import json;d=json.loads(open('gpurun_out/h.json').read().strip().splitlines()[-1]);print('nohelp=$h', '$c', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
  done
done
echo "== contract-on builds (round 3 flags), default vs iterative-ILP scheduler on the DynShape units"
L=$GRAFT_REPO_ROOT/irm_motion_planning_amd
IRM_LIB=$L/libirm_hip_cdef.so timeout -k 10 200 python tools/dyn_sched_check.py run gpurun_out/dyn_cdef.npz > gpurun_out/dyn_cdef.log 2>&1 || { echo "cdef failed"; tail -3 gpurun_out/dyn_cdef.log; exit 2; }
IRM_LIB=$L/libirm_hip_cilp.so timeout -k 10 200 python tools/dyn_sched_check.py run gpurun_out/dyn_cilp.npz > gpurun_out/dyn_cilp.log 2>&1 || { echo "cilp failed"; tail -3 gpurun_out/dyn_cilp.log; exit 2; }
python tools/dyn_sched_check.py cmp gpurun_out/dyn_cdef.npz gpurun_out/dyn_cilp.npz
