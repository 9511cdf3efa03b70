cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu/suite_nox.sh || exit $?
echo "== dyn sched check"
IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_dynilp.so timeout -k 10 200 python tools/dyn_sched_check.py run gpurun_out/dyn_ilp.npz > gpurun_out/dyn_ilp.log 2>&1 || { echo "dynilp run failed"; tail -3 gpurun_out/dyn_ilp.log; }
timeout -k 10 200 python tools/dyn_sched_check.py run gpurun_out/dyn_def.npz > gpurun_out/dyn_def.log 2>&1 || { echo "def run failed"; tail -3 gpurun_out/dyn_def.log; exit 2; }
python tools/dyn_sched_check.py cmp gpurun_out/dyn_def.npz gpurun_out/dyn_ilp.npz
LIBS="base release" CONFIGS="c3|c3bls|c2 --faithful|c3bls --faithful|c7 --faithful|c5 --faithful" REPS=1 bash tools/gpu/varab.sh
