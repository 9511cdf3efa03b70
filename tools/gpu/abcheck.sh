# Bit-identity (tools/sched_check.py cases) and same-box timing of the release library against
# libirm_hip_$VARIANT.so (e.g. the previous commit's build kept as libirm_hip_base.so)
#   VARIANT=base CONFIGS="c3|c3 --faithful" bash tools/gpu/abcheck.sh
cd $GRAFT_REPO_ROOT
V=${VARIANT:-base}
mkdir -p gpurun_out
IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_$V.so timeout -k 10 240 python tools/sched_check.py run gpurun_out/chk_$V.npz > gpurun_out/chk_$V.log 2>&1 || { echo "check $V failed"; tail -5 gpurun_out/chk_$V.log; exit 2; }
timeout -k 10 240 python tools/sched_check.py run gpurun_out/chk_release.npz > gpurun_out/chk_release.log 2>&1 || { echo "check release failed"; tail -5 gpurun_out/chk_release.log; exit 2; }
python tools/sched_check.py cmp gpurun_out/chk_$V.npz gpurun_out/chk_release.npz
VARIANT=$V bash tools/gpu/ab2.sh
