cd $GRAFT_REPO_ROOT
bash tools/gpu/run.sh tests "bls or BLS or helpers" > gpurun_out/t1.txt 2>&1; rc=$?; tail -5 gpurun_out/t1.txt; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -20; exit $rc; }
V=base REPS=2 bash tools/gpu/run.sh ab "c3bls|c3bls --faithful|c2 --faithful" || exit 2
export IRM_PROFILE_LEAN=1
IRM_LIB=$PWD/irm_motion_planning_amd/libirm_hip_baseprof.so timeout -k 10 200 python tools/phase_profile.py c3bls > gpurun_out/ph_base.log 2>&1 || exit 2
IRM_LIB=$PWD/irm_motion_planning_amd/libirm_hip_prof.so timeout -k 10 200 python tools/phase_profile.py c3bls > gpurun_out/ph_new.log 2>&1 || exit 2
grep -v amdgpu gpurun_out/ph_base.log; grep -v amdgpu gpurun_out/ph_new.log
timeout -k 10 300 python tools/bls_drift.py 16 gpurun_out/bls_drift.txt > /dev/null 2>gpurun_out/bls_drift.err || { tail -5 gpurun_out/bls_drift.err; exit 2; }
tail -3 gpurun_out/bls_drift.txt
