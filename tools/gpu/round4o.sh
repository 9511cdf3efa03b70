# scheduler-option variants of every unit (metric bias 0; no unclustered high-RP reschedule) against the
# release library: bit-identity on sched_check's cases, then interleaved timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/sched_check.py run gpurun_out/chk_release.npz > gpurun_out/chk_release.log 2>&1 || { echo "check release failed"; exit 2; }
for V in mb0 nourp; do
  IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/libirm_hip_$V.so timeout -k 10 240 python tools/sched_check.py run gpurun_out/chk_$V.npz > gpurun_out/chk_$V.log 2>&1 || { echo "check $V failed"; tail -3 gpurun_out/chk_$V.log; exit 2; }
  echo "== $V"; python tools/sched_check.py cmp gpurun_out/chk_release.npz gpurun_out/chk_$V.npz | grep -v bit-equal
done
for rep in 1 2 3; do
  for c in "c3" "c3 --faithful" "c7"; do
    tag=$(echo $c | tr ' ' '_' | tr -d '-')
    for lib in release mb0 nourp; do
      if [ $lib = release ]; then L=irm_motion_planning_amd/libirm_hip.so; else L=irm_motion_planning_amd/libirm_hip_$lib.so; fi
      IRM_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab3_${tag}_$lib.json 2> gpurun_out/ab3.err || { echo "bench $c $lib failed"; tail -3 gpurun_out/ab3.err; exit 2; }
      python -c "import json;d=json.loads(open('gpurun_out/ab3_${tag}_$lib.json').read().strip().splitlines()[-1]);print('$rep $tag $lib', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
    done
  done
done
