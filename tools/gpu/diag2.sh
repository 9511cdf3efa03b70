cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/ens_check.py pp:4 || exit 2
echo "== drift c5d 12"; LADDER=1,5,10,20,30,40,50,60,70,80,90,100 timeout -k 10 400 python tools/drift_diag.py c5d 12 16 || exit 2
for v in base release; do
  if [ $v = release ]; then L=libirm_hip.so; else L=libirm_hip_$v.so; fi
  echo "== rounds $v"; IRM_LIB=$GRAFT_REPO_ROOT/irm_motion_planning_amd/$L timeout -k 10 200 python tools/faithful_rounds.py c3bls || exit 2
done
NOPMC=1 LIBS="base r2 release" CONFIGS="c3|c3bls|c2 --faithful|c7" REPS=2 bash tools/gpu/varab.sh
