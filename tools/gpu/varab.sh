#!/bin/bash
# Same-box A/B of build variants: per-round instruction counts (one rocprofv3 --pmc pass per variant)
# and interleaved bench timing.  LIBS: variant names (release = libirm_hip.so, X = libirm_hip_X.so).
#   LIBS="release noslp" CONFIGS="c3|c3 --faithful" REPS=3 bash tools/gpu/varab.sh
cd $GRAFT_REPO_ROOT
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/varab
mkdir -p $OUT
IFS='|' read -ra CFGS <<< "${CONFIGS:-c3}"
lib_of() { if [ $1 = release ]; then echo $ROOT/irm_motion_planning_amd/libirm_hip.so; else echo $ROOT/irm_motion_planning_amd/libirm_hip_$1.so; fi; }
if [ -z "$NOPMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  for v in ${LIBS:-release}; do
    IRM_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
      --output-format csv -d $OUT/pmc_$v -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 3 --warmup 1 --config ${PMCCFG:-c3} > $OUT/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -3 $OUT/pmc_$v.log; exit 3; }
    echo "== $v"; python3 $ROOT/tools/summarize_sq.py $OUT/pmc_$v | sed 's/^/   /'
  done
  cd $ROOT
fi
for rep in $(seq ${REPS:-3}); do
  for c in "${CFGS[@]}"; do
    tag=$(echo $c | tr ' ' '_' | tr -d '-')
    for v in ${LIBS:-release}; do
      IRM_LIB=$(lib_of $v) timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > $OUT/b_${tag}_$v.json 2> $OUT/b.err || { echo "bench $c $v failed"; tail -3 $OUT/b.err; exit 2; }
      python -c "import json;d=json.loads(open('$OUT/b_${tag}_$v.json').read().strip().splitlines()[-1]);print('$rep $tag $v', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
    done
  done
done
