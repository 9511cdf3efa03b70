#!/bin/bash
# One parameterised runner for the GPU-box sessions (replaces the per-session round*/ab*/… scripts).
# Every GPU step runs under its own time limit and the script stops at the first failure.
#
#   bash tools/gpu/run.sh suite                         full -m gpu suite + smoke()
#   bash tools/gpu/run.sh tests "<pytest -k expr>"      a subset of the -m gpu suite
#   R=r05 bash tools/gpu/run.sh lines "c3|c3bls --faithful"   bench lines (CPU baselines included) → gpurun_out/$R_bench_<cfg>.json
#   R=r05 bash tools/gpu/run.sh lines all               every config of the round table
#   bash tools/gpu/run.sh fast "c3|c2 --faithful"       bench lines without CPU baselines (quick timing)
#   V=base bash tools/gpu/run.sh ab "c3|c3 --faithful"  same-box interleaved timing: release vs libirm_hip_$V.so (REPS=3)
#   V=base bash tools/gpu/run.sh abcheck "c3"           tools/sched_check.py bit-identity of the two libraries, then ab
#   bash tools/gpu/run.sh sq "release base" c3          per-round SQ instruction counts of libraries (one --pmc pass each)
#   bash tools/gpu/run.sh phase "c3 c3bls"              phase profile (needs the --prof build, libirm_hip_prof.so)
#   bash tools/gpu/run.sh rounds "c3bls c5"             per-problem round breakdown of faithful runs
cd "$GRAFT_REPO_ROOT" || exit 2
export PYTHONUNBUFFERED=1
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
ALL="c3|c3 --faithful|c3bls|c3bls --faithful|c2 --faithful|c4|c4 --faithful|c5|c5 --faithful|c5 --operator-rank -1|c7|c7 --faithful"
lib_of() { if [ "$1" = release ]; then echo "$ROOT/irm_motion_planning_amd/libirm_hip.so"; else echo "$ROOT/irm_motion_planning_amd/libirm_hip_$1.so"; fi; }
tag_of() { echo "$1" | tr ' ' '_' | tr -d '-'; }
show() {  # one summary line of a bench JSON file
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], '%.4g'%d['value'], d['unit'], '%.4f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])" "$1" "$2"
}
bench_one() {  # bench_one <lib> <outfile> <cpu: yes|no> <config args...>
  local lib=$1 out=$2 cpu=$3; shift 3
  local extra=""; [ "$cpu" = no ] && extra="--no-cpu-baseline"
  IRM_LIB=$(lib_of "$lib") timeout -k 10 300 python bench.py $extra --config "$@" > "$out" 2> "$out.err" || {
    echo "bench $* ($lib) failed"; tail -3 "$out.err"; exit 2; }
}
cmd=${1:?subcommand}
shift
case "$cmd" in
  suite)
    timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/suite.log" 2>&1
    rc=$?; tail -4 "$OUT/suite.log"
    [ $rc -ne 0 ] && { echo "tests rc $rc"; exit $rc; }
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
    rc=$?; tail -2 "$OUT/smoke.log"; exit $rc ;;
  tests)
    timeout -k 10 ${TMO:-900} python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/ -k "${1:?-k expression}" > "$OUT/tests.log" 2>&1
    rc=$?; grep -vE "^\s*$|amdgpu.ids" "$OUT/tests.log" | tail -60; exit $rc ;;
  lines|fast)
    R=${R:-rXX}
    sel=${1:-all}; [ "$sel" = all ] && sel=$ALL
    IFS='|' read -ra CFGS <<< "$sel"
    for c in "${CFGS[@]}"; do
      t=$(tag_of "$c")
      if [ "$cmd" = lines ]; then f="$OUT/${R}_bench_$t.json"; bench_one release "$f" yes $c
      else f="$OUT/fast_$t.json"; bench_one release "$f" no $c; fi
      show "$f" "$c"
    done ;;
  ab)
    V=${V:?V=variant}
    IFS='|' read -ra CFGS <<< "${1:-c3}"
    for rep in $(seq ${REPS:-3}); do
      for c in "${CFGS[@]}"; do
        t=$(tag_of "$c")
        for lib in release $V; do
          f="$OUT/ab_${t}_$lib.json"; bench_one $lib "$f" no $c; show "$f" "$rep $t $lib"
        done
      done
    done ;;
  abcheck)
    V=${V:?V=variant}
    IRM_LIB=$(lib_of $V) timeout -k 10 240 python tools/sched_check.py run "$OUT/chk_$V.npz" > "$OUT/chk_$V.log" 2>&1 || { echo "check $V failed"; tail -5 "$OUT/chk_$V.log"; exit 2; }
    timeout -k 10 240 python tools/sched_check.py run "$OUT/chk_release.npz" > "$OUT/chk_release.log" 2>&1 || { echo "check release failed"; tail -5 "$OUT/chk_release.log"; exit 2; }
    python tools/sched_check.py cmp "$OUT/chk_$V.npz" "$OUT/chk_release.npz" || exit 2
    exec_args=("$@"); V=$V bash "$0" ab "${exec_args[@]}" ;;
  sq)
    cd /tmp && export TMPDIR=/tmp
    for v in ${1:-release}; do
      d="$OUT/sq_${v}_$(tag_of "${2:-c3}")"
      IRM_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
        --output-format csv -d "$d/p1" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --config ${2:-c3} > "$d.log" 2>&1 || { echo "pmc $v failed"; tail -3 "$d.log"; exit 3; }
      echo "== $v ${2:-c3}"; python3 "$ROOT/tools/summarize_pmc_round.py" "$d" | sed 's/^/   /'
    done ;;
  phase)
    IRM_LIB=$ROOT/irm_motion_planning_amd/libirm_hip_prof.so IRM_PROFILE_LEAN=1 timeout -k 10 240 python tools/phase_profile.py ${1:-c3 c3bls} > "$OUT/phase.log" 2>&1
    rc=$?; grep -v amdgpu.ids "$OUT/phase.log"; exit $rc ;;
  rounds)
    for c in ${1:-c3bls}; do
      timeout -k 10 180 python tools/faithful_rounds.py $c > "$OUT/rounds_$c.txt" 2>&1 || { echo "rounds $c failed"; tail -3 "$OUT/rounds_$c.txt"; exit 2; }
      cat "$OUT/rounds_$c.txt"
    done ;;
  *) echo "unknown subcommand $cmd"; exit 2 ;;
esac
