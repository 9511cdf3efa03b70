# diagnostic: two 256-thread C3 workgroups per CU (--tb 2) with their loop starts staggered (IRM_STAGGER)
cd $GRAFT_REPO_ROOT
b() { timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 2 "$@" > gpurun_out/st.json 2>gpurun_out/st.err || { echo "bench rc $?"; tail -3 gpurun_out/st.err; exit 2; }
      python -c "import json;d=json.loads(open('gpurun_out/st.json').read().strip().splitlines()[-1]);print('   ', d['value'], d['roofline']['kernel_ms'])"; }
echo "c3 default"; b
echo "c3 tb2"; b --tb 2
for s in 1 2; do for c in 2000 4000 8000; do echo "c3 tb2 stagger $s cyc $c"; IRM_STAGGER=$s IRM_STAGGER_CYC=$c b --tb 2; done; done
echo "c3 tb4 stagger 1 (no co-resident partner: control)"; IRM_STAGGER=1 b
