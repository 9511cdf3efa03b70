cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
KEXPR="bls or BLS or helpers or neighbour or tiny" bash tools/gpu/suite_nox.sh || exit $?
timeout -k 10 300 python tools/help_rounds.py c3bls 1024 || exit $?
timeout -k 10 300 python tools/help_ab.py c3bls 1024 || exit $?
timeout -k 10 120 python tools/help_ab.py c2 1 || exit $?
for c in "c3bls" "c3bls --faithful" "c2 --faithful"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/h.json 2> gpurun_out/h.err || { echo "bench failed"; tail -3 gpurun_out/h.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/h.json').read().strip().splitlines()[-1]);print('$c', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
done
