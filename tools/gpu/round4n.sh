# final library: two more default bench lines (box spread of the headline) and the multi-rank path
# rehearsed on the one GPU (2 ranks, gloo collectives on host tensors)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu-baseline > gpurun_out/r04_c3_rep$i.json 2> gpurun_out/r04_c3_rep$i.err || { echo "bench rep $i failed"; tail -3 gpurun_out/r04_c3_rep$i.err; exit 2; }
  python -c "import json;d=json.loads(open('gpurun_out/r04_c3_rep$i.json').read().strip().splitlines()[-1]);print('c3 rep $i', '%.4g'%d['value'], '%.4f ms'%d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline > gpurun_out/r04_gloo2.json 2> gpurun_out/r04_gloo2.err; echo "gloo2 rc $?"; tail -1 gpurun_out/r04_gloo2.json | cut -c1-400
