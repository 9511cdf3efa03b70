# Re-issue a gpurun call while the pool reports a transient (infrastructure) status: nothing ran then.
# usage: bash tools/gpu/retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  if grep -q "status=transient" "$out"; then sleep 120; else break; fi
done
