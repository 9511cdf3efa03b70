cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/perm_diag.py c3bls 64 && KEXPR="bls or BLS or helpers or neighbour or tiny" bash tools/gpu/suite_nox.sh
