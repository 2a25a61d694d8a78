set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4 100 > gpurun_out/slab_overhead.log 2>&1; echo "rc=$?"; tail -4 gpurun_out/slab_overhead.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_slab" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_overhead.py" 2 40 > gpurun_out/prof_slab.log 2>&1; echo "prof rc=$?"
