# The slab-step tests and the per-slab cost (serialised local group + kernel trace)
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slabtrace; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_slab.py tests/test_gpu_resort.py -m gpu -q -p no:cacheprovider --timeout=300 --timeout-method thread > gpurun_out/pytest_slab.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_slab.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > gpurun_out/slab_overhead.log 2>&1; rc=$?
echo "slab_overhead rc=$rc"; tail -4 gpurun_out/slab_overhead.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/k4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" 4 30 > gpurun_out/slabtrace/k4.log 2>&1; rc=$?
echo "trace rc=$rc"
exit 0
