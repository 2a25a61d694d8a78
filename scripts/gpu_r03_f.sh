set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -p no:cacheprovider --timeout=300 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_slab.py > gpurun_out/pytest_f.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/pytest_f.log | tail -8
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4 100 > gpurun_out/slab_overhead_f.log 2>&1; echo "rc=$?"; tail -2 gpurun_out/slab_overhead_f.log
