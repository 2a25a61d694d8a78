# First call of a round: GPU tests, smoke, the default bench line and the slab step's per-GPU cost.
# (Counters, clocks and the profiled bench are scripts/gpu_round.sh.)
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -12
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c 1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 > gpurun_out/slab_overhead.log 2>&1; rc=$?
echo "slab_overhead rc=$rc"; tail -4 gpurun_out/slab_overhead.log
exit 0
