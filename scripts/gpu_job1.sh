set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -p no:cacheprovider --timeout=200 --timeout-method thread tests/test_gpu_readback.py -m gpu -q > gpurun_out/readback.log 2>&1; rc=$?
echo "readback rc=$rc"; tail -3 gpurun_out/readback.log
[ $rc -eq 124 -o $rc -eq 137 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_clock.sh
