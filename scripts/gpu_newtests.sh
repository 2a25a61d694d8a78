set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_headline.py tests/test_gpu_physics.py -m gpu -v -s -p no:cacheprovider --timeout=300 --timeout-method thread > gpurun_out/newtests.log 2>&1; rc=$?
echo "new tests rc=$rc"; grep -E "PASS|FAIL|Error|label|slope|ratio" gpurun_out/newtests.log | tail -30
[ $rc -eq 124 -o $rc -eq 137 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 --timeout-method thread --deselect tests/test_gpu_parity_headline.py --deselect tests/test_gpu_physics.py > gpurun_out/pytest_gpu.log 2>&1; rc2=$?
echo "rest rc=$rc2"; tail -5 gpurun_out/pytest_gpu.log
exit $rc
