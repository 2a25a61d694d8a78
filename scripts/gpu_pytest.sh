# usage: bash scripts/gpu_pytest.sh <pytest args...>   (one pytest process, per-test timeout, log in gpurun_out/)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -p no:cacheprovider --timeout=300 --timeout-method thread "$@" > gpurun_out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|label|slope|ratio|passed|failed" gpurun_out/pytest.log | tail -40
exit $rc
