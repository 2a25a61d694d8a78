# r6 k: the one-launch Model R step with the movers' new cell ranges handed to the next step (FusedIO.mc): every Model R
# bit-exactness test, the phase clocks, and the small-N rates.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06k; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_contact_team.py -m gpu -x -v -p no:cacheprovider --timeout=200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 > $O/contact_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -1 $O/contact_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; rc=$?; tail -5 $O/small_n.log
exit $rc
