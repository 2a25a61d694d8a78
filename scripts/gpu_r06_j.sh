# r6 j: Model R one-launch step: the finish's angular damping from the host (ContactConst::ang_damp). Bit-exactness
# tests of every Model R path, the phase clocks with the finish split, and the small-N rates.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06j; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_small.py tests/test_gpu_contact_team.py -m gpu -x -q -p no:cacheprovider --timeout=200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 > $O/contact_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -1 $O/contact_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; rc=$?; tail -5 $O/small_n.log
exit $rc
