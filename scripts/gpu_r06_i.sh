# r6 i: the headline parity tests with the support-edge conditioning term (oracle.h or_sph_step_diag) and the
# decomposed C4/C5 oracle steps, printing every state's margins (err over S and over the whole bound).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06i; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity_headline.py "tests/test_gpu_multi.py::test_baseline_config_decomposed_full_size" -m gpu -v -s -p no:cacheprovider --timeout=600 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "acc_err_over|passed|failed|FAILED|Error" $O/pytest.log | cut -c 1-300 | tail -20
exit $rc
