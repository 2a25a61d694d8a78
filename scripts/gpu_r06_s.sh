# r6 s: the flat contact form's int torque sums by DPP scans and its float totals by readlane; row selection of a
# candidate by a compare chain over wave-uniform values (one-launch kernel, small-N Model S); the one-launch
# permutation table from a scan of the movers per stayer rank instead of a binary search per run. Tests, probe, rates.

set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06s; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_contact_team.py tests/test_gpu_path_independence.py -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 > $O/contact_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -1 $O/contact_probe.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in base new; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_${v}_$r.log 2>&1; rc=$?
  echo "== $v $r rc=$rc"; grep -E "sphere N=4096 team default|sphere N=32768 team default|C1" $O/small_n_${v}_$r.log | cut -c 1-110; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
