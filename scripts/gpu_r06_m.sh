# r6 m: as r6 l, with the counts and range keys read through the vector path (ld_vec, vzero), so the first loads of
# k_mv_rank, both cell-share forms and the one-launch builds issue in one round trip; plus the probe.
# and of the re-sort, then the small-N rates (base = HEAD before the change, new; new with SPH_FUSED_MC=0) and an
# interleaved C3 A/B (base, new).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06m; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_small.py tests/test_gpu_contact_team.py tests/test_gpu_resort.py tests/test_gpu_path_independence.py tests/test_gpu_slab.py -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 > $O/contact_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -1 $O/contact_probe.log; [ $rc -ne 0 ] && exit $rc
for v in base new; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep sphere $O/small_n_$v.log; [ $rc -ne 0 ] && exit $rc
done
SPH_FUSED_MC=0 SPHHIP_LIB=build/variants/lib_new.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_new_mc0.log 2>&1; rc=$?
echo "== new mc0 rc=$rc"; grep sphere $O/small_n_new_mc0.log; [ $rc -ne 0 ] && exit $rc
for v in base new; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_${v}_2.log 2>&1; rc=$?
  echo "== $v (2) rc=$rc"; grep sphere $O/small_n_${v}_2.log; [ $rc -ne 0 ] && exit $rc
done
bash scripts/variant_ab.sh "base new" 3 > $O/ab.log 2>&1; rc=$?
cat $O/ab.log
exit $rc
