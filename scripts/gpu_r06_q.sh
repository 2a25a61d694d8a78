# r6 q: Model S at the reference's scale (C1): k_force_small loads a candidate's velocity and pass-1 terms with its
# position (one round trip per round), k_density_fused loads the target's old key unconditionally and a row's two
# table reads together. Small-N / parity / fused tests, then the small-N rates against base (HEAD before r6 n).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06q; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_physics.py tests/test_gpu_path_independence.py -m gpu -x -q -p no:cacheprovider --timeout=300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in base new; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_${v}_$r.log 2>&1; rc=$?
  echo "== $v $r rc=$rc"; grep -E "sphere N=4096 team default|sphere N=32768 team default|C1" $O/small_n_${v}_$r.log | cut -c 1-110; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
