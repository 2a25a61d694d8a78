# Pass-2 lane order by fx halves, and the self pair dropped from the mask walk: parity, lane use, A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in fx2 noself; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py tests/test_gpu_resort.py tests/test_gpu_slab.py > gpurun_out/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
done
SPHHIP_LIB=build/variants/lib_fx2diag.so timeout -k 10 300 python -u scripts/pass_util.py > gpurun_out/pass_util_fx2.log 2>&1 || { echo "diag failed"; tail -5 gpurun_out/pass_util_fx2.log; exit 1; }
grep state gpurun_out/pass_util_fx2.log
bash scripts/variant_ab.sh "head fx2 noself" 3
