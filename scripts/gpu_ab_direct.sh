# Direct-from-mask plane loop in pass 2: parity through the C ABI, lane utilisation, interleaved A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_dfx.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py tests/test_gpu_resort.py tests/test_gpu_physics.py > gpurun_out/pytest_direct.log 2>&1 || { echo "direct tests failed"; tail -30 gpurun_out/pytest_direct.log; exit 1; }
tail -2 gpurun_out/pytest_direct.log
for v in ddiag dfxdiag; do SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 300 python -u scripts/pass_util.py > gpurun_out/pass_util_$v.log 2>&1 || { echo "diag failed"; tail -5 gpurun_out/pass_util_$v.log; exit 1; }; grep state gpurun_out/pass_util_$v.log; done

bash scripts/variant_ab.sh "base direct dfx" 3
