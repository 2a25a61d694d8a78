# Parity of the packed-math variant through the C ABI, then an interleaved A/B against the head build.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_pk2.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py tests/test_gpu_resort.py tests/test_gpu_physics.py > gpurun_out/pytest_pk2.log 2>&1 || { echo "pk2 tests failed"; tail -30 gpurun_out/pytest_pk2.log; exit 1; }
tail -2 gpurun_out/pytest_pk2.log
bash scripts/variant_ab.sh "base pk pk2" 3
