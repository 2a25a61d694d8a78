# Pass-1 occupancy: 4, 5 and 8 workgroups per CU (smaller plane budgets) against the head build: parity of 8 waves,
# then an interleaved A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_d4.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/pytest_dq.log 2>&1 || { echo "dq tests failed"; tail -30 gpurun_out/pytest_dq.log; exit 1; }
echo "d4: $(tail -1 gpurun_out/pytest_dq.log)"
bash scripts/variant_ab.sh "head d4 d5 d8" 3
