# Pass-1 lane order: quadrants (head), plain sorted order, halves by fx, halves by fy: parity of the plain
# order, then an interleaved A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_dq0.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py > gpurun_out/pytest_dq.log 2>&1 || { echo "dq tests failed"; tail -30 gpurun_out/pytest_dq.log; exit 1; }
echo "dq0: $(tail -1 gpurun_out/pytest_dq.log)"
bash scripts/variant_ab.sh "head dq0 dq2 dqy2" 3
