# LDS padding of pass 2's staged plane (one 16-B pad every 16 / 32 slots) against the head build and a
# head build at the padded variant's plane budget: parity of one padded build, then an interleaved A/B.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_pad4.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py > gpurun_out/pytest_pad.log 2>&1 || { echo "pad tests failed"; tail -30 gpurun_out/pytest_pad.log; exit 1; }
echo "pad4: $(tail -1 gpurun_out/pytest_pad.log)"
bash scripts/variant_ab.sh "head pad4 pad5 g1195" 3
