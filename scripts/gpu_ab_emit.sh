# Pass-1 hit-mask emit with the word computed every group and only the store conditional (A/B), parity.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in esel; do SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_resort.py > gpurun_out/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/pytest_$v.log; exit 1; }; echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"; done
bash scripts/variant_ab.sh "head esel" 4
