# Hit lists removed from pass 2 (mask walk for every masked plane, distance loop otherwise): full GPU
# suite on the product build, then an interleaved A/B against the previous head and two LDS/occupancy variants.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/variant_ab.sh "direct nl nl1270 nlw5" 3
