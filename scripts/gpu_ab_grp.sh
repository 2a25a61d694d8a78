# Oversized planes staged as groups of fitting rows: resort/slab/multi tests on the variant, then an interleaved
# A/B, then the mid-collapse kernel trace of the variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPHHIP_LIB=build/variants/lib_grp.so timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_parity.py tests/test_gpu_resort.py tests/test_gpu_slab.py tests/test_gpu_multi.py tests/test_gpu_physics.py > gpurun_out/pytest_grp.log 2>&1 || { echo "grp tests failed"; tail -30 gpurun_out/pytest_grp.log; exit 1; }
echo "grp: $(tail -1 gpurun_out/pytest_grp.log)"
bash scripts/variant_ab.sh "head grp" 3 || exit 1
export TMPDIR=/tmp
SPHHIP_LIB=build/variants/lib_grp.so timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/profmid4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 200 --no-cpu-baseline --no-profile > gpurun_out/profmid4.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/profmid4.log; exit 1; }
python3 scripts/trace_kstats.py gpurun_out/profmid4/run_kernel_trace.csv 1000
