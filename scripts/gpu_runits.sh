# r-unit neighbour passes (SPH_RUNITS=1, the product build) against the q forms: GPU suite, interleaved A/B, slab trace
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slabtrace; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/variant_ab.sh "head qform" 3
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/k4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" 4 30 > gpurun_out/slabtrace/k4.log 2>&1; echo "trace rc=$?"
exit 0
