set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python scripts/nb_variants.py --config C3 --variants 0,1 --steps 50 --rounds 3 > gpurun_out/variants.log 2>&1; rc=$?
echo "variants rc=$rc"; cat gpurun_out/variants.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
exit $rc
