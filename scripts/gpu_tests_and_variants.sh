set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/nb_variants.py --config C3 --variants 0,1 --steps 50 --rounds 2 > gpurun_out/variants.log 2>&1; rc2=$?
echo "variants rc=$rc2"; grep -v amdgpu.ids gpurun_out/variants.log
exit $rc
