set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/variant_ab.sh "head swz x0" 3 parity; echo "ab rc=$?"
bash scripts/gpu_pmc_libs.sh build/variants/lib_head.so build/variants/lib_swz.so build/variants/lib_x0.so 2>&1 | tail -8
