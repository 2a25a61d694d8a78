set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_check_steps.py > gpurun_out/diag_check_steps.log 2>&1; echo "diag rc=$?"; cat gpurun_out/diag_check_steps.log | tail -14
timeout -k 10 300 python -u -m pytest -q -p no:cacheprovider --timeout=200 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_parity_headline.py tests/test_gpu_profile.py tests/test_gpu_resort.py > gpurun_out/pytest_c.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/pytest_c.log | tail -8
for r in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 200 > gpurun_out/bench_c.log 2>&1; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_c.log').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], d['kernels_ms_per_step'], 'mid', d.get('ms_per_step_mid_collapse'))"; done
