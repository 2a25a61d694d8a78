# Interleaved A/B of library variants build/variants/lib_<v>.so (scripts/build_variant.sh):
#   bash scripts/variant_ab.sh "head v1 v2" [rounds] [parity]
# parity (optional, "parity"): first run the headline parity and re-sort tests on every variant.
# Each round runs bench.py (200 steps from rest + 200 mid-collapse) once per variant, in turn.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "${3:-}" = "parity" ]; then
  for v in $1; do
    SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py tests/test_gpu_resort.py > gpurun_out/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/pytest_$v.log; exit 1; }
    echo "$v: $(tail -1 gpurun_out/pytest_$v.log)"
  done
fi
for round in $(seq 1 ${2:-2}); do
  for v in $1; do
    SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 200 > gpurun_out/ab_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_$v.log; exit 1; }
    python3 - "$v" "$round" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[1], "ms", d["ms_per_step"], d["kernels_ms_per_step"], "mid", d.get("ms_per_step_mid_collapse"), d.get("kernels_ms_per_step_mid_collapse"), flush=True)
PY
  done
done
