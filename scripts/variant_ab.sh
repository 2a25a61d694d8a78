# Interleaved A/B of library variants build/variants/lib_<v>.so: bash scripts/variant_ab.sh "v1 v2 ..." [rounds]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
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
