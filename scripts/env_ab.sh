# Interleaved A/B of one library under environment settings:
#   bash scripts/env_ab.sh VAR "v1 v2" [rounds]
# Each round runs bench.py (200 steps from rest + 200 mid-collapse) once per value of VAR, in turn.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
var=$1
for round in $(seq 1 ${3:-2}); do
  for v in $2; do
    env "$var=$v" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 200 > gpurun_out/ab_env_$v.log 2>&1 || { echo "$var=$v failed"; tail -3 gpurun_out/ab_env_$v.log; exit 1; }
    python3 - "$v" "$round" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_env_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[1], "ms", d["ms_per_step"], d["kernels_ms_per_step"], "mid", d.get("ms_per_step_mid_collapse"), d.get("kernels_ms_per_step_mid_collapse"), flush=True)
PY
  done
done
