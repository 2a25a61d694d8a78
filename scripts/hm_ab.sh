# A/B of the force pass's hit-mask reader variants (build/variants/lib_*.so), interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for round in 1 2; do
  for v in ${HM_VARIANTS:-off queue prefetch prefetch_wpe5 queue_wpe5}; do
    SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 200 > gpurun_out/hm_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/hm_$v.log; exit 1; }
    python3 - "$v" "$round" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/hm_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[1], "ms", d["ms_per_step"], d["kernels_ms_per_step"], "mid", d.get("ms_per_step_mid_collapse"), d.get("kernels_ms_per_step_mid_collapse"), flush=True)
PY
  done
done
