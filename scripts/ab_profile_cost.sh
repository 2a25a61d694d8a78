cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
 for v in "--profile-every 4" "--no-profile" "--profile-every 16"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 0 $v > gpurun_out/abp.log 2>&1 || exit 1
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/abp.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['gpu_event_ms_per_step'])" "$r $v"
 done
done
