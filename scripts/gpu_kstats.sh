# rocprofv3 kernel-trace stats of a plain C3 stepping run (per-kernel average durations).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/kst" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" ${RUNARGS:---config ${CFG:-C3}} --steps 50 --warmup 5 > gpurun_out/kst.log 2>&1
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kst/run_kernel_stats.csv")))
for r in rows:
    print(f'{r["Name"].split("(")[0]:40s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1000:8.2f}')
PY
