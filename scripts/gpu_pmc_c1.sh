# PMC of the C1 small-N step (k_density_fused, k_force_small), one counter group per run.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pmc1; mkdir -p $O; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/$O/g$i" -o run --output-format csv -- python3 scripts/run_steps.py --config C1 --steps 50 --warmup 10 > $O/g$i.log 2>&1; rc=$?
  echo "group $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/g$i.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc1/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for key in ("k_density_fused", "k_force_small"):
            if key in r["Kernel_Name"]:
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, d in acc.items():
    print(key, {c: round(sum(v) / len(v), 1) for c, v in sorted(d.items())})
PY
exit 0
