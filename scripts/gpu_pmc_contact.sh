# PMC passes over the one-launch Model R step (k_contact_fused): the rate table's R = 15 sphere and the controller's
# InitParticles scene, N = 4,096, one counter group per run.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/pmcc; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
i=0
for scene in "--sphere 4096" "--model-r 4096"; do
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/$O/g$i" -o run --output-format csv -- python3 scripts/run_steps.py $scene --steps 50 --warmup 10 > $O/g$i.log 2>&1; rc=$?
  echo "scene $scene group $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/g$i.log; exit $rc; }
done
done
python3 - <<'PY'
import csv, glob, collections
for half, gs in (("sphere", (1, 2)), ("controller", (3, 4))):
    acc = collections.defaultdict(list)
    for g in gs:
        for f in glob.glob(f"gpurun_out/pmcc/g{g}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_contact_fused" in r["Kernel_Name"]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(half, {c: round(sum(v) / len(v), 1) for c, v in sorted(acc.items())})
PY
exit 0
