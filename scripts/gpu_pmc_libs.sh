# PMC comparison of library builds (profiling only): for each library path (relative to the repo
# root), one rocprofv3 --pmc pass per counter group on a C3 stepping run; summarised per kernel.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcl
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); g=0
  for grp in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"; do
    g=$((g+1))
    SPHHIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmcl/l${i}_g$g" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" --config C3 --steps 10 --warmup 2 > gpurun_out/pmcl/l${i}_g$g.log 2>&1
  done
  echo "lib $i = $lib"
done
python3 - "$@" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
for i, lib in enumerate(sys.argv[1:], 1):
    acc = defaultdict(lambda: defaultdict(list))
    for d in glob.glob(f"gpurun_out/pmcl/l{i}_g*"):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("sph::", "")
            if k in ("k_force_tiled", "k_density_tiled"):
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(lib, k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(cs.items())})
PY
