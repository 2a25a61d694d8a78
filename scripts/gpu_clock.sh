# Shader clock during the VALU microbenchmark and the force pass (C3 and C5 force dispatches).
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/clock
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/valu_peak.bin 65536 > gpurun_out/clock/valu_peak_long.log 2>&1; rc=$?
echo "valu_peak rc=$rc"; cat gpurun_out/clock/valu_peak_long.log
[ $rc -ne 0 ] && exit $rc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$GRAFT_REPO_ROOT/gpurun_out/clock/valu" -o run --output-format csv -- ./scripts/valu_peak.bin 65536 > gpurun_out/clock/valu_pmc.log 2>&1; rc=$?
echo "valu pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/clock/valu_pmc.log; exit $rc; }
for c in C3 C5; do
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d "$GRAFT_REPO_ROOT/gpurun_out/clock/$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" --config $c --steps 20 --warmup 3 > gpurun_out/clock/$c.log 2>&1; rc=$?
  echo "$c pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/clock/$c.log; exit $rc; }
done
python3 scripts/clock_summary.py gpurun_out/clock/clock.json valu=gpurun_out/clock/valu C3=gpurun_out/clock/C3 C5=gpurun_out/clock/C5 valu_peak=gpurun_out/clock/valu_peak_long.log > gpurun_out/clock/summary.log 2>&1
echo "summary rc=$?"; grep -A6 '"k_force_tiled"\|"k_fma"\|"k_density_tiled"' gpurun_out/clock/summary.log | head -60
