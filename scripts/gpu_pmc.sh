# PMC passes (one counter group per run, --kernel-trace only; no sys/runtime trace with --pmc)
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  for v in 1; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/v${v}_g$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" --config C3 --steps 10 --warmup 2 > gpurun_out/pmc/v${v}_g$i.log 2>&1; rc=$?
    echo "group $i v$v rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/v${v}_g$i.log; exit $rc; fi
  done
done
# request-size breakdown (traffic accounting): a failed group is reported, not fatal
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum TCC_WRITEBACK_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum TCC_STREAMING_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/v1_g$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" --config C3 --steps 10 --warmup 2 > gpurun_out/pmc/v1_g$i.log 2>&1; rc=$?
  echo "group $i (extra) rc=$rc"
  [ $rc -ne 0 ] && tail -3 gpurun_out/pmc/v1_g$i.log
done
exit 0
