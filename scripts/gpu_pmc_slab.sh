# PMC passes over the force pass at the per-rank shape of BASELINE's 8-GPU configuration (C5 on 8 GPUs: a rank holds
# ~2M particles of C5's 256 x 512 cross-section, ~7 columns): one context of C5's cross-section 16 lattice layers
# deep in x, with the y-band schedule (schedule.hip) and without, against C3 (DESIGN.md §4, round-5 verdict item 3). --kernel-trace only; one counter group per run.
set +e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for case in "slab8:--scenario 0,3,16,256,512,64,512,512" "slab8sched:--scenario 0,3,16,256,512,64,512,512" "C3:--config C3"; do
  name=${case%%:*}; args=${case#*:}
  if [ "$name" = slab8sched ]; then export SPH_SCHED=1; else unset SPH_SCHED; fi
  mkdir -p gpurun_out/pmc_$name
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$name/v1_g$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" $args --steps 10 --warmup 2 > gpurun_out/pmc_$name/v1_g$i.log 2>&1; rc=$?
    echo "$name group $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$name/v1_g$i.log; exit $rc; fi
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_$name gpurun_out/pmc_$name.json $name > gpurun_out/pmc_summary_$name.log 2>&1; echo "$name summary rc=$?"
  cat gpurun_out/pmc_summary_$name.log
done
exit 0
