# PMC passes over BASELINE's larger configurations on one GPU, on the strong bench command itself
# (bench.py --strong --config C4|C5: one rank, the whole configuration), summarised into profiles/pmc_<C>.json for the
# `traffic` / `valu` fields of those lines:  CONFIGS="C4 C5" bash scripts/gpu_pmc_strong.sh
set +e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for cfg in ${CONFIGS:-C4 C5}; do
  mkdir -p gpurun_out/pmc_$cfg
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$cfg/v1_g$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --strong --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --mid-steps 0 > gpurun_out/pmc_$cfg/v1_g$i.log 2>&1; rc=$?
    echo "$cfg group $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$cfg/v1_g$i.log; exit $rc; fi
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_$cfg gpurun_out/pmc_$cfg.json $cfg > gpurun_out/pmc_summary_$cfg.log 2>&1; echo "$cfg summary rc=$?"
  cp gpurun_out/pmc_$cfg.json profiles/   # the box copy of the tree: the bench line below reads it
  timeout -k 10 300 python bench.py --strong --config $cfg --steps 100 --warmup 10 > gpurun_out/bench_strong_$cfg.log 2>&1; echo "$cfg bench rc=$?"
done
exit 0
