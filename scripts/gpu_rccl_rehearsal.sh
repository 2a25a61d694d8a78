# The in-library RCCL step (sph_comm_init, early sends, the flags' all-reduce) with two and four ranks on the box's
# one GPU: each rank poses as its own host (SPH_RCCL_HOST_PER_RANK -> NCCL_HOSTID), the exchanges go over RCCL's
# socket transport on loopback. bench.py checks the decomposed step against one context before timing.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export SPH_DIST_BACKEND=gloo SPH_RCCL_HOST_PER_RANK=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 SPH_HOST_TIMING=1
for n in ${RANKS:-2 4}; do
  timeout -k 10 ${LIMIT:-400} python bench.py --gpus $n --steps ${STEPS:-100} --warmup ${WARMUP:-10} --no-cpu-baseline --mid-steps 0 --watchdog 300 ${BENCH_EXTRA:-} > gpurun_out/rccl_$n.log 2> gpurun_out/rccl_$n.err; rc=$?
  echo "ranks $n rc=$rc"; grep -h '^{' gpurun_out/rccl_$n.log | cut -c 1-400; grep -h "\[host\]" gpurun_out/rccl_$n.err | head -8
  [ $rc -ne 0 ] && { tail -30 gpurun_out/rccl_$n.err; exit $rc; }
done
exit 0
