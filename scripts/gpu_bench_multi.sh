# rehearse bench.py --gpus 2 on one GPU (gloo, host-staged halos), then N=1
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SPH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench2.log 2>&1; rc=$?
echo "bench2 rc=$rc"; grep -v amdgpu.ids gpurun_out/bench2.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 8 > gpurun_out/bench1.log 2>&1; rc=$?
echo "bench1 rc=$rc"; grep -v amdgpu.ids gpurun_out/bench1.log | tail -3
exit $rc
