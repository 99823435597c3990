cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
echo "== gloo 2 ranks"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 30 --warmup 5 --dist-backend gloo > gpurun_out/mg_gloo2.log 2>&1; echo rc=$?
tail -3 gpurun_out/mg_gloo2.log | cut -c1-1500
echo "== nccl 2 ranks on 1 GPU"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/mg_nccl2.log 2>&1; echo rc=$?
tail -5 gpurun_out/mg_nccl2.log | cut -c1-2500
