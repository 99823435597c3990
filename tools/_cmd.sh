cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
bash tools/gpu_run.sh smoke tests bench bench_c3 bench_c4 bench_c5 prof || exit 3
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 40 --warmup 5 --dist-backend gloo --cpu-seconds 0 > gpurun_out/mg_gloo2.log 2>&1; echo "gloo2 rc=$?"
tail -1 gpurun_out/mg_gloo2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gloo2', d['ms_per_step'], d['gather_check'], d['loop'], d['gather'])"
