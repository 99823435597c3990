cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for cfg in c3 c4; do for mode in "1 1" "8 1" "8 0" "1 0" "4 0"; do set -- $mode
RV_GI_PRIO=$2 timeout -k 10 300 python bench.py --config $cfg --cpu-seconds 0 --steps 80 --inflight $1 > gpurun_out/b_$cfg.log 2>&1 || exit 3
tail -1 gpurun_out/b_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg inflight $1 giprio $2', d['ms_per_step'], d['stage_ms'])"
done; done
