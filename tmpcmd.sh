for i in 1 2; do
timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_floor$i.json 2>/dev/null || exit 1
PPO_SPLIT_CEIL=1 timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_ceil$i.json 2>/dev/null || exit 1
PPO_SERIAL=1 timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_sfloor$i.json 2>/dev/null || exit 1
PPO_SERIAL=1 PPO_SPLIT_CEIL=1 timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_sceil$i.json 2>/dev/null || exit 1
done
