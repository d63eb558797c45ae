timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_pipe$i.json 2>/dev/null || exit 1
PPO_X3_NOPIPE=1 timeout -k 10 400 python bench.py --no-rollout --no-cpu-baseline --steps 8 > gpurun_out/ab_nopipe$i.json 2>/dev/null || exit 1
done
