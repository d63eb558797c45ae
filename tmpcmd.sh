cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-events --no-rollout"
PPO_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fz/s -o run --output-format csv -- $B > $R/gpurun_out/fz_s.log 2>&1
