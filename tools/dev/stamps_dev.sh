#!/bin/bash
# run a short bench with a MGN_STAMPS build; per-launch phase stamps go to gpurun_out/stamps.log
timeout -k 10 300 python3 bench.py --steps 3 --warmup 2 --cpu-steps 0 --no-mse --no-profile > gpurun_out/stamps.log 2>&1
