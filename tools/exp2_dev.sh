for X in 0 32; do
MGN_ABLATE=$X timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse > gpurun_out/abl_$X.log 2>&1 || exit 1
done
