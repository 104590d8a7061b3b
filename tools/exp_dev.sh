export TMPDIR=/tmp
for X in 1 2; do
rm -rf gpurun_out/tr$X; mkdir -p gpurun_out/tr$X
MGN_WG_EXP=$X timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr$X -o run -- python3 bench.py --steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile > gpurun_out/tr$X/log 2>&1 || exit 1
f=$(find gpurun_out/tr$X -name '*kernel_trace.csv' | head -1)
python3 tools/trace_summary.py $f 8 > gpurun_out/tr$X/summary.txt
rm -f $f
done
