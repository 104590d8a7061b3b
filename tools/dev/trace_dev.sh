export TMPDIR=/tmp
rm -rf gpurun_out/tr; mkdir -p gpurun_out/tr
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr -o run -- python3 bench.py --steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile > gpurun_out/tr/log 2>&1
f=$(find gpurun_out/tr -name '*kernel_trace.csv' | head -1)
python3 tools/trace_summary.py $f 8 > gpurun_out/tr/summary.txt
cp $f gpurun_out/tr/kt.csv
