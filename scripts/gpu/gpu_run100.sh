source scripts/gpu/guard.sh
mkdir -p gpurun_out/r100
for rep in 1 2 3; do
step b$rep timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r100/b$rep.log 2>&1
echo RUN $rep $(grep -o '"value": [0-9.]*' gpurun_out/r100/b$rep.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r100/b$rep.log)
done
step long timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2000 > gpurun_out/r100/long.log 2>&1
echo LONG $(grep -o '"value": [0-9.]*' gpurun_out/r100/long.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/r100/long.log)
