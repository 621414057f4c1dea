set -u
mkdir -p gpurun_out/r17
timeout -k 10 300 python scripts/debug_plaquette2.py > gpurun_out/r17/d.log 2>&1; echo "rc=$?"; cat gpurun_out/r17/d.log | head -60
