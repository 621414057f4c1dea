set -u
bash scripts/profile.sh r01 > gpurun_out/profile_r01.log 2>&1; echo "profile rc=$?"; tail -30 gpurun_out/profile_r01.log
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench_full.log
