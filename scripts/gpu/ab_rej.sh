mkdir -p gpurun_out/r3_rej
timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 300 > gpurun_out/r3_rej/new.log 2>&1 && \
SV_CHUNK=0 timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 300 > gpurun_out/r3_rej/nochunk.log 2>&1 && \
SV_CHUNK=0 SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_skipfj.so timeout -k 10 200 python -u scripts/perf/reject_window.py 4096 20 300 > gpurun_out/r3_rej/old.log 2>&1
cat gpurun_out/r3_rej/*.log
