source scripts/gpu/guard.sh
O=gpurun_out/r3_phc; mkdir -p $O
step cur timeout -k 10 200 python -u scripts/perf/philox_check.py 20000 > $O/cur.log 2>&1
cat $O/cur.log
step head env SV_LIB_OVERRIDE=supervillain_amd/variants/libsvhip_head.so timeout -k 10 200 python -u scripts/perf/philox_check.py 20000 > $O/head.log 2>&1
cat $O/head.log
