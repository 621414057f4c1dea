source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r5_tsplit}
mkdir -p $O
export AMD_LOG_LEVEL=1
step tests timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_domain.py tests/test_gpu_split.py tests/test_gpu_villain.py tests/test_gpu_overflow.py tests/test_gpu_00_two_ranks.py > $O/tests.log 2>&1
tail -2 $O/tests.log
grep -E "[0-9]+ passed" $O/tests.log > /dev/null && ! grep -E "[0-9]+ (failed|errors?)( |,|$)" $O/tests.log > /dev/null || { echo "[tests] not green"; exit 1; }
unset AMD_LOG_LEVEL
step w24p env SV_DOMAIN_PREDICT=1 timeout -k 10 600 python -u bench.py --tiles 2x4 --weak --steps 10 --warmup 3 --warmup-s 0 --no-cpu-baseline > $O/w24p.json 2> $O/w24p.err
python -c "import json; d=json.loads(open('$O/w24p.json').readline()); print('weak 2x4 predicted', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling']['E_N'])"
step w11 timeout -k 10 300 python -u bench.py --tiles 1x1 --weak --steps 40 --warmup 5 --no-cpu-baseline > $O/w11.json 2> $O/w11.err
python -c "import json; d=json.loads(open('$O/w11.json').readline()); print('weak 1x1', round(d['value']/1e9,2), 'G', round(d['ms_per_step']*1e3,2), 'us wall', round(d['roofline']['avg_launch_us'],2), 'us kernel', d['config']['weak_scaling']['E_N'])"
