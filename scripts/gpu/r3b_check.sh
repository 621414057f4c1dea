# Re-entry check: full -m gpu suite, smoke, one driver-form bench line.
source scripts/gpu/guard.sh
export TMPDIR=/tmp
O=gpurun_out/r3b_check
mkdir -p $O
step tests timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/tests.log 2>&1
tail -5 $O/tests.log
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step d1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_1.json 2> $O/driver_1.err
cat $O/driver_1.json
