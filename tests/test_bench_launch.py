"""bench.py's multi-GPU launcher on CPU: `python bench.py --gpus N` (the form the driver may use) starts N ranks
through torch.distributed.run when WORLD_SIZE is unset, and refuses a world size that differs from --gpus."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=e, capture_output=True,
                          text=True, timeout=240)


def test_gpus_flag_spawns_ranks():
    p = _run(['--gpus', '2', '--workload', 'ranks'])
    assert p.returncode == 0, p.stderr[-2000:]
    line = [x for x in p.stdout.splitlines() if x.startswith('{')][-1]
    d = json.loads(line)
    assert d['world'] == 2 and d['rank_sum'] == 1.0 and d['master_addr'] == '127.0.0.1'


def test_world_size_mismatch_fails():
    p = _run(['--gpus', '4', '--workload', 'ranks'], env={'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert p.returncode == 2 and 'WORLD_SIZE=2' in p.stderr


def test_launch_command_shape():
    import bench
    cmd = bench.launch_command(8, ['--gpus', '8', '--steps', '5'], 29512)
    assert cmd[1:4] == ['-m', 'torch.distributed.run', '--nnodes=1'] and '--nproc-per-node=8' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1' and cmd[-4:] == ['--gpus', '8', '--steps', '5']
