"""Two ranks on ONE GPU (SV_DEVICE=0 for both), a 1x2 decomposition through RCCL, checked bit-for-bit against
the single-process emulation.  Launch: torchrun --nproc-per-node 2 scripts/perf/two_rank_same_gpu.py"""
import os, sys
import numpy as np
sys.path.insert(0, '.')
import torch.distributed as dist
from supervillain_amd.domain import VillainDomain
dist.init_process_group('gloo')
rank = dist.get_rank()
Nt, Nx = 256, 512
dom = VillainDomain.distributed(Nt, Nx, (1, 2), kappa=0.5, W=1)
dom.cold()
g = np.random.default_rng(11)
dom.run(40, g)
phi, n = dom.download()
dom.close()
out = [None, None]
dist.all_gather_object(out, (phi, n))
if rank == 0:
    phi = out[0][0].copy(); n = out[0][1].copy()
    phi[:, Nx // 2:] = out[1][0][:, Nx // 2:]; n[:, :, Nx // 2:] = out[1][1][:, :, Nx // 2:]
    ref = VillainDomain(Nt, Nx, (1, 2), kappa=0.5, W=1)
    ref.cold()
    ref.run(40, np.random.default_rng(11))
    p2, n2 = ref.download()
    print('two-rank RCCL == one-process emulation:', bool((p2 == phi).all() and (n2 == n).all()), flush=True)
dist.destroy_process_group()
