"""supervillain_amd -- an MI355X (gfx950) Metropolis sweep engine behind supervillain's generator API.

The hot path of evanberkowitz/supervillain -- NeighborhoodUpdate (Villain), CoexactUpdate and
PlaquetteUpdate (Worldline) -- runs as hand-written HIP kernels in libsvhip.so (C-ABI:
include/supervillain_amd.h), reached from these Python classes, which keep the reference's plugin
interface: Ensemble(S).generate(steps, G) with G.step(cfg) -> cfg.
"""
from supervillain_amd import action, generator, lattice
from supervillain_amd.action import Villain, Worldline
from supervillain_amd.ensemble import Ensemble
from supervillain_amd.lattice import Form, Lattice, Lattice2D

__all__ = ['Ensemble', 'Lattice', 'Lattice2D', 'Form', 'Villain', 'Worldline', 'action', 'generator', 'lattice']
