"""The two actions the hot-path generators sample (host side; NumPy).

Villain  (supervillain/action/villain.py:12-141):  S = kappa/2 sum_l (d phi - 2 pi n)_l^2, fields phi
(float 0-form) and n (int 1-form), constraint dn = 0 mod W.
Worldline (supervillain/action/worldline.py:12-114): S = 1/(2 kappa) sum_l (m - delta v / W)_l^2 + const,
fields m (int 1-form, delta m = 0) and v (int 2-form; float when W is infinite).
"""
import numpy as np

from supervillain_amd.batch import Batch
from supervillain_amd.configurations import Configurations
from supervillain_amd.lattice import Form, Lattice, d, delta


class Villain:
    def __init__(self, lattice, kappa, W=1):
        if not isinstance(lattice, Lattice):
            raise TypeError(f'Villain requires a supervillain_amd.lattice.Lattice, got {type(lattice).__name__}')
        self.Lattice = lattice
        self.kappa = kappa
        self.W = W

    def __str__(self):
        return f'Villain({self.Lattice}, κ={self.kappa}, W={self.W})'

    def links(self, phi, n):
        return d(phi) - 2 * np.pi * n

    def __call__(self, phi, n, **kwargs):
        return (self.kappa / 2) * (self.links(phi, n) ** 2).sum()

    def configurations(self, count):
        L = self.Lattice
        return Configurations({
            'phi': Batch(count, cls=Form, degree=0, lattice=L),
            'n': Batch(count, cls=Form, degree=1, lattice=L, dtype=int),
        })

    def valid(self, configuration):
        dn = d(configuration['n'])
        zero = np.mod(dn, self.W) if self.W < float('inf') else dn
        return bool((zero == 0).all())


class Worldline:
    def __init__(self, lattice, kappa, W=1):
        self.Lattice = lattice
        self.kappa = kappa
        self.W = W
        self._constant_offset = lattice.links / 2 * np.log(2 * np.pi * kappa) - lattice.sites * np.log(2 * np.pi)
        self._W = W if W < float('inf') else 2 * np.pi

    def __str__(self):
        return f'Worldline({self.Lattice}, κ={self.kappa}, W={self.W})'

    def valid(self, configuration):
        return bool((delta(configuration['m']) == 0).all())

    def __call__(self, m, v, **kwargs):
        if not self.valid({'m': m}):
            raise ValueError('The one-form m does not satisfy the constraint δm = 0 everywhere.')
        return 0.5 / self.kappa * np.sum((m - delta(v) / self._W) ** 2) + self._constant_offset

    def configurations(self, count):
        L = self.Lattice
        v_dtype = int if self.W < float('inf') else float
        return Configurations({
            'm': Batch(count, cls=Form, degree=1, lattice=L, dtype=int),
            'v': Batch(count, cls=Form, degree=2, lattice=L, dtype=v_dtype),
        })
