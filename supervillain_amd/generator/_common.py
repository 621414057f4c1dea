"""Shared plumbing of the device-backed generators."""
import numpy as np

from supervillain_amd import _native
from supervillain_amd._abi import rng_from_numpy, rng_to_numpy


def wrap_like(template, data, degree, lattice):
    """Return `data` as the caller's Form type (ours or the reference's), so results drop into either."""
    cls = type(template)
    if hasattr(template, 'degree') and hasattr(template, 'lattice') and cls is not np.ndarray:
        try:
            return cls(data, degree=degree, lattice=lattice)
        except TypeError:
            pass
    from supervillain_amd.lattice import Form
    return Form(data, degree=degree, lattice=lattice)


class DeviceState:
    """Lazily created device-resident field state; never pickled (generators stay persistable)."""

    def __getstate__(self):
        d = self.__dict__.copy()
        d.pop('_dev', None)
        return d

    def _device_context(self):
        return _native.context(getattr(self, 'device', None))


__all__ = ['wrap_like', 'DeviceState', 'rng_from_numpy', 'rng_to_numpy']
