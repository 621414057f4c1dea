"""Extendable on-disk ensemble storage: the role the reference's extendable HDF5 datasets play
(supervillain/h5/extendable.py:62-74: a dataset created with maxshape (None, ...) and resized along the draw
axis by `extend_h5`, which Ensemble inherits, ensemble.py:16), without HDF5 (h5py is absent from this image and
from the GPU box; SURVEY.md 2 keeps the h5 layer out of scope).

A store is a directory: one raw C-order file per column (configuration fields, inline observables, index,
weight) plus `manifest.json` with each column's dtype, per-draw shape and draw count.  `extend` appends draws
to every column and then rewrites the manifest atomically, so a store read after a crash holds whole draws.
Columns are read back as read-only memory maps.
"""
import json
import os

import numpy as np

MANIFEST = 'manifest.json'


class ExtendableStore:
    def __init__(self, path, create=True):
        self.path = os.fspath(path)
        m = os.path.join(self.path, MANIFEST)
        if os.path.exists(m):
            with open(m) as f:
                self.manifest = json.load(f)
        elif create:
            os.makedirs(self.path, exist_ok=True)
            self.manifest = {'columns': {}, 'draws': 0}
        else:
            raise FileNotFoundError(f'{self.path} holds no {MANIFEST}')

    def __len__(self):
        return self.manifest['draws']

    def columns(self):
        return list(self.manifest['columns'])

    def _file(self, name):
        return os.path.join(self.path, name + '.bin')

    def extend(self, columns):
        """Append draws: `columns` maps each column name to an array whose leading axis is the draw axis (all
        of one length).  The first extend fixes the column set, dtypes and per-draw shapes; later ones must
        match them (as the reference's extendable datasets do)."""
        arrays = {k: np.ascontiguousarray(np.asarray(v)) for k, v in columns.items()}
        lengths = {a.shape[0] for a in arrays.values()}
        if len(lengths) != 1:
            raise ValueError(f'columns of unequal length: { {k: a.shape[0] for k, a in arrays.items()} }')
        k = lengths.pop()
        cols = self.manifest['columns']
        if cols:
            if set(cols) != set(arrays):
                raise KeyError(f'store columns {sorted(cols)} differ from {sorted(arrays)}')
            for name, a in arrays.items():
                c = cols[name]
                if np.dtype(c['dtype']) != a.dtype or tuple(c['shape']) != a.shape[1:]:
                    raise ValueError(f'column {name}: {a.dtype} {a.shape[1:]} does not extend '
                                     f'{c["dtype"]} {tuple(c["shape"])}')
        else:
            for name, a in arrays.items():
                cols[name] = {'dtype': a.dtype.str, 'shape': list(a.shape[1:])}
                open(self._file(name), 'wb').close()
        draws = self.manifest['draws']
        for name, a in arrays.items():
            item = a.dtype.itemsize * int(np.prod(a.shape[1:], dtype=np.int64))
            with open(self._file(name), 'r+b') as f:
                f.seek(draws * item)   # drop the tail a crashed extend may have left
                f.truncate()
                f.write(a.tobytes())
        self.manifest['draws'] = draws + k
        tmp = os.path.join(self.path, MANIFEST + '.tmp')
        with open(tmp, 'w') as f:
            json.dump(self.manifest, f)
        os.replace(tmp, os.path.join(self.path, MANIFEST))
        return self

    def read(self, name):
        """The column as a read-only (draws, *shape) memory map."""
        c = self.manifest['columns'][name]
        shape = (self.manifest['draws'],) + tuple(c['shape'])
        if shape[0] == 0:
            return np.zeros(shape, dtype=np.dtype(c['dtype']))
        return np.memmap(self._file(name), dtype=np.dtype(c['dtype']), mode='r', shape=shape)
