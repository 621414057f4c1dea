"""Per-draw storage columns (supervillain/batch.py:53-227), without the HDF5 layer.

A Batch is an array with a leading draw axis.  Writing a draw goes through a lossless-cast check
(batch.py:206-227): the generators must return float phi and integer n/m/v."""
import numbers
import warnings

import numpy as np


class Batch:
    def __init__(self, draws_or_data, *, cls=None, shape=None, dtype=None, **item_kwargs):
        if isinstance(draws_or_data, numbers.Integral) and not isinstance(draws_or_data, bool):
            if cls is not None:
                spatial = cls.spatial_shape(**item_kwargs)
            elif shape is None:
                raise ValueError('Batch(draws, …) requires shape= when cls is None.')
            else:
                spatial = tuple(shape)
            arr = np.zeros((int(draws_or_data),) + spatial, dtype=float if dtype is None else dtype)
        else:
            arr = np.asarray(draws_or_data) if dtype is None else self._checked_array(draws_or_data, dtype)
        self._data = arr
        self.cls = cls
        self.dtype = arr.dtype
        self._item_kwargs = item_kwargs

    @property
    def array(self):
        return self._data

    @staticmethod
    def as_array(column):
        return column.array if isinstance(column, Batch) else column

    @property
    def shape(self):
        return self._data.shape

    def __len__(self):
        return len(self._data)

    def __getitem__(self, index):
        if isinstance(index, numbers.Integral) and not isinstance(index, bool):
            item = self._data[index]
            return item if self.cls is None else self.cls(item, dtype=self.dtype, **self._item_kwargs)
        if type(index) is slice:
            return Batch(self._data[index], cls=self.cls, dtype=self.dtype, **self._item_kwargs)
        return self._data[index]

    def __setitem__(self, index, item):
        self._data[index] = self._checked_array(item, self.dtype)

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    @staticmethod
    def _checked_array(data, dtype):
        arr = np.asarray(data)
        dtype = np.dtype(dtype)
        if arr.dtype == dtype:
            return arr
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            out = arr.astype(dtype)
        if not np.array_equal(out, arr):
            raise TypeError(f'Batch cannot store {arr.dtype} data as {dtype} without loss '
                            '(the values do not round-trip); convert it explicitly first.')
        return out

    def __repr__(self):
        name = self.cls.__name__ if self.cls is not None else 'ndarray'
        return f'Batch(shape={self.shape}, cls={name}, dtype={self.dtype})'
