"""Markov-chain driver: the hot path's caller (supervillain/ensemble.py:16-302, minus HDF5 and analysis).

`Ensemble(S).generate(steps, G)` allocates storage from S.configurations, starts cold (all zeros)
or from a given configuration, and stores configuration[i] = G.step(configuration[i-1])
(ensemble.py:74-98)."""
import logging
import queue
import threading
import time

import numpy as np

from supervillain_amd.batch import Batch
from supervillain_amd.configurations import Configurations
from supervillain_amd.generator.combining import KeepEvery
from supervillain_amd.pipeline import DeviceChain, device_program, pinned_empty
from supervillain_amd.store import ExtendableStore

logger = logging.getLogger(__name__)


def _no_op(x, **kwargs):
    return x


class Ensemble:
    def __init__(self, action):
        self.Action = action

    def from_configurations(self, configurations):
        self.configuration = configurations
        return self

    def generate(self, steps, generator, start='cold', progress=_no_op, starting_index=0, index_stride=1,
                 device_resident=True, stream=None, stream_every=64):
        '''As the reference (ensemble.py:47-100).  With device_resident (default) and a generator built from this
        package's device generators (alone, Sequentially, KeepEvery), the fields stay in HBM for the whole run:
        each kept configuration is snapshotted on the device and copied straight into this ensemble's (page-locked)
        storage on a copy stream, overlapping the sweeps of the next one (supervillain_amd.pipeline; SURVEY.md 8f
        row 3) -- the same chain, counters and rng states as the per-step loop.

        stream: an ExtendableStore (or a path for one); every `stream_every` configurations, the finished ones (with
        their index and weight) are appended to it by a writer thread while generation goes on -- the role of the
        reference's extend_h5 (h5/extendable.py:62-74) for runs written out as they are produced.'''
        self.configuration = self.Action.configurations(steps)
        self.configuration |= generator.inline_observables(steps)
        self.index_stride = index_stride
        self.index = Batch(starting_index + self.index_stride * np.arange(steps))
        self.weight = Batch(np.ones(steps))
        if start == 'cold':
            seed = self.Action.configurations(1)[0]
        elif type(start) is dict:
            seed = start
        else:
            raise ValueError(f'Not sure how to transform a {type(start)} into a starting configuration.')
        writer = _StreamWriter(self, stream) if stream is not None else None
        t0 = time.perf_counter()
        try:
            program = device_program(generator) if device_resident and steps > 0 else None
            if program is not None:
                self._generate_resident(steps, program, seed, progress, writer, stream_every)
            else:
                self.configuration[0] = generator.step(seed)
                for i in progress(range(1, steps), desc='Generation'):
                    self.configuration[i] = generator.step(self.configuration[i - 1])
                    if writer is not None and (i + 1) % stream_every == 0:
                        writer.put(i + 1)
            if writer is not None:
                writer.put(steps)
        finally:
            if writer is not None:
                writer.close()
        self.start = start
        self.generator = generator
        logger.info(f'Generation of {steps} configurations: {time.perf_counter() - t0:.3f} s')
        for line in generator.report().split('\n'):
            logger.info(line)
        return self

    def _generate_resident(self, steps, program, seed, progress, writer, stream_every):
        chain = DeviceChain(self.Action, program)
        fields = self.configuration.fields
        x, y = chain.names
        ax, ay = Batch.as_array(fields[x]), Batch.as_array(fields[y])
        direct = (ax.dtype == chain.a.dtype and ay.dtype == chain.b.dtype and ax.shape[1:] == chain.a.shape
                  and ay.shape[1:] == chain.b.shape and ax.flags['C_CONTIGUOUS'] and ay.flags['C_CONTIGUOUS'])
        if direct and isinstance(fields[x], Batch) and isinstance(fields[y], Batch):
            # emissions land in library-owned page-locked storage (pipeline.pinned_empty), which the Batches keep
            fields[x]._data, fields[y]._data = pinned_empty(ax.shape, ax.dtype), pinned_empty(ay.shape, ay.dtype)
            ax, ay = fields[x]._data, fields[y]._data
        done = landed = 0  # draws queued for emission / confirmed landed by emit_wait
        try:
            chain.upload(seed)
            for i in progress(range(steps), desc='Generation'):
                obs = chain.advance()
                if direct:
                    chain.emit(ax[i], ay[i])
                    for k, v in obs.items():
                        fields[k][i] = v
                else:
                    self.configuration[i] = chain.download() | obs
                done = i + 1
                if writer is not None and (i + 1) % stream_every == 0:
                    if direct:
                        chain.emit_wait()
                        landed = done
                    writer.put(i + 1)
            if direct:
                chain.emit_wait()
                landed = done
        finally:
            try:
                if direct and landed < done:
                    chain.emit_wait()  # (a failure before the loop's last wait: land what was queued, if possible)
                    landed = done
            finally:
                if direct:
                    # the pinned storage is uninitialised (pinned_empty): rows no confirmed emission wrote read as zeros
                    ax[landed:], ay[landed:] = 0, 0
                chain.close()

    def columns(self, start=0, stop=None):
        """The ensemble's draws [start, stop) as store columns: configuration fields, index, weight."""
        cols = {k: Batch.as_array(v)[start:stop] for k, v in self.configuration.items()}
        cols['index'] = Batch.as_array(self.index)[start:stop]
        cols['weight'] = Batch.as_array(self.weight)[start:stop]
        return cols

    def to_store(self, path):
        """Write the ensemble as a new ExtendableStore at `path`; a store there that already holds draws is refused
        (FileExistsError: append with extend_store)."""
        store = ExtendableStore(path)
        if len(store):
            raise FileExistsError(f'{path} already holds {len(store)} draws; use extend_store')
        return store.extend(self.columns())

    def extend_store(self, store):
        """Append this ensemble's draws to an ExtendableStore (the reference's extend_h5, extendable.py:62-74)."""
        store = store if isinstance(store, ExtendableStore) else ExtendableStore(store, create=False)
        return store.extend(self.columns())

    @classmethod
    def from_store(cls, action, store):
        """An ensemble of the draws a store holds (copied into memory)."""
        store = store if isinstance(store, ExtendableStore) else ExtendableStore(store, create=False)
        fields = {k: Batch(np.array(store.read(k))) for k in store.columns() if k not in ('index', 'weight')}
        e = cls(action).from_configurations(Configurations(fields))
        e.index = Batch(np.array(store.read('index')))
        e.weight = Batch(np.array(store.read('weight')))
        e.index_stride = int(e.index.array[1] - e.index.array[0]) if len(e.index) > 1 else 1
        return e

    @classmethod
    def continue_from(cls, ensemble, steps, progress=_no_op):
        if not isinstance(ensemble, Ensemble):
            raise ValueError('ensemble should be a supervillain_amd.Ensemble.')
        try:
            generator, action = ensemble.generator, ensemble.Action
            last = ensemble.configuration[-1]
            index = ensemble.index[-1] + ensemble.index_stride
        except Exception:
            raise ValueError('The ensemble must provide a generator, an Action, and at least one configuration.')
        return Ensemble(action).generate(steps, generator, last, progress=progress, starting_index=index,
                                         index_stride=ensemble.index_stride)

    def __len__(self):
        return len(self.configuration)

    def cut(self, start):
        e = Ensemble(self.Action).from_configurations(self.configuration[start:])
        e.index = self.index[start:]
        e.index_stride = self.index_stride
        e.weight = self.weight[start:]
        e.generator = self.generator
        return e

    def every(self, stride):
        e = Ensemble(self.Action).from_configurations(self.configuration[::stride])
        e.index = self.index[::stride]
        e.index_stride = self.index_stride * stride
        e.weight = self.weight[::stride]
        e.generator = KeepEvery(stride, self.generator, blocked_inline=False)
        return e

    def __getattr__(self, name):
        if name == 'configuration':
            raise AttributeError(name)
        return getattr(self.configuration, name)


class _StreamWriter:
    """Appends finished draws of an ensemble to a store from a background thread (disk writes overlap the
    generation); errors surface in put() or close()."""

    def __init__(self, ensemble, store):
        self.ensemble = ensemble
        self.store = store if isinstance(store, ExtendableStore) else ExtendableStore(store)
        self.done = 0  # draws of this ensemble written so far
        self.q = queue.Queue()
        self.err = None
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        while True:
            stop = self.q.get()
            if stop is None:
                return
            if self.err is None and stop > self.done:
                try:
                    self.store.extend(self.ensemble.columns(self.done, stop))
                    self.done = stop
                except Exception as e:  # reported to the generating thread
                    self.err = e

    def _raise(self):
        if self.err is not None:
            raise self.err

    def put(self, stop):
        self._raise()
        self.q.put(stop)

    def close(self):
        self.q.put(None)
        self.thread.join()
        self._raise()
