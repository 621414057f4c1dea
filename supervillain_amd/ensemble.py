"""Markov-chain driver: the hot path's caller (supervillain/ensemble.py:16-302, minus HDF5 and analysis).

`Ensemble(S).generate(steps, G)` allocates storage from S.configurations, starts cold (all zeros)
or from a given configuration, and stores configuration[i] = G.step(configuration[i-1])
(ensemble.py:74-98)."""
import logging
import time

import numpy as np

from supervillain_amd.batch import Batch
from supervillain_amd.generator.combining import KeepEvery
from supervillain_amd.pipeline import DeviceChain, device_program

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
                 device_resident=True):
        '''As the reference (ensemble.py:47-100).  With device_resident (default) and a generator built from this
        package's device generators (alone, Sequentially, KeepEvery), the fields stay in HBM for the whole run and
        only each kept configuration is copied back (supervillain_amd.pipeline) -- the same
        chain, counters and rng states as the per-step loop.'''
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
        t0 = time.perf_counter()
        program = device_program(generator) if device_resident and steps > 0 else None
        if program is not None:
            chain = DeviceChain(self.Action, program)
            try:
                chain.upload(seed)
                self.configuration[0] = self._emit(chain)
                for i in progress(range(1, steps), desc='Generation'):
                    self.configuration[i] = self._emit(chain)
            finally:
                chain.close()
        else:
            self.configuration[0] = generator.step(seed)
            for i in progress(range(1, steps), desc='Generation'):
                self.configuration[i] = generator.step(self.configuration[i - 1])
        self.start = start
        self.generator = generator
        logger.info(f'Generation of {steps} configurations: {time.perf_counter() - t0:.3f} s')
        for line in generator.report().split('\n'):
            logger.info(line)
        return self

    @staticmethod
    def _emit(chain):
        obs = chain.advance()
        return chain.download() | obs

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
