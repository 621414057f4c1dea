"""Composite generators (supervillain/generator/combining.py:9-116).

KeepEvery(n, G) folds n steps of a hot-path generator into ONE device call (G._steps) when no
inline observable needs blocking, so an Ensemble stride pays one host<->device round trip."""
from supervillain_amd.generator.generator import Generator


class Sequentially(Generator):
    def __init__(self, generators):
        self.generators = generators

    def __str__(self):
        return 'Sequentially((' + ', '.join(str(g) for g in self.generators) + '))'

    def step(self, cfg):
        result = cfg
        for g in self.generators:
            result = g.step(result)
        return result

    def inline_observables(self, steps):
        combined = dict()
        for g in self.generators:
            combined |= g.inline_observables(steps)
        return combined

    def report(self):
        return '\n\n'.join(g.report() for g in self.generators)


class KeepEvery(Generator):
    def __init__(self, n, generator, blocked_inline=True):
        self.stride = n
        self.generator = generator
        self.blocked_inline = blocked_inline

    def __str__(self):
        return f'KeepEvery({self.stride}, {str(self.generator)})'

    def step(self, cfg):
        blocked = self.inline_observables(1) if self.blocked_inline else dict()
        if not blocked and hasattr(self.generator, '_steps'):
            return self.generator._steps(cfg, self.stride)
        for o in blocked:
            blocked[o] = blocked[o][0]
        result = cfg
        for _ in range(self.stride):
            result = self.generator.step(result)
            for o in blocked:
                blocked[o] += result[o] / self.stride
        return result | blocked

    def inline_observables(self, steps):
        return self.generator.inline_observables(steps)

    def report(self):
        return self.generator.report()
