"""The generator plugin protocol (supervillain/generator/generator.py:3-33).

A generator maps a configuration dict to the next one with `step(cfg) -> cfg`, may declare inline
observables with `inline_observables(steps) -> dict[str, Batch]`, and reports acceptance statistics
with `report() -> str`."""


class Generator:
    def step(self, configuration):
        return configuration.copy()

    def inline_observables(self, steps):
        return dict()

    def report(self):
        return ''
