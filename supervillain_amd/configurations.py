"""A dict of Batch columns addressed by draw (supervillain/configurations.py:9-126, minus HDF5)."""


class Configurations:
    def __init__(self, dictionary):
        self.__dict__['fields'] = dictionary

    def __str__(self):
        return str(self.fields)

    def __contains__(self, name):
        return name in self.fields

    def __getitem__(self, index):
        if type(index) is int:
            return {k: v[index] for k, v in self.fields.items()}
        return Configurations({k: v[index] for k, v in self.fields.items()})

    def __setitem__(self, index, new):
        for k, v in new.items():
            self.fields[k][index] = v

    def __len__(self):
        n = None
        for v in self.fields.values():
            try:
                m = len(v)
            except TypeError:
                continue
            if n is None:
                n = m
            elif n != m:
                raise ValueError('Configurations have no consistent length')
        return n

    def items(self):
        return self.fields.items()

    def __getattr__(self, name):
        try:
            return self.fields[name]
        except KeyError:
            raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in self.fields:
            self.fields[name] = value
        else:
            self.__dict__[name] = value

    def __ior__(self, value):
        self.fields |= value
        return self

    def copy(self):
        return Configurations(self.fields.copy())
