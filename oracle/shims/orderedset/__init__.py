"""Stand-in for the third-party `orderedset` package (absent here), enough for
the reference modules the golden generator imports (plenum/server/propagator.py
uses OrderedSet as an insertion-ordered set).  TEST INFRASTRUCTURE only."""


class OrderedSet:
    def __init__(self, iterable=()):
        self._d = dict.fromkeys(iterable)

    def add(self, x):
        self._d[x] = None

    def discard(self, x):
        self._d.pop(x, None)

    def remove(self, x):
        del self._d[x]

    def pop(self, last=True):
        if not self._d:
            raise KeyError('pop from an empty set')
        k = next(reversed(self._d)) if last else next(iter(self._d))
        del self._d[k]
        return k

    def __contains__(self, x):
        return x in self._d

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def __getitem__(self, i):
        return list(self._d)[i]

    def __repr__(self):
        return 'OrderedSet(%r)' % list(self._d)
