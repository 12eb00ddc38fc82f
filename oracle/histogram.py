"""oracle/histogram.py — TEST INFRASTRUCTURE ONLY (checker, never shipped).

Pure-Python restatement of fantoch's exact `Histogram`
(fantoch/src/metrics/histogram.rs:14-236) over a sorted {value: count} map,
used to check the product's dense-bin statistics (fx_hist_stats_compute /
fx_hist_percentile) and pinned by the reference's own KATs
(histogram.rs:390-463, see tests/test_oracle_kat.py).
"""
import math


class Histogram:
    """BTreeMap<u64, usize> of value -> occurrences (histogram.rs:15-18)."""

    def __init__(self, values=()):
        self.values = {}
        for v in values:
            self.increment(v)

    @classmethod
    def from_pairs(cls, pairs):
        h = cls()
        for v, c in pairs:
            if c:
                h.values[int(v)] = h.values.get(int(v), 0) + int(c)
        return h

    def increment(self, value):  # histogram.rs:55-59
        self.values[int(value)] = self.values.get(int(value), 0) + 1

    def merge(self, other):  # histogram_merge, histogram.rs:259-326 (key-wise sum)
        for v, c in other.values.items():
            self.values[v] = self.values.get(v, 0) + c

    def items(self):
        return sorted(self.values.items())

    def count(self):  # histogram.rs:34-36
        return sum(self.values.values())

    def _mean_and_count(self):  # histogram.rs:172-191
        s = sum(v * c for v, c in self.values.items())
        n = self.count()
        return (s / n if n else float("nan")), float(n)

    def mean(self):
        return self._mean_and_count()[0]

    def stddev(self):  # histogram.rs:199-219, corrected (n - 1)
        mean, count = self._mean_and_count()
        acc = 0.0
        for x, xc in self.items():
            diff = mean - float(x)
            acc += (diff * diff) * float(xc)
        return math.sqrt(acc / (count - 1.0)) if count > 1 else (0.0 if count == 1 else float("nan"))

    def cov(self):  # histogram.rs:193-197
        return self.stddev() / self.mean()

    def mdtm(self):  # histogram.rs:221-235
        mean, count = self._mean_and_count()
        acc = 0.0
        for x, xc in self.items():
            acc += abs(mean - float(x)) * float(xc)
        return acc / count

    def min(self):
        it = self.items()
        return float(it[0][0]) if it else float("nan")

    def max(self):
        it = self.items()
        return float(it[-1][0]) if it else float("nan")

    def percentile(self, p):  # histogram.rs:111-170
        assert 0.0 <= p <= 1.0
        if not self.values:
            return 0.0
        count = float(self.count())
        index = p * count
        index_rounded = float(round_half_away(index))
        is_whole = abs(index - index_rounded) == 0.0
        idx = int(index_rounded)
        data = self.items()
        pos = 0
        while True:
            value, c = data[pos]
            pos += 1
            if idx == c:
                left = float(value)
                right = float(data[pos][0]) if pos < len(data) else None
                break
            if idx < c:
                left = float(value)
                right = left
                break
            idx -= c
        if is_whole:
            return (left + right) / 2.0
        return left


def round_half_away(x):
    """Rust f64::round: half away from zero."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def round1(x):
    """F64::round (float.rs:22-24): format!("{:.1}") — Rust rounds half to even on the
    decimal representation like Python's format."""
    return "%.1f" % x
