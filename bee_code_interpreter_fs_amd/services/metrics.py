"""Service metrics in Prometheus text format (no client library needed).

The reference has no metrics at all; this adds request
counters and latency histograms per RPC/route and per execution phase,
exposed on the HTTP server's ``GET /metrics``.
"""

from __future__ import annotations

import bisect
import threading
from collections import defaultdict
from typing import Dict, Tuple

_BUCKETS_MS = (1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 10000, 30000, 60000)


class Histogram:
    def __init__(self) -> None:
        self.counts = [0] * (len(_BUCKETS_MS) + 1)
        self.total = 0.0
        self.n = 0

    def observe(self, v: float) -> None:
        self.counts[bisect.bisect_left(_BUCKETS_MS, v)] += 1
        self.total += v
        self.n += 1


class Metrics:
    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._phase_keys: dict = {}
        self.counters: Dict[Tuple[str, Tuple], float] = defaultdict(float)
        self.hists: Dict[Tuple[str, Tuple], Histogram] = {}

    def inc(self, name: str, value: float = 1.0, **labels) -> None:
        with self._lock:
            self.counters[(name, tuple(sorted(labels.items())))] += value

    def observe_ms(self, name: str, value_ms: float, **labels) -> None:
        key = (name, tuple(sorted(labels.items())))
        with self._lock:
            h = self.hists.get(key)
            if h is None:
                h = self.hists[key] = Histogram()
            h.observe(value_ms)

    def observe_phases(self, name: str, timings_ms: dict, label: str = "phase") -> None:
        """observe_ms for every (phase, ms) of one request under one lock:
        one cached lookup per phase straight to its histogram, the update
        inlined (called on every Execute, ~20 phases each)."""
        cache = self._phase_keys
        bl = bisect.bisect_left
        with self._lock:
            for phase, ms in timings_ms.items():
                h = cache.get((name, label, phase))
                if h is None:
                    key = (name, ((label, phase),))
                    h = self.hists.get(key)
                    if h is None:
                        h = self.hists[key] = Histogram()
                    cache[(name, label, phase)] = h
                h.counts[bl(_BUCKETS_MS, ms)] += 1
                h.total += ms
                h.n += 1

    def render(self) -> str:
        lines = []
        with self._lock:
            seen = set()
            for (name, labels), v in sorted(self.counters.items()):
                if name not in seen:
                    lines.append(f"# TYPE {name} counter")
                    seen.add(name)
                lines.append(f"{name}{_fmt(labels)} {v}")
            for (name, labels), h in sorted(self.hists.items(), key=lambda kv: kv[0]):
                if name not in seen:
                    lines.append(f"# TYPE {name} histogram")
                    seen.add(name)
                acc = 0
                for b, c in zip(_BUCKETS_MS, h.counts):
                    acc += c
                    lines.append(f"{name}_bucket{_fmt(labels + (('le', str(b)),))} {acc}")
                acc += h.counts[-1]
                lines.append(f"{name}_bucket{_fmt(labels + (('le', '+Inf'),))} {acc}")
                lines.append(f"{name}_sum{_fmt(labels)} {h.total}")
                lines.append(f"{name}_count{_fmt(labels)} {h.n}")
        return "\n".join(lines) + "\n"


def _fmt(labels) -> str:
    if not labels:
        return ""
    inner = ",".join(f'{k}="{str(v)}"' for k, v in labels)
    return "{" + inner + "}"


METRICS = Metrics()
