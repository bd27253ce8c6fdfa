"""Minimal complex-event processing (the ``flink-cep`` subset used by the reference's
"Johnny" example, ``EX/inception/johnny.scala:52-62``):

    Pattern.begin("a").where(p1).followed_by("b").where(p2).followed_by("c").where(p3).within(60)
    CEP.pattern(stream, pattern).select(on_match, on_timeout)

Semantics: stages are matched in order; ``followed_by`` is relaxed contiguity with
skip-till-next-match (non-matching events in between are ignored; a partial match advances
on the first matching event), ``next`` is strict contiguity.  A partial match whose first
event is older than ``within`` times out: ``on_timeout(partial, timeout_ts)`` is emitted.
Time is the record timestamp when present, else processing time.  Optional keying
(``key_by`` before ``CEP.pattern``) runs one NFA per key.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Any, Callable

from .executor import Partitioner
from .operators import Operator


@dataclass
class _Stage:
    name: str
    conditions: list = field(default_factory=list)
    strict: bool = False

    def accepts(self, v) -> bool:
        return all(c(v) for c in self.conditions)


class Pattern:
    def __init__(self, stages: list[_Stage], window: float | None = None):
        self.stages = stages
        self.window = window

    @staticmethod
    def begin(name: str) -> "Pattern":
        return Pattern([_Stage(name)])

    def where(self, cond: Callable[[Any], bool]) -> "Pattern":
        st = [_Stage(s.name, list(s.conditions), s.strict) for s in self.stages]
        st[-1].conditions.append(cond)
        return Pattern(st, self.window)

    def followed_by(self, name: str) -> "Pattern":
        return Pattern(self.stages + [_Stage(name)], self.window)

    followedBy = followed_by

    def next(self, name: str) -> "Pattern":
        return Pattern(self.stages + [_Stage(name, strict=True)], self.window)

    def within(self, seconds: float) -> "Pattern":
        return Pattern(self.stages, seconds)


@dataclass
class _Partial:
    events: dict
    start: float
    stage: int


class CEPOperator(Operator):
    def __init__(self, pattern: Pattern, on_match, on_timeout, key_selector=None, name="cep"):
        super().__init__(None, name)
        self.pattern = pattern
        self.on_match = on_match
        self.on_timeout = on_timeout
        self.key_selector = key_selector
        self.partials: dict[Any, list[_Partial]] = {}

    def _now(self, ts):
        return ts if ts is not None else time.time()

    _evt = False  # event-time mode: records carry timestamps

    def process(self, rec, input_index=0):
        if rec.ts is not None:
            self._evt = True
        now = self._now(rec.ts)
        key = self.key_selector(rec.value) if self.key_selector else None
        self._expire(now, key)
        st = self.pattern.stages
        nxt: list[_Partial] = []
        for p in self.partials.get(key, []):
            stage = st[p.stage]
            if stage.accepts(rec.value):
                ev = dict(p.events)
                ev[stage.name] = rec.value
                if p.stage + 1 == len(st):
                    self.out.emit(self.on_match(ev), rec.ts)
                else:
                    nxt.append(_Partial(ev, p.start, p.stage + 1))
            elif not stage.strict:
                nxt.append(p)
        if st[0].accepts(rec.value):
            ev = {st[0].name: rec.value}
            if len(st) == 1:
                self.out.emit(self.on_match(ev), rec.ts)
            else:
                nxt.append(_Partial(ev, now, 1))
        self.partials[key] = nxt

    def _expire(self, now, key=None):
        w = self.pattern.window
        if w is None:
            return
        keys = [key] if key is not None and key in self.partials else list(self.partials)
        for k in keys:
            keep = []
            for p in self.partials.get(k, []):
                if now - p.start > w:
                    if self.on_timeout is not None:
                        self.out.emit(self.on_timeout(p.events, p.start + w), None)
                else:
                    keep.append(p)
            self.partials[k] = keep

    def on_idle(self, now):
        if not self._event_time():
            self._expire(time.time())

    def on_watermark(self, ts):
        if self._event_time():
            self._expire(ts)

    def _event_time(self) -> bool:
        return self._evt or self.current_watermark > float("-inf")

    def next_deadline(self):
        if self._event_time():
            return None
        w = self.pattern.window
        starts = [p.start for ps in self.partials.values() for p in ps]
        return (min(starts) + w) if (w is not None and starts) else None

    def end_input(self):
        self._expire(float("inf"))

    def snapshot_extra(self):
        return {"partials": self.partials}

    def restore_extra(self, extra):
        if extra:
            self.partials = extra.get("partials", {})


class PatternStream:
    def __init__(self, stream, pattern: Pattern):
        self.stream = stream
        self.pattern = pattern

    def select(self, on_match: Callable[[dict], Any], on_timeout: Callable[[dict, float], Any] | None = None,
               name: str = "cep-select"):
        pat = self.pattern
        ks = getattr(self.stream, "key_selector", None)
        part = Partitioner("hash", ks) if ks is not None else Partitioner("global")
        par = None if ks is not None else 1
        return self.stream._add(name, lambda: CEPOperator(pat, on_match, on_timeout, ks, name), par, part)


class CEP:
    @staticmethod
    def pattern(stream, pattern: Pattern) -> PatternStream:
        return PatternStream(stream, pattern)
