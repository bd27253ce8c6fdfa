"""Operator and keyed state (Flink managed state), snapshotted at checkpoint barriers."""
from __future__ import annotations

import copy
from dataclasses import dataclass
from typing import Any, Callable


@dataclass(frozen=True)
class ValueStateDescriptor:
    name: str
    default: Any = None


@dataclass(frozen=True)
class ListStateDescriptor:
    name: str


@dataclass(frozen=True)
class MapStateDescriptor:
    name: str


@dataclass(frozen=True)
class ReducingStateDescriptor:
    name: str
    reduce: Callable


class ListState:
    def __init__(self, backing: list):
        self._l = backing

    def get(self) -> list:
        return list(self._l)

    def add(self, v):
        self._l.append(v)

    def add_all(self, vs):
        self._l.extend(vs)

    def update(self, vs):
        self._l[:] = list(vs)

    def clear(self):
        self._l.clear()


class OperatorStateStore:
    """Per-subtask list states (re-distributable on rescale: even split / union)."""

    def __init__(self, snapshot: dict | None = None):
        self._lists: dict[str, list] = copy.deepcopy(snapshot.get("lists", {})) if snapshot else {}
        self.blobs: dict[str, Any] = dict(snapshot.get("blobs", {})) if snapshot else {}

    def get_list_state(self, desc) -> ListState:
        name = desc.name if hasattr(desc, "name") else str(desc)
        return ListState(self._lists.setdefault(name, []))

    get_union_list_state = get_list_state

    def snapshot(self) -> dict:
        return {"lists": copy.deepcopy(self._lists), "blobs": dict(self.blobs)}


class _KeyedValue:
    def __init__(self, store: "KeyedStateStore", desc):
        self._s, self._d = store, desc

    def value(self):
        return self._s.data.setdefault(self._d.name, {}).get(self._s.current_key, copy.copy(self._d.default))

    def update(self, v):
        self._s.data.setdefault(self._d.name, {})[self._s.current_key] = v

    def clear(self):
        self._s.data.setdefault(self._d.name, {}).pop(self._s.current_key, None)


class _KeyedList(_KeyedValue):
    def get(self):
        return list(self._s.data.setdefault(self._d.name, {}).get(self._s.current_key, []))

    def add(self, v):
        self._s.data.setdefault(self._d.name, {}).setdefault(self._s.current_key, []).append(v)

    def update(self, vs):
        self._s.data.setdefault(self._d.name, {})[self._s.current_key] = list(vs)


class _KeyedMap(_KeyedValue):
    def _m(self):
        return self._s.data.setdefault(self._d.name, {}).setdefault(self._s.current_key, {})

    def get(self, k):
        return self._m().get(k)

    def put(self, k, v):
        self._m()[k] = v

    def contains(self, k):
        return k in self._m()

    def remove(self, k):
        self._m().pop(k, None)

    def items(self):
        return list(self._m().items())

    def keys(self):
        return list(self._m().keys())


class _KeyedReducing(_KeyedValue):
    def add(self, v):
        cur = self.value()
        self.update(v if cur is None else self._d.reduce(cur, v))

    def get(self):
        return self.value()


class KeyedStateStore:
    """State scoped to the current key of a keyed operator."""

    def __init__(self, snapshot: dict | None = None):
        self.data: dict[str, dict] = copy.deepcopy(snapshot) if snapshot else {}
        self.current_key = None

    def get_state(self, desc):
        if isinstance(desc, ValueStateDescriptor):
            return _KeyedValue(self, desc)
        if isinstance(desc, ListStateDescriptor):
            return _KeyedList(self, desc)
        if isinstance(desc, MapStateDescriptor):
            return _KeyedMap(self, desc)
        if isinstance(desc, ReducingStateDescriptor):
            return _KeyedReducing(self, desc)
        raise TypeError(f"unknown state descriptor {desc!r}")

    def snapshot(self) -> dict:
        return copy.deepcopy(self.data)
