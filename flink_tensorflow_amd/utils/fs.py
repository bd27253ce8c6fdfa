"""File-system helpers with URI schemes (``LIB/util/GraphUtils.java:31-65`` read through
Flink's FileSystem; ``DefaultSavedModelLoader`` copies non-local model dirs to a local
temp dir, ``LIB/models/savedmodel/DefaultSavedModelLoader.scala:40-70``).

``file://`` and plain paths are local.  Other schemes are served by registered
``FileSystem`` implementations (``register_filesystem``); an in-memory ``mem://`` FS is
built in (used by tests to exercise the remote-copy path).
"""
from __future__ import annotations

import atexit
import fnmatch
import os
import shutil
import tempfile
import threading
from typing import Protocol
from urllib.parse import urlparse


class FileSystem(Protocol):
    def read_bytes(self, path: str) -> bytes: ...
    def list(self, path: str) -> list[str]: ...
    def is_dir(self, path: str) -> bool: ...
    def exists(self, path: str) -> bool: ...
    def write_bytes(self, path: str, data: bytes) -> None: ...


class LocalFS:
    def read_bytes(self, path):
        with open(path, "rb") as f:
            return f.read()

    def list(self, path):
        return sorted(os.path.join(path, p) for p in os.listdir(path))

    def is_dir(self, path):
        return os.path.isdir(path)

    def exists(self, path):
        return os.path.exists(path)

    def write_bytes(self, path, data):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "wb") as f:
            f.write(data)


class MemoryFS:
    """A process-local in-memory file system (``mem://bucket/path``)."""

    def __init__(self):
        self.files: dict[str, bytes] = {}
        self._lock = threading.Lock()

    def _k(self, path):
        return path.rstrip("/")

    def read_bytes(self, path):
        try:
            return self.files[self._k(path)]
        except KeyError:
            raise FileNotFoundError(path) from None

    def list(self, path):
        p = self._k(path) + "/"
        children = set()
        for k in self.files:
            if k.startswith(p):
                children.add(p + k[len(p):].split("/")[0])
        return sorted(children)

    def is_dir(self, path):
        p = self._k(path) + "/"
        return any(k.startswith(p) for k in self.files)

    def exists(self, path):
        return self._k(path) in self.files or self.is_dir(path)

    def write_bytes(self, path, data):
        with self._lock:
            self.files[self._k(path)] = bytes(data)


_LOCAL = LocalFS()
_REGISTRY: dict[str, FileSystem] = {"": _LOCAL, "file": _LOCAL, "mem": MemoryFS()}


def register_filesystem(scheme: str, fs: FileSystem) -> None:
    _REGISTRY[scheme] = fs


def get_fs(uri: str) -> tuple[FileSystem, str]:
    u = urlparse(uri)
    scheme = u.scheme if len(u.scheme) > 1 else ""  # windows drive letters are not schemes
    try:
        fs = _REGISTRY[scheme]
    except KeyError:
        raise ValueError(f"no file system registered for scheme {scheme!r}") from None
    if scheme in ("", "file"):
        return fs, (u.path if scheme == "file" else uri)
    return fs, uri


def is_local(uri: str) -> bool:
    return get_fs(uri)[0] is _LOCAL


def read_bytes(uri: str) -> bytes:
    fs, p = get_fs(uri)
    return fs.read_bytes(p)


def write_bytes(uri: str, data: bytes) -> None:
    fs, p = get_fs(uri)
    fs.write_bytes(p, data)


def read_all_lines(uri: str, encoding: str = "utf-8") -> list[str]:
    """``GraphUtils.readAllLines``."""
    return read_bytes(uri).decode(encoding).splitlines()


def exists(uri: str) -> bool:
    fs, p = get_fs(uri)
    return fs.exists(p)


def list_files(uri: str, recursive: bool = True, include: list[str] | None = None,
               exclude: list[str] | None = None) -> list[str]:
    """Lists files under a directory URI, filtered by glob include/exclude patterns
    (``**`` patterns as used by ``EX/inception/ImageInputFormat.scala:49-52``)."""
    fs, p = get_fs(uri)
    out = []
    stack = [p]
    while stack:
        cur = stack.pop()
        if not fs.is_dir(cur):
            out.append(cur)
            continue
        for child in fs.list(cur):
            if fs.is_dir(child):
                if recursive:
                    stack.append(child)
            else:
                out.append(child)

    def match(path, pats):
        name = os.path.basename(path)
        return any(fnmatch.fnmatch(path, pt) or fnmatch.fnmatch(name, pt.replace("**/", "").replace("**", "*"))
                   for pt in pats)

    if include:
        out = [f for f in out if match(f, include)]
    if exclude:
        out = [f for f in out if not match(f, exclude)]
    return sorted(out)


_TEMP_DIRS: list[str] = []


def _cleanup():
    for d in _TEMP_DIRS:
        shutil.rmtree(d, ignore_errors=True)


atexit.register(_cleanup)


def copy_to_local(uri: str) -> str:
    """Copies a (possibly remote) directory tree to a local temp dir deleted at exit."""
    if is_local(uri):
        return get_fs(uri)[1]
    fs, p = get_fs(uri)
    tmp = tempfile.mkdtemp(prefix="ftm-model-")
    _TEMP_DIRS.append(tmp)
    base = p.rstrip("/")
    for f in list_files(uri):
        rel = f[len(base):].lstrip("/")
        dst = os.path.join(tmp, rel)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        with open(dst, "wb") as out:
            out.write(fs.read_bytes(f))
    return tmp
