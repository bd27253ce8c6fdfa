"""In-tree build of the three native extensions.

* ``_native``  — host C++ runtime (csrc/*.cpp): wire codecs, protobuf scanning, Example
  parsing, STRING tensors, CRC32C/SSTable bundle I/O, staging gather.  Built with g++.
* ``_hip``     — CDNA4 (gfx950) HIP kernels (kernels/*.hip) + their pybind11 launchers.
  Built with ``hipcc --offload-arch=gfx950``; cross-compiles without a GPU.
* ``_rccl``    — direct RCCL C-API binding (csrc_rccl/rccl.cpp): communicator init from a
  ncclUniqueId, broadcast / all-reduce / all-gather / reduce-scatter on HIP streams.
  Host-only code built with hipcc, linked against ``librccl.so.1``.

All land next to this file (``setup.py build_ext --inplace`` semantics) so that the
``.so`` travels with a repo snapshot to the GPU box.  A content hash of the sources and
flags is stored beside each library; a rebuild happens only when it changes.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
CSRC_RCCL = PKG / "csrc_rccl"
KERNELS = PKG / "kernels"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
# what the last build_* call did per library: "compiled" (from source) or "reused" (the
# stamped library matched the sources and flags); FTM_FORCE_BUILD=1 forces "compiled"
STATUS: dict[str, str] = {}


def _forced(force: bool) -> bool:
    return force or os.environ.get("FTM_FORCE_BUILD", "") == "1"
HIP_ARCH = os.environ.get("FTM_HIP_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _digest(files: list[Path], flags: list[str]) -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _up_to_date(lib: Path, digest: str) -> bool:
    stamp = lib.with_suffix(lib.suffix + ".sha256")
    return lib.exists() and stamp.exists() and stamp.read_text().strip() == digest


def _stamp(lib: Path, digest: str) -> None:
    lib.with_suffix(lib.suffix + ".sha256").write_text(digest + "\n")


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def native_lib_path() -> Path:
    return PKG / f"_native{EXT_SUFFIX}"


def hip_lib_path() -> Path:
    return PKG / f"_hip{EXT_SUFFIX}"


def build_native(force: bool = False, verbose: bool = False) -> Path:
    srcs = sorted(CSRC.glob("*.cpp"))
    hdrs = sorted(CSRC.glob("*.h"))
    flags = ["-O3", "-std=c++17", "-shared", "-fPIC", "-msse4.2", "-mavx2", "-mfma", "-pthread", "-fvisibility=hidden"]
    extra = os.environ.get("FTM_NATIVE_CFLAGS", "").split()  # e.g. sanitizer builds
    lib = native_lib_path()
    dig = _digest(srcs + hdrs, flags + extra)
    if not _forced(force) and _up_to_date(lib, dig):
        STATUS["_native"] = "reused"
        return lib
    STATUS["_native"] = "compiled"
    cxx = os.environ.get("CXX", "g++")
    tmp = lib.with_name(lib.name + ".tmp")
    cmd = [cxx, *flags, *extra, *_pybind_includes(), *map(str, srcs), "-lrt", "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    _run(cmd)
    os.replace(tmp, lib)
    _stamp(lib, dig)
    return lib


SANITIZERS = {
    "asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer"],
}


def build_native_sanitized(kind: str, out_dir: str | os.PathLike) -> Path:
    """Host runtime built with a sanitizer (``asan`` = AddressSanitizer + UBSan, ``tsan`` =
    ThreadSanitizer) into ``out_dir`` — never over the production library.  Load it in a
    child process with the matching runtime preloaded (``LD_PRELOAD``) and
    ``FTM_NATIVE_LIB`` pointing at it (``tests/test_sanitizers.py``)."""
    srcs = sorted(CSRC.glob("*.cpp"))
    flags = ["-O1", "-g", "-std=c++17", "-shared", "-fPIC", "-msse4.2", "-pthread", *SANITIZERS[kind]]
    out = Path(out_dir) / f"_native{EXT_SUFFIX}"
    out.parent.mkdir(parents=True, exist_ok=True)
    _run([os.environ.get("CXX", "g++"), *flags, *_pybind_includes(), *map(str, srcs), "-lrt", "-o", str(out)])
    return out


def sanitizer_runtime(kind: str) -> str:
    lib = {"asan": "libasan.so", "tsan": "libtsan.so"}[kind]
    cxx = os.environ.get("CXX", "g++")
    return subprocess.run([cxx, f"-print-file-name={lib}"], stdout=subprocess.PIPE, text=True).stdout.strip()


def hip_flags() -> list[str]:
    return [
        f"--offload-arch={HIP_ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-ffp-contract=fast",
        "-munsafe-fp-atomics",
        "-fvisibility=hidden",
        f"-I{KERNELS}",
    ]


def build_hip(force: bool = False, verbose: bool = False, jobs: int | None = None) -> Path:
    srcs = sorted(KERNELS.glob("*.hip"))
    hdrs = sorted(KERNELS.glob("*.h")) + sorted(KERNELS.glob("*.cuh"))
    flags = hip_flags()
    lib = hip_lib_path()
    dig = _digest(srcs + hdrs, flags)
    if not _forced(force) and _up_to_date(lib, dig):
        STATUS["_hip"] = "reused"
        return lib
    STATUS["_hip"] = "compiled"
    hipcc = os.environ.get("HIPCC", f"{ROCM}/bin/hipcc")
    objdir = PKG / "build" / "hip_obj"
    objdir.mkdir(parents=True, exist_ok=True)
    inc = _pybind_includes()

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        cmd = [hipcc, *flags, *inc, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        return obj

    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = lib.with_name(lib.name + ".tmp")
    _run([hipcc, f"--offload-arch={HIP_ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)])
    os.replace(tmp, lib)
    _stamp(lib, dig)
    return lib


def rccl_lib_path() -> Path:
    return PKG / f"_rccl{EXT_SUFFIX}"


def build_rccl(force: bool = False, verbose: bool = False) -> Path:
    srcs = sorted(CSRC_RCCL.glob("*.cpp"))
    flags = ["-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__",
             f"-I{ROCM}/include", f"-L{ROCM}/lib", "-lrccl", "-lamdhip64"]
    lib = rccl_lib_path()
    dig = _digest(srcs, flags)
    if not _forced(force) and _up_to_date(lib, dig):
        STATUS["_rccl"] = "reused"
        return lib
    STATUS["_rccl"] = "compiled"
    hipcc = os.environ.get("HIPCC", f"{ROCM}/bin/hipcc")
    tmp = lib.with_name(lib.name + ".tmp")
    # -x c++ : host-only translation unit (no device code, no offload bundle)
    cmd = [hipcc, "-x", "c++", *_pybind_includes(), *map(str, srcs), *flags, "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    _run(cmd)
    os.replace(tmp, lib)
    _stamp(lib, dig)
    return lib


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_native(force=force, verbose=verbose)
    build_hip(force=force, verbose=verbose)
    build_rccl(force=force, verbose=verbose)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("what", nargs="?", default="all", choices=["all", "native", "hip", "rccl"])
    a = ap.parse_args()
    if a.what in ("all", "native"):
        print(build_native(a.force, a.verbose), STATUS.get("_native"))
    if a.what in ("all", "hip"):
        print(build_hip(a.force, a.verbose), STATUS.get("_hip"))
    if a.what in ("all", "rccl"):
        print(build_rccl(a.force, a.verbose), STATUS.get("_rccl"))
