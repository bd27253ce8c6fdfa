"""Host runtime under sanitizers: the C++ library is rebuilt with
AddressSanitizer+UBSan and with ThreadSanitizer into a temp dir and every entry point is
driven from several threads in a child process with the sanitizer runtime preloaded.
GPU sanitizers are not available on the pool (no xnack / GPU ASan): kernels are covered by
host-side shape validation and the numerics tests instead."""
import os
import subprocess
import sys

import pytest

from flink_tensorflow_amd import _build

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_native_library_under_sanitizer(kind, tmp_path):
    rt = _build.sanitizer_runtime(kind)
    if not os.path.exists(rt):
        pytest.skip(f"{kind} runtime not installed")
    lib = _build.build_native_sanitized(kind, tmp_path)
    # libstdc++ must be mapped at start-up too, or the runtime's __cxa_throw interceptor
    # finds no real symbol (python itself does not link libstdc++)
    stdcxx = subprocess.run(["g++", "-print-file-name=libstdc++.so.6"], stdout=subprocess.PIPE, text=True).stdout.strip()
    env = dict(os.environ, FTM_NATIVE_LIB=str(lib), LD_PRELOAD=f"{rt} {stdcxx}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "native", "exercise_native.py")], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0 and "native exercise ok" in r.stdout, r.stdout[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stdout and "runtime error:" not in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stdout, r.stdout[-4000:]
