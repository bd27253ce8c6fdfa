"""Shared helpers of the multi-process tests (importable: pytest puts tests/ on sys.path)."""
import os
import socket


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun_smoke(nproc, *args, timeout=180, script="comm_smoke.py"):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "tools", script), *args]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return sorted(_rank_records(r.stdout), key=lambda d: d["rank"])


def _rank_records(text):
    """Every ``{"rank": ...}`` JSON object in the ranks' merged stdout.  Ranks share torchrun's
    stdout pipe, so two records can land on one line (a rank's text and its newline are
    separate writes): decode objects wherever they start instead of line by line."""
    import json

    dec = json.JSONDecoder()
    out, i = [], text.find('{"rank"')
    while i >= 0:
        obj, end = dec.raw_decode(text, i)
        out.append(obj)
        i = text.find('{"rank"', end)
    return out



def run_isolated(target, timeout=240):
    """Runs ``"module:function"`` (a module under tests/) in a fresh Python process with
    ``faulthandler`` on for all threads.  Tests that put several GPU subtasks into one
    process use it: a native abort (SIGABRT / SIGSEGV) then fails that one test, with every
    thread's Python stack in the failure message, instead of killing the whole pytest run."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mod, fn = target.split(":")
    code = (f"import sys; sys.path[:0] = [{root!r}, {os.path.join(root, 'tests')!r}]\n"
            f"import {mod}\n{mod}.{fn}()\nprint('__ISOLATED_OK__', flush=True)\n")
    env = dict(os.environ, PYTHONFAULTHANDLER="1", PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", code], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=timeout, env=env, cwd=root)
    out = r.stdout or ""
    assert r.returncode == 0 and "__ISOLATED_OK__" in out, f"{target} exited with {r.returncode}:\n{out[-12000:]}"
    return out
