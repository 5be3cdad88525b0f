"""The engine's host worker pool (gk_engine.cpp HostPool) under back-to-back dispatches: every
item runs exactly once per dispatch and a worker's error reaches the caller (CPU only: the
stress program, tools/pool_stress.cpp, compiles the engine source and makes no GPU call).

The pool claims items from one (generation, count, next item) word and sleeps workers on a
futex; an earlier version read the item count apart from the claim and hung under this test
when a worker woke a generation late.
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

LIB = os.path.join(ROOT, "grok_amd", "libgrok_amd.so")


@pytest.mark.skipif(shutil.which("hipcc") is None or not os.path.exists(LIB),
                    reason="needs hipcc and the built libgrok_amd.so")
def test_pool_items_run_once(tmp_path):
    exe = str(tmp_path / "pool_stress")
    src = os.path.join(ROOT, "tools", "pool_stress.cpp")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-x", "hip", src, "-o", exe,
                           "-x", "none", LIB, "-Wl,-rpath," + os.path.dirname(LIB)],
                          cwd=os.path.join(ROOT, "tools"))
    r = subprocess.run([exe, "20000"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "error propagated: yes" in r.stdout
