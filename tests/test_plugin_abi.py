"""B2 plugin library on the CPU (no GPU needed): libgrokj2k_plugin.so exports every entry point
Grok's loader resolves by name (grok.cpp:550-567, plugin_bridge.cpp:299-300, minpf
minpf_plugin_manager.cpp:140-175), registers through minpf_post_load_plugin with the checks of
minpf_register_object, reports the production debug state, and refuses plugin_init cleanly
when no MI355X is visible (the host then keeps its CPU path)."""
import ctypes
import os
import subprocess

import pytest

import grok_amd as G
from conftest import ROOT

PLUGIN = os.path.join(os.path.dirname(G.LIB_PATH), "libgrokj2k_plugin.so")
EXPORTS = ["minpf_post_load_plugin", "plugin_init", "plugin_get_debug_state", "plugin_encode",
           "plugin_batch_encode", "plugin_is_batch_complete", "plugin_stop_batch_encode", "plugin_decompress",
           "plugin_init_batch_decompress", "plugin_batch_decompress", "plugin_stop_batch_decompress",
           "plugin_debug_mqc_next_cxd", "plugin_debug_mqc_next_plane"]


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    d = tmp_path_factory.mktemp("plugin")
    exe = str(d / "plugin_host")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi", "plugin_host.cpp"), "-o", exe, "-ldl"])
    return exe, d


def test_plugin_exports():
    assert os.path.exists(PLUGIN), "build with python -m grok_amd.build"
    lib = ctypes.CDLL(PLUGIN, mode=os.RTLD_LOCAL)
    for name in EXPORTS:
        assert hasattr(lib, name), name
    lib.plugin_get_debug_state.restype = ctypes.c_uint32
    assert lib.plugin_get_debug_state() == 0            # GRK_PLUGIN_STATE_NO_DEBUG
    lib.plugin_is_batch_complete.restype = ctypes.c_bool
    assert lib.plugin_is_batch_complete()


def test_plugin_exports_no_grk_api():
    # a Grok host process already holds the grk_* symbols: the plugin must not export its own
    out = subprocess.run(["nm", "-D", "--defined-only", PLUGIN], capture_output=True, text=True).stdout
    names = {l.split()[-1] for l in out.splitlines() if l.strip()}
    assert not [n for n in names if n.startswith("grk_")]
    assert set(EXPORTS) <= names


def test_plugin_load_without_gpu(host):
    exe, d = host
    pnm = d / "x.pgm"
    pnm.write_bytes(b"P5\n4 4\n255\n" + bytes(range(16)))
    r = subprocess.run([exe, os.path.dirname(PLUGIN), "enc", str(pnm), str(d / "dump")], capture_output=True,
                       text=True, timeout=120)
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: covered by tests/test_gpu_plugin.py")
    # loaded, registered (minpf checks), debug state 0; plugin_init reports no device
    assert r.returncode == 6, (r.returncode, r.stdout, r.stderr)
    assert "plugin_init failed" in r.stderr
