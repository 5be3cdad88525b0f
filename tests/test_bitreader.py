"""The T2 decoder's packet-header bit reader (grok_amd/csrc/gk_bitio.h: 64-bit register,
runs by leading-zero count, align() by walking loaded bytes back) against a bit-at-a-time
restatement of Grok's BitIO reader (BitIO.cpp bytein / getbit / inalign) on random
0xFF-dense streams, ends past the data and small source windows (tests/capi/bitreader_test.cpp)."""
import os
import subprocess

from conftest import ROOT


def test_packet_header_bit_reader(tmp_path):
    exe = str(tmp_path / "bitreader_test")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "grok_amd", "csrc"),
                           os.path.join(ROOT, "tests", "capi", "bitreader_test.cpp"), "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
