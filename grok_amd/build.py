"""Build the in-tree HIP extension libgrok_amd.so for gfx950 (hipcc, no JIT cache)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libgrok_amd.so")
# Grok's plugin loader opens <pluginPath>/libgrokj2k_plugin.so (grok.cpp:579-605)
PLUGIN = os.path.join(HERE, "libgrokj2k_plugin.so")
ENGINE = ["gk_kernels.hip", "gk_dwt97.hip", "gk_dwt_any.hip", "gk_t1enc.hip", "gk_t1dec.hip", "gk_t1ms.hip", "gk_ht.hip", "gk_engine.cpp"]
SOURCES = ENGINE + ["grk_shim.cpp", "grk_plugin.cpp"]


def needs_build():
    if not os.path.exists(LIB) or not os.path.exists(PLUGIN):
        return True
    t = min(os.path.getmtime(LIB), os.path.getmtime(PLUGIN))
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + \
        [os.path.join(HERE, "..", "include", f) for f in ("grok_amd.h", "grk_abi.h", "grk_plugin_abi.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    objs = {}
    cmds = []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(CSRC, s.rsplit(".", 1)[0] + ".o")
        cmds.append(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-c", src, "-o", obj])
        if verbose:
            print(" ".join(cmds[-1]), file=sys.stderr)
        objs[s] = obj
    # one compiler per source, at most 8 at a time (container: 8 CPUs; the box sets MAX_JOBS)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "8")), 8))
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(subprocess.check_call, c) for c in cmds]:
            f.result()
    engine = [objs[s] for s in ENGINE]
    # the grk_* drop-in, and the T1 plugin a Grok host loads (its own copy of the engine: a
    # host process already holds Grok's grk_* symbols)
    for lib, extra in ((LIB, "grk_shim.cpp"), (PLUGIN, "grk_plugin.cpp")):
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + engine + [objs[extra]]
        subprocess.check_call(cmd)
    for o in objs.values():
        os.remove(o)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
