"""Build libratelimit_hip.so in-tree for gfx950 (explicit hipcc; no cmake).

    python -m ratelimit_amd.build          # or __graft_entry__.build()
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libratelimit_hip.so")
# The same library with the history log's tear hook compiled into its lookups
# (RL_LOG_TEAR: rl_debug_log_tear, tests/test_gpu_log_tear.py); only
# rl_kernels.hip differs. The product library has no hook.
TEAR_LIB = os.path.join(HERE, "libratelimit_hip_tear.so")
SOURCES = ["rl_kernels.hip", "rl_route.hip", "rl_match.hip", "rl_engine.hip", "rl_transport.hip", "rl_comm.hip",
           "rl_api.hip",
           "rl_pack.cpp"]
HEADERS = ["rl_device.h", "rl_kernels.h", "rl_match.h", "rl_engine.h", "rl_comm.h", "rl_transport.h",
           os.path.join("..", "..", "include", "ratelimit_hip.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RL_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include")]


def _stale():
    if not os.path.exists(LIB) or not os.path.exists(TEAR_LIB):
        return True
    t = min(os.path.getmtime(LIB), os.path.getmtime(TEAR_LIB))
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, out=None, defines=()):
    """Compile and link; ``out``/``defines`` make side builds (e.g. RL_ABL ablations)."""
    lib = out or LIB
    if out is None and not force and not _stale():
        return LIB
    objs, procs = [], []
    tag = "" if out is None else "_%x" % (hash(lib) & 0xFFFFFF)

    def compile_(s, o, extra=()):
        cmd = [HIPCC] + FLAGS + ["-D" + d for d in tuple(defines) + tuple(extra)] + ["-c", os.path.join(CSRC, s),
                                                                                     "-o", o]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))

    for s in SOURCES:  # (compiled side by side: one hipcc per source)
        o = os.path.join(CSRC, os.path.splitext(s)[0] + tag + ".o")
        compile_(s, o)
        objs.append(o)
    tear_obj = None
    if out is None:
        tear_obj = os.path.join(CSRC, "rl_kernels_tear.o")
        compile_("rl_kernels.hip", tear_obj, ["RL_LOG_TEAR=1"])
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)

    def link(path, objects):  # (RCCL is dlopen'ed by rl_comm.hip (libdl), never linked)
        cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", path] + objects + ["-ldl"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)

    link(lib, objs)
    if tear_obj:
        link(TEAR_LIB, [tear_obj] + objs[1:])
        os.remove(tear_obj)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
