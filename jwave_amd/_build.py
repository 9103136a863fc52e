"""In-tree build of libjwave_hip.so (gfx950) via jwave_amd/csrc/Makefile."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libjwave_hip.so")


def _sources():
    out = []
    for d in (CSRC, os.path.join(HERE, "..", "include")):
        for f in os.listdir(d):
            if f.endswith((".hip", ".cpp", ".hpp", ".h")) or f == "Makefile":
                out.append(os.path.join(d, f))
    return out


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in _sources())


def build(force=False, jobs=5):
    if force or stale():
        jobs = min(int(jobs), 16)
        subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", CSRC])
    return LIB
